"""LayerNorm-fold diagnostic: the fold on vs off (16-bit) and each against the fp32 engine, for a few DiT widths."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import configs, synthetic  # noqa: E402
from test_gpu_contract import _model, DEV  # noqa: E402

for name, over, total in (("F5TTS_v1_Small_4L", {}, 564), ("F5TTS_v1_Small_4L", {"depth": 1}, 300),
                          ("F5TTS_v1_Base", {"depth": 2}, 564), ("DiT_tiny", {"text_num_embeds": 64}, 200)):
    arch = configs.get_arch(name, **over)
    inp = synthetic.make_case(B=1, ref_frames=[total // 2], total_frames=[total], n_text=[40],
                              vocab=min(64, arch["text_num_embeds"]) if name == "DiT_tiny" else 2545)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, 1)
    kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
              steps=4, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)
    ref = _model(arch, "fp32").sample(**kw)[0].float().cpu()
    m = _model(arch, "bf16")
    eng = m.transformer.get_engine("bf16", m.device)
    res = {}
    for fold in (0, 1):
        eng.set_ln_fold(bool(fold))
        res[fold] = m.sample(**kw)[0].float().cpu()
    sup, n = eng.ln_fold_stats()
    r = lambda a: float((a - ref).norm() / ref.norm())
    print(f"{name} {over} d={arch['dim']}: fold supported {sup}, folded passes {n}; rel-L2 vs fp32: off {r(res[0]):.4e} "
          f"on {r(res[1]):.4e}; on vs off {float((res[1] - res[0]).norm() / res[0].norm()):.4e}", flush=True)
