"""Round-6 chain race isolation: repeated C2 sample calls (chain on) under different interleavings, each variant on
a fresh model, every output compared bitwise with the chain-off output of the same model."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import configs, synthetic  # noqa: E402
from test_gpu_contract import _model, _plugin_euler, DEV  # noqa: E402

arch = configs.get_arch("F5TTS_v1_Base")
inp = synthetic.make_case(**gc.C2)
dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
y0 = synthetic.reference_noise(dur, gc.SEED)
kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
          steps=16, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)
X = torch.randn(8192, 8192, device=DEV, dtype=torch.bfloat16)


def variant(name, inter, graph=True, n=10):
    m = _model(arch, "bf16")
    eng = m.transformer.get_engine("bf16", m.device)
    eng.set_graph_mode(graph)
    eng.set_chain(False)
    ref = m.sample(**kw)[0].float().cpu()
    eng.set_chain(True)
    bad = []
    for i in range(n):
        out = m.sample(**kw)[0]
        if inter == "plugin" and i % 3 == 2:
            _plugin_euler(m.transformer, inp, inp["duration"], 16, 2.0, -1.0, y0)
        elif inter == "matmul" and i % 3 == 2:
            for _ in range(20):
                X @ X
        elif inter == "sync" :
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        out = out.float().cpu()
        if not torch.equal(out, ref):
            bad.append((i, round(gc.rel_err(out.numpy(), ref.numpy()), 4)))
    print(f"{name}: {len(bad)} of {n} chained calls differ from the unchained output: {bad}", flush=True)
    del m, eng


tag = os.environ.get("STRESS_TAG", "")
if os.environ.get("STRESS_SHORT") == "1":
    variant(f"back-to-back graph {tag}", None, n=4)
else:
    variant("plugin-interleaved graph", "plugin")
    variant("matmul-interleaved graph", "matmul")
    variant("back-to-back graph", None)
    variant("synced graph", "sync")
    variant("plugin-interleaved eager", "plugin", graph=False)
    variant("back-to-back eager", None, graph=False)
