"""Determinism stress of the C2 sample (round 6): repeated f5h_sample calls on one input must be bitwise equal,
with the phase chain on and off, with plugin Euler loops (another workspace, its own graphs) interleaved as in
tests/test_gpu_contract.py::test_plugin_euler_loop_c2_time_close_to_engine_sample. Prints every mismatch."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import configs, synthetic  # noqa: E402
from test_gpu_contract import _model, _plugin_euler, DEV  # noqa: E402

N = int(os.environ.get("STRESS_N", "12"))
arch = configs.get_arch("F5TTS_v1_Base")
m = _model(arch, "bf16")
if os.environ.get("STRESS_BF16_PARAMS", "1") == "1":
    m.transformer.to(torch.bfloat16)
inp = synthetic.make_case(**gc.C2)
dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
y0 = synthetic.reference_noise(dur, gc.SEED)
kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
          steps=16, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=True)
eng = m.transformer.get_engine("bf16", m.device)
for chain in (True, False):
    eng.set_chain(chain)
    ref, ref_tr = None, None
    bad = 0
    for i in range(N):
        out, tr = m.sample(**kw)
        if i % 3 == 2:
            _plugin_euler(m.transformer, inp, inp["duration"], 16, 2.0, -1.0, y0)
        torch.cuda.synchronize()
        out, tr = out.float().cpu(), tr.float().cpu()
        if ref is None:
            ref, ref_tr = out, tr
            continue
        if not torch.equal(out, ref):
            bad += 1
            steps = [k for k in range(tr.shape[0]) if not torch.equal(tr[k], ref_tr[k])]
            print(f"chain={chain} call {i}: MISMATCH rel {gc.rel_err(out.numpy(), ref.numpy()):.3e}, first differing "
                  f"trajectory point {steps[0] if steps else None} of {tr.shape[0]}", flush=True)
    n_chain = eng.chain_stats()[:2] if hasattr(eng, "chain_stats") else None
    print(f"chain={chain}: {bad} of {N - 1} repeated calls differ from the first; chain stats {n_chain}", flush=True)
eng.set_chain(True)
