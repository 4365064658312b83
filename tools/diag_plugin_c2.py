"""Diagnostic (round 6): the C2 plugin Euler loop vs f5h_sample, each with the phase chain on and off, repeated,
to find which path moved (tests/test_gpu_contract.py::test_plugin_euler_loop_c2_time_close_to_engine_sample).
Run with F5H_LIB=<lib> to compare builds."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import configs, synthetic  # noqa: E402
from test_gpu_contract import _model, _plugin_euler, DEV  # noqa: E402

arch = configs.get_arch("F5TTS_v1_Base")
m = _model(arch, "bf16")
if os.environ.get("DIAG_BF16_PARAMS", "1") == "1":
    m.transformer.to(torch.bfloat16)
inp = synthetic.make_case(**gc.C2)
dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
y0 = synthetic.reference_noise(dur, gc.SEED)
kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
          steps=16, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)
eng = m.transformer.get_engine("bf16", m.device)
outs = {}
for chain in (True, False):
    eng.set_chain(chain)
    for rep in range(2):
        outs[f"sample_chain{int(chain)}_{rep}"] = m.sample(**kw)[0].float().cpu()
        outs[f"plugin_chain{int(chain)}_{rep}"] = _plugin_euler(m.transformer, inp, inp["duration"], 16, 2.0, -1.0,
                                                               y0)[0].float().cpu()
        torch.cuda.synchronize()
eng.set_chain(True)
ref = outs["sample_chain0_0"]
for k, v in outs.items():
    print(f"{k:20s} rel vs sample_chain0_0 {gc.rel_err(v.numpy(), ref.numpy()):.3e}  equal {torch.equal(v, ref)}  "
          f"finite {bool(torch.isfinite(v).all())}", flush=True)
