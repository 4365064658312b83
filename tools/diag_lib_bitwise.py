"""Run one seeded bf16 sample (tiny DiT, 2 utterances of 300/237 frames: several full K/V tiles, a
ragged last tile, the batch mask) with the library F5H_LIB points at and save the output, so two
builds can be compared bit for bit: python tools/diag_lib_bitwise.py OUT.npy."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import numpy as np
import torch
import golden_cases as gc
from f5_tts_amd import synthetic
from f5_tts_amd.model import CFM, DiT

DEV = "cuda:0"
arch = gc.arch_of("tiny")
kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
m = CFM(transformer=net, num_channels=100, compute="bf16").to(DEV)
outs = []
for n in (300, 237):
    inp = synthetic.make_case(B=1, ref_frames=n // 3, total_frames=n, n_text=20, vocab=64, seed=7 + n)
    y0 = synthetic.reference_noise(inp["duration"], n)
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
                      steps=8, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)
    outs.append(out.float().cpu().numpy().ravel())
np.save(sys.argv[1], np.concatenate(outs))
print("saved", sys.argv[1], flush=True)
