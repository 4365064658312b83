"""Run seeded samples with the library F5H_LIB points at and save the outputs, so two builds can be compared
bit for bit:  F5H_LIB=... python tools/diag_lib_bitwise.py OUT.npy [tiny|base]

tiny: one bf16 sample of the tiny DiT, 2 utterances of 300/237 frames (several full K/V tiles, a ragged last
      tile, the batch mask).
base: F5TTS_v1_Base (every fused GEMM epilogue at its real width: QKV + RoPE, GELU-tanh, gated residual; the
      conv position embedding; attention) in bf16 and fp16, B=2 mixed 600/437 frames (batch mask, pad skip),
      and E2 UNetT Base bf16 B=1, NFE 2 each.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import configs, synthetic  # noqa: E402
from f5_tts_amd.model import CFM, DiT, UNetT  # noqa: E402

DEV = "cuda:0"


def model(arch, compute):
    cls = DiT if arch["backbone"] == "DiT" else UNetT
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = cls(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute=compute).to(DEV)


def sample(m, inp, y0, steps):
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
                      steps=steps, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)
    return out.float().cpu().numpy().ravel()


def main(path, mode="tiny"):
    outs = []
    if mode == "tiny":
        m = model(gc.arch_of("tiny"), "bf16")
        for n in (300, 237):
            inp = synthetic.make_case(B=1, ref_frames=n // 3, total_frames=n, n_text=20, vocab=64, seed=7 + n)
            outs.append(sample(m, inp, synthetic.reference_noise(inp["duration"], n), 8))
    else:
        inp = synthetic.make_case(B=2, ref_frames=[200, 150], total_frames=[600, 437], n_text=[90, 60])
        y0 = synthetic.reference_noise(inp["duration"], 5)
        for compute in ("bf16", "fp16"):
            outs.append(sample(model(configs.get_arch("F5TTS_v1_Base"), compute), inp, y0, 2))
        inp = synthetic.make_case(B=1, ref_frames=150, total_frames=480, n_text=70)
        outs.append(sample(model(configs.get_arch("E2TTS_Base"), "bf16"), inp,
                           synthetic.reference_noise(inp["duration"], 6), 2))
    np.save(path, np.concatenate(outs))
    print("saved", path, flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "tiny")
