"""Golden vectors for the STFT magnitude of the mel front end, produced by the REFERENCE's own
conv STFT (runtime/triton_trtllm/scripts/conv_stft.py:15-194: reflect padding, librosa-style
"continue" framing, periodic Hann window as scipy get_window('hann'), rfft basis).

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden_mel.py
Stores seeded waveforms and conv_stft's magnitudes (transform(..., "magphase")[0]).
"""

from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/src/f5_tts/runtime/triton_trtllm/scripts/conv_stft.py"


def main():
    spec = importlib.util.spec_from_file_location("ref_conv_stft", SRC)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    stft = mod.STFT(win_len=1024, win_hop=256, fft_len=1024)
    g = torch.Generator().manual_seed(7)
    out = {}
    for name, L in {"l6000": 6000, "l1300": 1300}.items():
        t = torch.arange(L) / 24000.0
        wav = (0.3 * torch.sin(2 * torch.pi * 220.0 * t) + 0.05 * torch.randn(L, generator=g))[None]
        with torch.no_grad():
            mag, _ = stft.transform(wav, return_type="magphase")
        out[f"{name}_wav"] = wav.numpy().astype(np.float32)
        out[f"{name}_mag"] = mag.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "mel_stft.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
