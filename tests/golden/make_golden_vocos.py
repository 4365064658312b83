"""Golden vectors for the Vocos inverse STFT, produced by the REFERENCE's own restatement of it.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden_vocos.py

The reference restates vocos' ISTFTHead for its TensorRT export with its own conv-based STFT
(src/f5_tts/runtime/triton_trtllm/scripts/conv_stft.py:15-234, used by
scripts/export_vocoder_to_onnx.py:45-60 with fft_len = win_len = 1024, hop 256). This script loads
that file as a module, feeds it seeded random spectra (real, imag; two lengths) and stores the
inputs and its output. conv_stft returns T*hop samples; vocos (torch.istft center=True) returns
the first (T-1)*hop of them, which is what tests/test_vocos.py compares. Only data is stored.
"""

from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True  # /root/reference is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/src/f5_tts/runtime/triton_trtllm/scripts/conv_stft.py"


def main():
    spec = importlib.util.spec_from_file_location("ref_conv_stft", SRC)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    stft = mod.STFT(win_len=1024, win_hop=256, fft_len=1024)  # as export_vocoder_to_onnx.py:49
    out = {}
    g = torch.Generator().manual_seed(20261016)
    for name, (B, T) in {"t24": (2, 24), "t5": (1, 5)}.items():
        mag = torch.exp(torch.randn(B, 513, T, generator=g) * 1.5).clip(max=1e2)  # head-like magnitudes
        ph = (torch.rand(B, 513, T, generator=g) * 2 - 1) * 6.0
        real, imag = mag * torch.cos(ph), mag * torch.sin(ph)
        with torch.no_grad():  # one utterance per call: conv_stft.py:231-232 divides by the window
            # envelope only at batch index 0 (its `coff` has batch 1), so batches are fed singly
            y = torch.cat([stft.inverse(input1=real[b:b + 1], input2=imag[b:b + 1], input_type="realimag")
                           for b in range(B)])
        out[f"{name}_real"] = real.numpy().astype(np.float32)
        out[f"{name}_imag"] = imag.numpy().astype(np.float32)
        out[f"{name}_audio"] = y.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "vocos_istft.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
