"""ORACLE — test infrastructure only. CPU restatement of the Vocos decoder (mel -> waveform).

Checker for the HIP Vocos path (libf5h.so f5h_vocos_*); never part of the product path. Only
`tests/` and `bench.py`'s `cpu_baseline` leg import it.

What it restates (fp32, PyTorch-CPU):
  The reference calls `vocoder.decode(mel)` (src/f5_tts/infer/utils_infer.py:506-511;
  runtime/triton_trtllm/benchmark.py:432-435) on vocos' "charactr/vocos-mel-24khz" model, built by
  `Vocos.from_hparams` (utils_infer.py:118). vocos is a third-party package (pyproject.toml:42,
  unpinned; its published 0.1.0 release) that is absent here, so its algorithm is restated:
    VocosBackbone(input_channels=100, dim=512, intermediate_dim=1536, num_layers=8):
      embed Conv1d(100, 512, k=7, pad=3) -> LayerNorm(512, eps=1e-6)
      -> 8 x ConvNeXtBlock: dwconv Conv1d(k=7, pad=3, groups=512) -> LayerNorm(eps=1e-6)
         -> Linear(512, 1536) -> GELU (erf) -> Linear(1536, 512) -> gamma * . -> + residual
      -> final LayerNorm(512, eps=1e-6)
    ISTFTHead(dim=512, n_fft=1024, hop_length=256, padding="center"):
      Linear(512, 1026) -> (mag, phase) = chunk(2, channel) -> mag = clip(exp(mag), max=100)
      -> S = mag * (cos p + i sin p) -> torch.istft(S, 1024, 256, 1024, hann_window(1024), center=True)
  The head's arithmetic is also restated inside the reference itself
  (runtime/triton_trtllm/scripts/export_vocoder_to_onnx.py:45-60) with its own inverse STFT
  (runtime/triton_trtllm/scripts/conv_stft.py:201-234); tests/golden/make_golden_vocos.py runs
  that inverse STFT to pin `istft` below (the first (T-1)*hop samples, torch.istft's length).
  The backbone's ConvNeXt arithmetic has no in-tree copy: parity unpinned for it beyond this
  restatement of the published package.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

VOCOS_MEL_24KHZ = dict(input_channels=100, dim=512, intermediate_dim=1536, num_layers=8, n_fft=1024, hop_length=256)


def param_shapes(arch: dict = VOCOS_MEL_24KHZ) -> "dict[str, tuple]":
    """State-dict names and shapes of vocos' Vocos (backbone + head; the feature extractor has no
    parameters on the decode path)."""
    C, d, I, nf = arch["input_channels"], arch["dim"], arch["intermediate_dim"], arch["n_fft"]
    s = {"backbone.embed.weight": (d, C, 7), "backbone.embed.bias": (d,),
         "backbone.norm.weight": (d,), "backbone.norm.bias": (d,)}
    for i in range(arch["num_layers"]):
        p = f"backbone.convnext.{i}."
        s.update({p + "dwconv.weight": (d, 1, 7), p + "dwconv.bias": (d,), p + "norm.weight": (d,),
                  p + "norm.bias": (d,), p + "pwconv1.weight": (I, d), p + "pwconv1.bias": (I,),
                  p + "pwconv2.weight": (d, I), p + "pwconv2.bias": (d,), p + "gamma": (d,)})
    s.update({"backbone.final_layer_norm.weight": (d,), "backbone.final_layer_norm.bias": (d,),
              "head.out.weight": (nf + 2, d), "head.out.bias": (nf + 2,)})
    return s


def backbone(W: dict, arch: dict, mel: torch.Tensor) -> torch.Tensor:
    """VocosBackbone.forward: mel [B, C, T] -> [B, T, dim]."""
    d = arch["dim"]
    x = F.conv1d(mel, W["backbone.embed.weight"], W["backbone.embed.bias"], padding=3)
    x = F.layer_norm(x.transpose(1, 2), (d,), W["backbone.norm.weight"], W["backbone.norm.bias"], 1e-6)
    x = x.transpose(1, 2)
    for i in range(arch["num_layers"]):
        p = f"backbone.convnext.{i}."
        r = x
        y = F.conv1d(x, W[p + "dwconv.weight"], W[p + "dwconv.bias"], padding=3, groups=d)
        y = F.layer_norm(y.transpose(1, 2), (d,), W[p + "norm.weight"], W[p + "norm.bias"], 1e-6)
        y = F.gelu(F.linear(y, W[p + "pwconv1.weight"], W[p + "pwconv1.bias"]))
        y = F.linear(y, W[p + "pwconv2.weight"], W[p + "pwconv2.bias"])
        y = W[p + "gamma"] * y
        x = r + y.transpose(1, 2)
    return F.layer_norm(x.transpose(1, 2), (d,), W["backbone.final_layer_norm.weight"],
                        W["backbone.final_layer_norm.bias"], 1e-6)


def istft(real: torch.Tensor, imag: torch.Tensor, n_fft: int = 1024, hop: int = 256) -> torch.Tensor:
    """vocos ISTFT(padding="center") = torch.istft(center=True), periodic Hann window."""
    S = torch.complex(real, imag)
    return torch.istft(S, n_fft, hop, n_fft, torch.hann_window(n_fft), center=True)


def head(W: dict, arch: dict, x: torch.Tensor) -> torch.Tensor:
    """ISTFTHead.forward: [B, T, dim] -> audio [B, (T-1)*hop]."""
    y = F.linear(x, W["head.out.weight"], W["head.out.bias"]).transpose(1, 2)
    mag, p = y.chunk(2, dim=1)
    mag = torch.clip(torch.exp(mag), max=1e2)
    return istft(mag * torch.cos(p), mag * torch.sin(p), arch["n_fft"], arch["hop_length"])


def decode(W: dict, arch: dict, mel: torch.Tensor) -> torch.Tensor:
    """Vocos.decode: mel [B, C, T] fp32 -> audio [B, (T-1)*hop]."""
    with torch.no_grad():
        return head(W, arch, backbone(W, arch, mel.float()))
