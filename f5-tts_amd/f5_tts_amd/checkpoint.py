"""Checkpoint formats -> engine: the reference's `load_checkpoint` / `load_model`
(src/f5_tts/infer/utils_infer.py:188-275) on this package's CFM/DiT/UNetT.

Same rules as the reference:
  * dtype default: fp16 when the device is a GPU of compute capability >= 7 (every ROCm device here),
    else fp32 (utils_infer.py:189-196). On this engine fp16 parameters select the fp16 MFMA mode
    (CFM.engine_compute "auto": the reference's own GPU arithmetic), bf16 parameters the bf16 mode
    and fp32 parameters the exact-fp32 parity mode.
  * `.safetensors` via safetensors (no code execution), anything else via
    torch.load(weights_only=True) (utils_infer.py:198-204).
  * use_ema: the EMA state ("ema_model_state_dict", or the whole safetensors file) with the
    "ema_model." prefix stripped and the "initted" / "step" bookkeeping keys dropped
    (utils_infer.py:206-213); legacy mel buffers removed (the 305e3ea patch, :215-218).
  * otherwise "model_state_dict" (or the whole safetensors file), :221-224.
The packed HIP engine is built lazily from the loaded parameters on the first sample() call.
"""

from __future__ import annotations

import torch

from .model import CFM
from .model.utils import get_tokenizer

_LEGACY_MEL_KEYS = ("mel_spec.mel_stft.mel_scale.fb", "mel_spec.mel_stft.spectrogram.window")


def _default_dtype(device: str) -> torch.dtype:
    if "cuda" in str(device) and torch.cuda.is_available() and torch.cuda.get_device_properties(device).major >= 7:
        return torch.float16
    return torch.float32


def read_state_dict(ckpt_path: str, use_ema: bool = True, map_location="cpu") -> dict:
    """The model state dict a reference checkpoint holds (EMA or raw), reference key names."""
    ckpt_type = ckpt_path.split(".")[-1]
    if ckpt_type == "safetensors":
        from safetensors.torch import load_file

        checkpoint = load_file(ckpt_path, device=str(map_location))
    else:
        checkpoint = torch.load(ckpt_path, map_location=map_location, weights_only=True)
    if use_ema:
        if ckpt_type == "safetensors":
            checkpoint = {"ema_model_state_dict": checkpoint}
        sd = {k.replace("ema_model.", ""): v for k, v in checkpoint["ema_model_state_dict"].items()
              if k not in ("initted", "step")}
        for key in _LEGACY_MEL_KEYS:
            sd.pop(key, None)
        return sd
    if ckpt_type == "safetensors":
        checkpoint = {"model_state_dict": checkpoint}
    return checkpoint["model_state_dict"]


def load_checkpoint(model: CFM, ckpt_path: str, device: str, dtype: torch.dtype | None = None, use_ema: bool = True):
    """utils_infer.py:188-232 on the engine-backed CFM."""
    if dtype is None:
        dtype = _default_dtype(device)
    model = model.to(dtype)
    sd = read_state_dict(ckpt_path, use_ema=use_ema, map_location="cpu")
    model.load_state_dict(sd)
    return model.to(device)


def load_model(model_cls, model_cfg: dict, ckpt_path: str, mel_spec_type: str = "vocos", vocab_file: str = "",
               ode_method: str = "euler", use_ema: bool = True, device: str = "cuda:0", n_mel_channels: int = 100,
               n_fft: int = 1024, hop_length: int = 256, win_length: int = 1024, target_sample_rate: int = 24000):
    """utils_infer.py:238-275: tokenizer ("custom" vocab file), CFM around `model_cls(**model_cfg)`,
    checkpoint load. `vocab_file` is required (the reference's default points into its own package)."""
    if not vocab_file:
        raise ValueError("vocab_file is required (path to the vocab.txt the checkpoint was trained with)")
    vocab_char_map, vocab_size = get_tokenizer(vocab_file)
    model = CFM(
        transformer=model_cls(**model_cfg, text_num_embeds=vocab_size, mel_dim=n_mel_channels),
        mel_spec_kwargs=dict(n_fft=n_fft, hop_length=hop_length, win_length=win_length,
                             n_mel_channels=n_mel_channels, target_sample_rate=target_sample_rate,
                             mel_spec_type=mel_spec_type),
        odeint_kwargs=dict(method=ode_method),
        vocab_char_map=vocab_char_map,
    )
    dtype = torch.float32 if mel_spec_type == "bigvgan" else None
    return load_checkpoint(model, ckpt_path, device, dtype=dtype, use_ema=use_ema)
