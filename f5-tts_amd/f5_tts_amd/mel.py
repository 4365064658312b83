"""Vocos log-mel front end on the HIP engine (reference `model/modules.py:80-151`).

`MelSpec` keeps the reference module's constructor and call surface (wav [B, L] or [B, 1, L] ->
log-mel [B, n_mels, 1 + L // hop]) and runs `f5h_mel_forward` (include/f5h.h): reflect-padded
frames, DFT and HTK filterbank as fp32 MFMA GEMMs, magnitude and clamp/log kernels. CFM.sample
calls it on raw-audio conditioning (cfm.py:106-108). There is no PyTorch fallback; the CPU
restatement used to check it lives in oracle/mel_cpu.py.
"""

from __future__ import annotations

import ctypes
import threading

import torch
from torch import nn

from . import _lib


class MelSpec(nn.Module):
    def __init__(self, n_fft=1024, hop_length=256, win_length=1024, n_mel_channels=100, target_sample_rate=24_000,
                 mel_spec_type="vocos"):
        super().__init__()
        if mel_spec_type != "vocos":
            raise NotImplementedError("only the vocos mel front end is provided (bigvgan's vocoder is not shipped)")
        if win_length != n_fft:
            raise NotImplementedError("win_length must equal n_fft (the vocos front end)")
        self.n_fft, self.hop_length, self.win_length = n_fft, hop_length, win_length
        self.n_mel_channels, self.target_sample_rate = n_mel_channels, target_sample_rate
        self._h = {}
        self._lock = threading.Lock()

    def _engine(self, device: torch.device):
        h = self._h.get(device.index)
        if h is None:
            a = _lib.MelArch(self.n_fft, self.hop_length, self.n_mel_channels, self.target_sample_rate)
            h = ctypes.c_void_p()
            with torch.cuda.device(device):
                _lib.check(_lib.lib().f5h_mel_create(ctypes.byref(a), device.index, ctypes.byref(h)), "f5h_mel_create")
            self._h[device.index] = h
        return h

    def forward(self, wav: torch.Tensor) -> torch.Tensor:
        if wav.ndim == 3:
            wav = wav.squeeze(1)
        assert wav.ndim == 2
        if wav.device.type != "cuda":
            raise RuntimeError("MelSpec runs on the HIP engine: move the waveform to a GPU device")
        dev = torch.device("cuda", wav.device.index if wav.device.index is not None else torch.cuda.current_device())
        B, L = wav.shape
        wav = wav.to(torch.float32).contiguous()
        T = 1 + L // self.hop_length
        out = torch.empty(B, self.n_mel_channels, T, dtype=torch.float32, device=dev)
        with self._lock:
            h = self._engine(dev)
            L_ = _lib.lib()
            ws = torch.empty(max(int(L_.f5h_mel_workspace_size(h, B, L)), 256), dtype=torch.uint8, device=dev)
            with torch.cuda.device(dev):
                _lib.check(L_.f5h_mel_forward(h, _lib.stream_handle(dev), B, L, wav.data_ptr(), out.data_ptr(),
                                              ws.data_ptr(), ws.numel()), "f5h_mel_forward")
        return out

    def __del__(self):
        for h in getattr(self, "_h", {}).values():
            try:
                _lib.lib().f5h_mel_destroy(h)
            except Exception:
                pass
