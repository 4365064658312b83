"""Vocos-style log-mel front end (reference `model/modules.py:80-151`).

The reference builds `torchaudio.transforms.MelSpectrogram(sample_rate=24000, n_fft=1024,
win_length=1024, hop_length=256, n_mels=100, power=1, center=True, normalized=False,
norm=None)` and returns `log(clamp(mel, 1e-5))`. torchaudio is not installed in this image,
so the transform is restated: periodic Hann window, reflect-padded centred STFT, magnitude
(power 1), HTK-scale triangular filterbank (torchaudio.functional.melscale_fbanks with
norm=None, mel_scale="htk", f_min=0, f_max=sr/2). Parity of this row is "unpinned": no
reference fixture exists in-tree and torchaudio cannot be imported here.

This runs before the sampling engine (cfm.py:106-108) and is host/torch code, not part of
the HIP hot path.
"""

from __future__ import annotations

import math

import torch
from torch import nn


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> torch.Tensor:
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + f_min / 700.0)
    m_max = 2595.0 * math.log10(1.0 + f_max / 700.0)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))  # [n_freqs, n_mels]


class MelSpec(nn.Module):
    def __init__(self, n_fft=1024, hop_length=256, win_length=1024, n_mel_channels=100, target_sample_rate=24_000,
                 mel_spec_type="vocos"):
        super().__init__()
        if mel_spec_type != "vocos":
            raise NotImplementedError("only the vocos mel front end is restated (bigvgan's vocoder is not shipped)")
        self.n_fft, self.hop_length, self.win_length = n_fft, hop_length, win_length
        self.n_mel_channels, self.target_sample_rate = n_mel_channels, target_sample_rate
        self.register_buffer("window", torch.hann_window(win_length), persistent=False)
        self.register_buffer("fb", melscale_fbanks(n_fft // 2 + 1, 0.0, float(target_sample_rate // 2),
                                                   n_mel_channels, target_sample_rate), persistent=False)

    def forward(self, wav: torch.Tensor) -> torch.Tensor:
        if wav.ndim == 3:
            wav = wav.squeeze(1)
        assert wav.ndim == 2
        win = self.window.to(wav.device, wav.dtype)
        spec = torch.stft(wav, self.n_fft, hop_length=self.hop_length, win_length=self.win_length, window=win,
                          center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
        spec = spec.abs()  # power = 1
        mel = torch.matmul(spec.transpose(-1, -2), self.fb.to(spec.device, spec.dtype)).transpose(-1, -2)
        return mel.clamp(min=1e-5).log()  # [b, n_mels, frames]
