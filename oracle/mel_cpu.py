"""ORACLE — test infrastructure only. CPU restatement of the vocos log-mel front end.

Checker for the HIP front end (libf5h.so f5h_mel_*), never part of the product path.

Reference: get_vocos_mel_spectrogram (src/f5_tts/model/modules.py:80-109):
torchaudio.transforms.MelSpectrogram(sample_rate=24000, n_fft=1024, win_length=1024,
hop_length=256, n_mels=100, power=1, center=True, normalized=False, norm=None) then
clamp(min=1e-5).log(). torchaudio is absent from this image, so the transform is restated from
its published algorithm: torch.stft (periodic Hann window, center, reflect pad, onesided) ->
|X| (power 1) -> matmul with torchaudio.functional.melscale_fbanks(n_freqs=513, f_min=0,
f_max=sr//2, n_mels, sr, norm=None, mel_scale="htk").
Pinning: the STFT magnitude is checked against the reference's own conv STFT
(runtime/triton_trtllm/scripts/conv_stft.py:151-194, `transform(..., "magphase")`) by
tests/golden/make_golden_mel.py; the HTK filterbank has no in-tree copy (parity unpinned beyond
this restatement of torchaudio's published formula).
"""

from __future__ import annotations

import math

import torch


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


def stft_mag(wav: torch.Tensor, n_fft: int = 1024, hop: int = 256) -> torch.Tensor:
    """|STFT| [B, n_fft/2+1, T] (torchaudio Spectrogram, power 1)."""
    spec = torch.stft(wav, n_fft, hop_length=hop, win_length=n_fft, window=torch.hann_window(n_fft), center=True,
                      pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    return spec.abs()


def log_mel(wav: torch.Tensor, n_fft: int = 1024, hop: int = 256, n_mels: int = 100, sr: int = 24000) -> torch.Tensor:
    """wav [B, L] -> log-mel [B, n_mels, 1 + L // hop]."""
    if wav.ndim == 3:
        wav = wav.squeeze(1)
    mag = stft_mag(wav.float(), n_fft, hop)
    fb = melscale_fbanks(n_fft // 2 + 1, 0.0, float(sr // 2), n_mels, sr)
    mel = torch.matmul(mag.transpose(-1, -2), fb).transpose(-1, -2)
    return mel.clamp(min=1e-5).log()
