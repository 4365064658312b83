"""Deterministic stand-ins for `model_obj` and `vocoder` used to pin the host orchestration of
`infer_process` / `infer_batch_process` against the reference's own (tests/golden/make_golden_infer.py):
every input the reference hands them (cond wave, text list, duration, steps, CFG, sway) leaves a
trace in their outputs, and they record the calls."""

from __future__ import annotations

import threading

import torch


class FakeModel:
    device = torch.device("cpu")

    def __init__(self):
        self.calls = []
        self._lock = threading.Lock()

    def sample(self, cond, text, duration, steps, cfg_strength, sway_sampling_coef):
        with self._lock:
            self.calls.append(("".join(text[0]), int(duration), int(steps), float(cfg_strength),
                               float(sway_sampling_coef)))
        n = torch.arange(duration, dtype=torch.float64)[:, None]
        c = torch.arange(100, dtype=torch.float64)[None, :]
        sig = float(cond.double().abs().mean()) + 1e-3 * len(text[0]) + 1e-4 * steps
        out = torch.sin(0.013 * n * (c + 1) + sig) * (1 + 0.1 * cfg_strength) + sway_sampling_coef * 0.01
        return out[None].float(), None


class FakeVocoder:
    def decode(self, mel):
        # mel [1, 100, T] -> wave [1, T * 256]
        m = mel.double().mean(1, keepdim=True)  # [1, 1, T]
        w = m.repeat_interleave(256, dim=-1)[:, 0]
        ph = torch.arange(w.shape[-1], dtype=torch.float64)
        return (0.3 * torch.tanh(w) + 0.05 * torch.sin(0.02 * ph)).float()


def ref_audios(amps):
    """The reference waves of the golden cases: seeded CPU normal noise, mono/stereo alternating."""
    g = torch.Generator().manual_seed(5)
    return [(torch.randn(1 if i % 2 == 0 else 2, 24000 + 6000 * i, generator=g) * amp).float()
            for i, amp in enumerate(amps)]
