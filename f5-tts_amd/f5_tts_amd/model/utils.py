"""Host-side helpers of the sampling path (restated from model/utils.py of the reference).

lens_to_mask ........ utils.py:53-58
list_str_to_tensor .. utils.py:88-96 (utf-8 bytes, pad -1)
list_str_to_idx ..... utils.py:99-106 (vocab map, unknown -> 0, pad -1)
get_epss_timesteps .. utils.py:205-218
sway ................ cfm.py:215-216
"""

from __future__ import annotations

import torch
from torch.nn.utils.rnn import pad_sequence

_EPSS = {
    5: (0, 2, 4, 8, 16, 32),
    6: (0, 2, 4, 6, 8, 16, 32),
    7: (0, 2, 4, 6, 8, 16, 24, 32),
    10: (0, 2, 4, 6, 8, 12, 16, 20, 24, 28, 32),
    12: (0, 2, 4, 6, 8, 10, 12, 14, 16, 20, 24, 28, 32),
    16: (0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32),
}


def exists(v):
    return v is not None


def default(v, d):
    return v if v is not None else d


def lens_to_mask(t: torch.Tensor, length: int | None = None) -> torch.Tensor:
    if length is None:
        length = t.amax()
    return torch.arange(length, device=t.device)[None, :] < t[:, None]


def list_str_to_tensor(text, padding_value=-1) -> torch.Tensor:
    seqs = [torch.tensor([*bytes(t, "UTF-8")]) for t in text]
    return pad_sequence(seqs, padding_value=padding_value, batch_first=True)


def list_str_to_idx(text, vocab_char_map: dict, padding_value=-1) -> torch.Tensor:
    seqs = [torch.tensor([vocab_char_map.get(c, 0) for c in t]) for t in text]
    return pad_sequence(seqs, padding_value=padding_value, batch_first=True)


def get_epss_timesteps(n: int, device, dtype) -> torch.Tensor:
    """Empirically pruned step schedule (x 1/32) for the tabulated NFEs, else uniform."""
    if n not in _EPSS:
        return torch.linspace(0, 1, n + 1, device=device, dtype=dtype)
    return (1 / 32) * torch.tensor(_EPSS[n], device=device, dtype=dtype)


def time_grid(steps: int, sway_sampling_coef, use_epss: bool, device, dtype, t_start: float = 0.0) -> torch.Tensor:
    """The ODE grid exactly as CFM.sample builds it (cfm.py:211-216), in `dtype` on `device`."""
    if t_start == 0 and use_epss:
        t = get_epss_timesteps(steps, device=device, dtype=dtype)
    else:
        t = torch.linspace(t_start, 1, steps + 1, device=device, dtype=dtype)
    if sway_sampling_coef is not None:
        t = t + sway_sampling_coef * (torch.cos(torch.pi / 2 * t) - 1 + t)
    return t


def get_tokenizer(vocab_path: str):
    """vocab.txt (one token per line) -> ({token: idx}, size) like tokenizer='custom' (utils.py:112-142)."""
    with open(vocab_path, "r", encoding="utf-8") as f:
        vocab = {}
        for i, ch in enumerate(f):
            vocab[ch[:-1]] = i
    return vocab, len(vocab)
