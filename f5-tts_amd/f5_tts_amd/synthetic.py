"""Deterministic synthetic weights and inputs (SURVEY §8c golden-vector plan, §8d inputs).

Checkpoints are network-only (`api.py:78-81`), so every parity and bench run uses
weights from a portable counter-hash PRNG: element `i` of the tensor named `name`
is `lowbias32(lowbias32(i ^ k0) ^ k1)` with `k0, k1` derived from `crc32(name)` and
the global seed. The same bits come out on any machine (numpy uint32 arithmetic
wraps mod 2^32 by definition), so the GPU box regenerates the weights the golden
vectors were made with instead of shipping 1.3 GB of tensors.

The reference zero-inits AdaLN and `proj_out` (`dit.py:264-274`); those are
overwritten here, otherwise every prediction is trivially zero.
"""

from __future__ import annotations

import math
import zlib

import numpy as np

from .configs import param_shapes

_M32 = np.uint32(0xFFFFFFFF)


def _lowbias32(x: np.ndarray) -> np.ndarray:
    # Chris Wellons' lowbias32 integer hash; all arithmetic is uint32 (wraps).
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846CA68B)
    x = x ^ (x >> np.uint32(16))
    return x


def hash_uniform(name: str, n: int, seed: int = 0) -> np.ndarray:
    """n float32 values uniform in [-1, 1), a pure function of (name, index, seed)."""
    h = zlib.crc32(name.encode()) & 0xFFFFFFFF
    k0 = np.uint32((h ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF)
    k1 = np.uint32(((h * 0x85EBCA6B) ^ (seed + 0x27D4EB2F)) & 0xFFFFFFFF)
    out = np.empty(n, dtype=np.float32)
    chunk = 1 << 24
    with np.errstate(over="ignore"):
        for s in range(0, n, chunk):
            i = np.arange(s, min(n, s + chunk), dtype=np.uint32)
            x = _lowbias32(_lowbias32(i ^ k0) ^ k1)
            # top 24 bits -> exact float32 in [0,1)
            u = (x >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / (1 << 24))
            out[s : s + len(i)] = u * np.float32(2.0) - np.float32(1.0)
    return out


def _init_scale(name: str, shape: tuple) -> "tuple[float, float]":
    """(offset, half-width) of the uniform init for one parameter."""
    sq3 = math.sqrt(3.0)
    if name.endswith("text_embed.text_embed.weight"):
        return 0.0, sq3  # std 1, like nn.Embedding's N(0,1)
    if name.endswith(".g") or name.endswith("norm.weight"):
        return 1.0, 0.1 * sq3  # norm gains around 1
    if "grn." in name:
        return 0.0, 0.1 * sq3
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return 0.0, sq3 / math.sqrt(fan_in)  # unit-variance outputs
    return 0.0, 0.02 * sq3  # biases


def make_weights(arch: dict, seed: int = 0) -> "dict[str, np.ndarray]":
    """Full synthetic state dict (float32 numpy, reference names without `transformer.`)."""
    out = {}
    for name, shape in param_shapes(arch).items():
        n = int(np.prod(shape))
        off, a = _init_scale(name, shape)
        w = hash_uniform(name, n, seed) * np.float32(a) + np.float32(off)
        out[name] = w.reshape(shape)
    return out


def make_weights_torch(arch: dict, seed: int = 0, dtype=None):
    import torch

    return {k: torch.from_numpy(v) if dtype is None else torch.from_numpy(v).to(dtype)
            for k, v in make_weights(arch, seed).items()}


# ---------------------------------------------------------------- inputs

def make_case(B: int, ref_frames, total_frames, n_text, *, seed: int = 1234, vocab: int = 2545):
    """Synthetic sample() inputs: cond mel ~ N(-4, 2^2) (log-mel-like range),
    text ids uniform in [0, vocab) padded with -1, per-utterance ref/total frames.

    Returns dict(cond[B,max_ref,100] f32, text[B,nt] int64, lens[B], duration[B]).
    Uses the torch CPU generator so the bits are identical on every host.
    """
    import torch

    ref = [int(r) for r in (ref_frames if hasattr(ref_frames, "__len__") else [ref_frames] * B)]
    tot = [int(t) for t in (total_frames if hasattr(total_frames, "__len__") else [total_frames] * B)]
    ntx = [int(t) for t in (n_text if hasattr(n_text, "__len__") else [n_text] * B)]
    g = torch.Generator().manual_seed(seed)
    max_ref = max(ref)
    cond = torch.randn(B, max_ref, 100, generator=g) * 2.0 - 4.0
    for b in range(B):
        cond[b, ref[b]:] = 0.0
    text = torch.full((B, max(ntx)), -1, dtype=torch.long)
    for b in range(B):
        text[b, : ntx[b]] = torch.randint(0, vocab, (ntx[b],), generator=g)
    return dict(
        cond=cond,
        text=text,
        lens=torch.tensor(ref, dtype=torch.long),
        duration=torch.tensor(tot, dtype=torch.long),
    )


def reference_noise(durations, seed, n_mel: int = 100, dtype=None):
    """y0 exactly as `CFM.sample` builds it on a CPU model (`cfm.py:196-201`):
    per utterance `torch.manual_seed(seed); randn(dur, n_mel)`, zero-padded."""
    import torch
    from torch.nn.utils.rnn import pad_sequence

    dtype = dtype or torch.float32
    ys = []
    for dur in durations:
        if seed is not None:
            torch.manual_seed(seed)
        ys.append(torch.randn(int(dur), n_mel, dtype=dtype))
    return pad_sequence(ys, padding_value=0, batch_first=True)


# Benchmark / parity configurations
def c1_case():
    return dict(preset="F5TTS_v1_Small_4L", B=1, ref=282, total=564, nt=90, nfe=4, cfg=2.0, sway=-1.0)


def c2_case():
    return dict(preset="F5TTS_v1_Base", B=1, ref=938, total=1876, nt=300, nfe=16, cfg=2.0, sway=-1.0)


def c3_case():
    tot = [564 + (i * 1312) // 31 for i in range(32)]
    return dict(preset="F5TTS_v1_Base", B=32, ref=[t // 2 for t in tot], total=tot,
                nt=[max(1, int(t / 6.25)) for t in tot], nfe=32, cfg=2.0, sway=-1.0)


def c4_case():
    """C4 per GPU: 256 utterances of 938 prompt + 938 generated frames over 8 GPUs = 32 per rank
    (SURVEY §8d), NFE 16 EPSS, CFG 2, batch path (B > 1)."""
    return dict(preset="F5TTS_v1_Base", B=32, ref=938, total=1876, nt=300, nfe=16, cfg=2.0, sway=-1.0)


def c5_case():
    return dict(preset="E2TTS_Base", B=8, ref=938, total=1876, nt=300, nfe=16, cfg=2.0, sway=-1.0)
