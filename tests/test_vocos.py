"""Vocos decoder: the CPU oracle against the reference's own inverse STFT, and the
HIP path (f5h_vocos_decode through ctypes) against the oracle.

Tolerances (written here):
  * oracle iSTFT vs reference conv_stft fixture: max|diff| / max|ref| <= 1e-5 (both fp32).
  * fp32 engine vs oracle: max|diff| / max|ref| <= 1e-3 (the north star's fp32 bar).
  * bf16 backbone (head + iSTFT stay fp32) vs fp32 oracle: rel-L2 <= 5e-2 (bf16 operands in
    17 GEMMs; parity "bf16 envelope" as for the CFM path).
Synthetic weights (hash PRNG, f5_tts_amd.vocos.make_weights): the mel-24khz checkpoint is
network-only; the ConvNeXt backbone is "parity unpinned" beyond the restatement of vocos 0.1.0.
"""

import os

import numpy as np
import pytest
import torch

from oracle import vocos_cpu

HERE = os.path.dirname(os.path.abspath(__file__))
DEV = "cuda:0"


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _mel(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 100, T, generator=g) * 2.0 - 4.0  # log-mel range


def _maxrel(a, b):
    return float((a - b).abs().max() / b.abs().max())


# ---------------------------------------------------------------- CPU: oracle pinned
@pytest.mark.parametrize("case", ["t24", "t5"])
def test_oracle_istft_matches_reference_conv_stft(case):
    g = np.load(os.path.join(HERE, "golden", "vocos_istft.npz"))
    real, imag = torch.from_numpy(g[f"{case}_real"]), torch.from_numpy(g[f"{case}_imag"])
    y = vocos_cpu.istft(real, imag)
    T = real.shape[-1]
    assert y.shape == (real.shape[0], (T - 1) * 256)
    ref = torch.from_numpy(g[f"{case}_audio"])[:, : y.shape[1]]  # conv_stft keeps T*hop; vocos (T-1)*hop
    assert _maxrel(y, ref) <= 1e-5


def test_host_param_names_match_oracle():
    from f5_tts_amd import vocos as fv

    assert fv.param_shapes() == vocos_cpu.param_shapes()
    W = fv.make_weights()
    assert {k: tuple(v.shape) for k, v in W.items()} == vocos_cpu.param_shapes()


def test_oracle_decode_shapes_and_linearity_of_istft():
    """iSTFT is linear: istft(a S1 + S2) = a istft(S1) + istft(S2) (size-independent property)."""
    g = torch.Generator().manual_seed(3)
    r1, i1, r2, i2 = (torch.randn(1, 513, 9, generator=g) for _ in range(4))
    lhs = vocos_cpu.istft(2.5 * r1 + r2, 2.5 * i1 + i2)
    rhs = 2.5 * vocos_cpu.istft(r1, i1) + vocos_cpu.istft(r2, i2)
    assert _maxrel(lhs, rhs) < 1e-5


# ---------------------------------------------------------------- GPU: HIP path vs oracle
def _vocos(compute):
    from f5_tts_amd.vocos import Vocos, make_weights

    W = make_weights()
    v = Vocos(compute=compute)
    v.load_state_dict(W)
    return v.to(DEV).eval(), W


@pytest.mark.gpu
@pytest.mark.parametrize("B,T", [(1, 938), (2, 100), (3, 5), (1, 2)])
def test_vocos_fp32_matches_oracle(B, T):
    _gpu()
    v, W = _vocos("fp32")
    mel = _mel(B, T, seed=B * 1000 + T)
    ref = vocos_cpu.decode(W, vocos_cpu.VOCOS_MEL_24KHZ, mel)
    out = v.decode(mel.to(DEV)).cpu()
    assert out.shape == ref.shape
    assert torch.isfinite(out).all()
    assert _maxrel(out, ref) <= 1e-3, _maxrel(out, ref)


@pytest.mark.gpu
def test_vocos_bf16_close_to_oracle():
    _gpu()
    v, W = _vocos("bf16")
    mel = _mel(1, 938, seed=7)
    ref = vocos_cpu.decode(W, vocos_cpu.VOCOS_MEL_24KHZ, mel)
    out = v.decode(mel.to(DEV)).cpu()
    rel = float((out - ref).norm() / ref.norm())
    assert rel <= 5e-2, rel


@pytest.mark.gpu
def test_vocos_batch_equals_single_and_t1_is_empty():
    """Utterances of a batch are independent: a batched decode equals per-utterance decodes bit for
    bit (fixed per-element reduction order in every kernel). T = 1 gives an empty waveform."""
    _gpu()
    v, _ = _vocos("bf16")
    mel = _mel(3, 64, seed=11).to(DEV)
    batched = v.decode(mel)
    for b in range(3):
        assert torch.equal(batched[b], v.decode(mel[b:b + 1])[0])
    assert v.decode(_mel(1, 1, seed=1).to(DEV)).shape == (1, 0)
