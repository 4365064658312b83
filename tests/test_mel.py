"""Log-mel front end: the CPU oracle against the reference's own conv STFT, and the
HIP path (f5h_mel_forward through ctypes) against the oracle.

Tolerances (written here):
  * oracle |STFT| vs reference conv_stft fixture: max|diff| / max|ref| <= 1e-5.
  * HIP vs oracle, fp32: mel (linear) max|diff| / max|ref| <= 1e-4; log-mel max|diff| <= 2e-3 on bins
    whose mel exceeds 1e-3 (below that the log amplifies fp32 summation-order differences; the
    clamp at 1e-5 is exact on both sides).
"""

import os

import numpy as np
import pytest
import torch

from oracle import mel_cpu

HERE = os.path.dirname(os.path.abspath(__file__))
DEV = "cuda:0"


@pytest.mark.parametrize("case", ["l6000", "l1300"])
def test_oracle_stft_magnitude_matches_reference_conv_stft(case):
    g = np.load(os.path.join(HERE, "golden", "mel_stft.npz"))
    wav, ref = torch.from_numpy(g[f"{case}_wav"]), torch.from_numpy(g[f"{case}_mag"])
    mag = mel_cpu.stft_mag(wav)
    assert mag.shape == ref.shape
    assert float((mag - ref).abs().max() / ref.abs().max()) <= 1e-5


def test_oracle_filterbank_properties():
    fb = mel_cpu.melscale_fbanks(513, 0.0, 12000.0, 100, 24000)
    assert fb.shape == (513, 100)
    assert (fb >= 0).all() and float(fb.max()) <= 1.0 + 1e-6
    assert (fb.sum(0) > 0).all()  # every filter covers at least one bin at n_fft 1024


def _wav(B, L, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(L) / 24000.0
    f = 100.0 + 400.0 * torch.rand(B, 1, generator=g)
    return 0.3 * torch.sin(2 * torch.pi * f * t) + 0.05 * torch.randn(B, L, generator=g)


@pytest.mark.gpu
@pytest.mark.parametrize("B,L", [(1, 240000), (3, 6000), (2, 513), (1, 1300)])
def test_mel_hip_matches_oracle(B, L):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from f5_tts_amd.mel import MelSpec

    wav = _wav(B, L, seed=L + B)
    ref = mel_cpu.log_mel(wav)
    out = MelSpec()(wav.to(DEV)).cpu()
    assert out.shape == ref.shape == (B, 100, 1 + L // 256)
    lin_err = float((out.exp() - ref.exp()).abs().max() / ref.exp().abs().max())
    assert lin_err <= 1e-4, lin_err
    sel = ref > np.log(1e-3)
    assert float((out - ref)[sel].abs().max()) <= 2e-3


@pytest.mark.gpu
def test_cfm_sample_raw_wave_cond_and_vocoder_run_on_hip():
    """CFM.sample on raw audio (cfm.py:106-109) goes through the HIP MelSpec: identical to sampling
    from the mel it produces; `vocoder=` (cfm.py:226-227) accepts the HIP Vocos."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import golden_cases as gc
    from f5_tts_amd import synthetic
    from f5_tts_amd.model import CFM, DiT
    from f5_tts_amd.vocos import Vocos, make_weights

    arch = gc.arch_of("tiny")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    m = CFM(transformer=net, num_channels=100, compute="bf16").to(DEV)
    wav = _wav(1, 60 * 256, seed=5).to(DEV)
    text = torch.randint(0, arch["text_num_embeds"], (1, 20)).to(DEV)
    args = dict(text=text, duration=150, steps=4, cfg_strength=2.0, sway_sampling_coef=-1.0, seed=3)
    a, _ = m.sample(cond=wav, **args)
    mel = m.mel_spec(wav).permute(0, 2, 1)
    b, _ = m.sample(cond=mel, **args)
    assert torch.equal(a, b)
    voc = Vocos(compute="bf16")
    voc.load_state_dict(make_weights())
    voc.to(DEV)
    wave, _ = m.sample(cond=mel, vocoder=voc.decode, **args)
    assert wave.shape == (1, (150 - 1) * 256) and torch.isfinite(wave).all()
