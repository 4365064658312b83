"""The algorithmic FLOP counts behind bench.py's `path_tflops` and `roofline.achieved`, against the
figures SURVEY §8(d) derives from the reference's shapes (and thop's count, count_params_gflops.py)."""

import pytest

import bench
from f5_tts_amd import configs


def test_dit_base_sequence_forward_matches_survey():
    arch = configs.get_arch("F5TTS_v1_Base")
    n = 1876
    survey = 378.888e6 * n + 90112.0 * n * n  # F(N), SURVEY §8(d)
    assert bench.seq_flops(arch, n) == pytest.approx(survey, rel=1e-4)
    assert bench.seq_flops(arch, n) == pytest.approx(1027.9e9, rel=1e-3)
    # per NFE step (S = 2 with CFG) and per C2 call (NFE 16)
    assert 2 * bench.seq_flops(arch, n) == pytest.approx(2.056e12, rel=1e-3)
    assert 16 * 2 * bench.seq_flops(arch, n) == pytest.approx(32.89e12, rel=1e-3)


def test_e2_unett_sequence_forward_matches_survey():
    arch = configs.get_arch("E2TTS_Base")
    assert bench.seq_flops(arch, 1876) == pytest.approx(1591.3e9, rel=2e-3)
    attn = 4.0 * arch["depth"] * arch["dim"] * 1877 ** 2  # UNetT attends over N + 1 (time token)
    assert attn == pytest.approx(346.3e9, rel=2e-3)


def test_probe_class_flops():
    arch = configs.get_arch("F5TTS_v1_Base")
    S, L = 2, 1876
    assert bench.attn_flops(S, arch["heads"], L) == pytest.approx(28.83e9, rel=1e-3)
    assert bench.class_flops("attention", arch, S, L) == bench.attn_flops(S, arch["heads"], L)
    assert bench.class_flops("qkv", arch, S, L) == pytest.approx(23.6e9, rel=2e-3)
    assert bench.class_flops("out", arch, S, L) == pytest.approx(7.87e9, rel=2e-3)
    assert bench.class_flops("ffn1", arch, S, L) == pytest.approx(15.7e9, rel=3e-3)
    assert bench.class_flops("conv", arch, S, L) == pytest.approx(15.26e9, rel=3e-3)
    assert bench.class_flops("norm", arch, S, L) == 0.0  # HBM-bound: no FLOP roofline


def test_norm_bytes_follow_the_residual_width():
    """The pre-FFN LayerNorm reads the residual rows at the residual stream's width: the operand
    dtype on the 16-bit DiT path (engine.cpp backbone_part, EPI_RESID16), fp32 on the UNetT path."""
    S, L = 2, 1876
    dit, unett = configs.get_arch("F5TTS_v1_Base"), configs.get_arch("E2TTS_Base")
    assert bench.resid_bytes(dit) == 2 and bench.resid_bytes(unett) == 4
    assert bench.resid_bytes(dit, esz=4) == 4  # fp32 parity mode
    assert bench.class_bytes("norm", dit, S, L) == S * L * 1024 * (2 + 2)  # 15.37 MB
    assert bench.class_bytes("norm", unett, S, L) == S * L * 1024 * (4 + 2)


def test_pmc_traffic_only_at_the_measured_shape():
    """The committed PMC summary is attached to a bench line only at the launch shape it was measured
    on (C2: S=2, N=1876, Base); any other shape (C3, C5, fp32 tiny) reports no traffic."""
    c2 = {"S": 2, "L": 1876, "dim": 1024, "depth": 22}
    t, src = bench.pmc_traffic("attention", c2)
    assert t and t > 0 and src.startswith("profiles/")
    t, src = bench.pmc_traffic("attention", dict(c2, S=64))
    assert t is None and "not" in src


def test_conv_class_traffic_over_algorithmic():
    """The conv position embedding class carries its PMC traffic and algorithmic bytes (one grouped conv
    layer: input + output rows + the 16 groups' 31-tap weights) at the C2 shape."""
    arch = configs.get_arch("F5TTS_v1_Base")
    e = bench.class_entry("conv", 0.0257, 8, arch, 2, 1876, 16, 50.9, 1)
    assert e["algorithmic_bytes"] == 2 * 1876 * 1024 * 4 + 1024 * 64 * 31 * 2
    assert e["traffic"] and 1.0 < e["traffic_over_algorithmic"] < 10.0
