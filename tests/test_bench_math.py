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
    """The pre-FFN norm reads the residual rows at the residual stream's width: the operand dtype in the
    16-bit modes on both backbones (engine.cpp backbone_part `r16`: EPI_RESID16 on DiT, the 16-bit UNetT
    stream since a041ce0), fp32 in the fp32 parity mode."""
    S, L = 2, 1876
    dit, unett = configs.get_arch("F5TTS_v1_Base"), configs.get_arch("E2TTS_Base")
    assert bench.resid_bytes(dit) == 2 and bench.resid_bytes(unett) == 2
    assert bench.resid_bytes(dit, esz=4) == 4  # fp32 parity mode
    assert bench.class_bytes("norm", dit, S, L) == S * L * 1024 * (2 + 2)  # 15.37 MB
    assert bench.class_bytes("norm", unett, S, L) == S * L * 1024 * (2 + 2)
    assert bench.class_bytes("norm", unett, S, L, esz=4) == S * L * 1024 * (4 + 4)


def _summary(path, shape, classes, head="abc1234", src="match"):
    import json

    d = {"shape": shape, "classes": classes, "head": head,
         "src_hash": bench.src_hash() if src == "match" else src}
    path.write_text(json.dumps(d))


@pytest.fixture
def fake_profiles(tmp_path, monkeypatch):
    """A profiles/ directory of stamped summaries (the committed ones change every round; these pin the
    attachment rules): PMC traffic at C2/C3/C4/C5, a C2 kernel trace and C2 SQ counters (bf16)."""
    c2 = {"S": 2, "L": 1876, "dim": 1024, "depth": 22}
    _summary(tmp_path / "r05_pmc_classes_c2.json", c2,
             {"attention": {"hbm_bytes": 30.9e6}, "qkv": {"hbm_bytes": 84.1e6},
              "conv": {"hbm_bytes": 2 * 1876 * 1024 * 7 + 1024 * 64 * 31 * 2}})
    _summary(tmp_path / "r05_pmc_classes_c3.json", dict(c2, S=64, config="c3"), {"qkv": {"hbm_bytes": 2.3e9}})
    _summary(tmp_path / "r05_pmc_classes_c4.json", dict(c2, S=64, config="c4"), {"qkv": {"hbm_bytes": 2.2e9}},
             src="0000000000000000")
    _summary(tmp_path / "r05_pmc_classes_c5.json", {"S": 16, "L": 1877, "dim": 1024, "depth": 24, "config": "c5"},
             {"ffn1": {"hbm_bytes": 1.1e9}})
    _summary(tmp_path / "r05_rocprof_classes_c2.json", dict(c2, config="c2"), {"attention": {"avg_launch_us": 35.0}})
    _summary(tmp_path / "r05_pmc_mfma_c2.json", dict(c2, config="c2"), {"attention": {"mfma_busy": 0.4}})
    monkeypatch.setattr(bench, "PROFILES", str(tmp_path))
    return tmp_path


def test_pmc_traffic_only_at_the_measured_shape(fake_profiles):
    """A committed PMC summary is attached to a bench line only at the launch shape it was measured on
    (C2: S=2, N=1876, Base; C3/C4: S=64 and the workload named; C5: S=16, N=1877, UNetT depth 24); any
    other shape or workload reports no traffic. Every attached summary names the git head it was measured
    at and whether its engine source hash is this tree's."""
    c2 = {"S": 2, "L": 1876, "dim": 1024, "depth": 22}
    t, src, prov = bench.pmc_traffic("attention", c2)
    assert t and t > 0 and "r05_pmc_classes_c2" in src
    assert prov == {"head": "abc1234", "src_hash": bench.src_hash(), "matches_build": True}
    t, src, prov = bench.pmc_traffic("attention", dict(c2, S=8))
    assert t is None and "no profiles" in src and prov is None
    t3, src3, p3 = bench.pmc_traffic("qkv", dict(c2, S=64, config="c3"))
    t4, src4, p4 = bench.pmc_traffic("qkv", dict(c2, S=64, config="c4"))
    assert "c3" in src3 and "c4" in src4 and t3 != t4
    assert p3["matches_build"] and not p4["matches_build"]  # the C4 summary came from other sources
    t, src, _ = bench.pmc_traffic("qkv", dict(c2, S=64, config="c9"))
    assert t is None and "no profiles" in src
    t, src, _ = bench.pmc_traffic("ffn1", {"S": 16, "L": 1877, "dim": 1024, "depth": 24, "config": "c5"})
    assert t and "c5" in src


def test_attached_summaries_name_their_source_commit(fake_profiles):
    """A bench line's class entry carries, beside every attached summary (traffic, kernel trace, SQ counters),
    the commit the summary was measured at and whether it matches the library's sources."""
    arch = configs.get_arch("F5TTS_v1_Base")
    e = bench.class_entry("attention", 0.036, 8, arch, 2, 1876, 352, 52.0, 1, config="c2", compute="bf16")
    for k in ("traffic", "rocprof", "pmc"):
        prov = e[k + "_provenance"]
        assert prov["head"] == "abc1234" and prov["matches_build"] is True, k


def test_timing_summaries_only_for_the_measured_compute_type(fake_profiles):
    """The committed kernel-trace averages and SQ counters (measured in bf16) are attached to a bf16 line
    only: an fp16 line at the same shape gets neither (fp16 runs the same cycles at a lower clock), while
    the byte traffic, which does not depend on the 16-bit type, is attached to both."""
    arch = configs.get_arch("F5TTS_v1_Base")
    bf = bench.class_entry("attention", 0.036, 8, arch, 2, 1876, 352, 52.0, 1, config="c2", compute="bf16")
    fp = bench.class_entry("attention", 0.037, 8, arch, 2, 1876, 352, 52.0, 1, config="c2", compute="fp16")
    assert "rocprof_frac" in bf and "pmc" in bf
    assert "rocprof_frac" not in fp and "pmc" not in fp
    assert bf["traffic"] and fp["traffic"] == bf["traffic"]


def test_conv_class_traffic_over_algorithmic(fake_profiles):
    """The conv position embedding class carries its PMC traffic and algorithmic bytes (the mean of its two
    grouped conv layers: fp32 input + 16-bit output, then 16-bit input + fp32 residual + 16-bit output; plus
    the 16 groups' 31-tap weights) at the C2 shape."""
    arch = configs.get_arch("F5TTS_v1_Base")
    e = bench.class_entry("conv", 0.0257, 8, arch, 2, 1876, 16, 50.9, 1)
    assert e["algorithmic_bytes"] == 2 * 1876 * 1024 * 7 + 1024 * 64 * 31 * 2
    assert e["traffic"] and 0.8 < e["traffic_over_algorithmic"] < 1.5


# avg launch (us) per class measured by the round-3 final benches (profiles/archive/r03_final_bench_c{2,4,5}.log),
# the shapes they ran at, and the compute width: every class's fraction of its roofline must be <= 1
_R03 = {
    ("F5TTS_v1_Base", 2, 1876): {"qkv": 26.459, "attention": 39.594, "out": 13.812, "norm": 6.341, "ffn1": 21.227,
                                 "ffn2": 23.446, "conv": 27.03},
    ("F5TTS_v1_Base", 64, 1876): {"qkv": 796.296, "attention": 1263.983, "out": 303.667, "norm": 92.033,
                                  "ffn1": 558.906, "ffn2": 509.969, "conv": 754.97},
    ("E2TTS_Base", 16, 1877): {"qkv": 210.808, "attention": 313.483, "out": 79.899, "norm": 22.413, "ffn1": 286.598,
                               "ffn2": 266.688, "conv": 193.805},
}


def test_no_class_fraction_exceeds_its_roofline():
    """Bookkeeping guard (round-3 verdict: the C5 norm class read 1.029 of HBM peak because the UNetT
    residual was priced at 4 B after it became 16-bit): with the measured launch times every class's
    algorithmic work per launch / time stays below peak; the C5 norm class reads ~0.69."""
    for (preset, S, L), times in _R03.items():
        arch = configs.get_arch(preset)
        for kc, us in times.items():
            e = bench.class_entry(kc, us * 1e-3, 8, arch, S, L, 352, 50.0, 1, config=None, esz=2)
            assert 0.0 < e["frac"] <= 1.0, (preset, S, kc, e["frac"])
    e = bench.class_entry("norm", 22.413e-3, 8, configs.get_arch("E2TTS_Base"), 16, 1877, 384, 480.0)
    assert e["frac"] == pytest.approx(0.686, abs=0.01)


def test_unett_residual_is_16_bit():
    unett = configs.get_arch("E2TTS_Base")
    assert bench.resid_bytes(unett) == 2 and bench.resid_bytes(unett, esz=4) == 4


def _bench_cmd(*args, env=None):
    import os
    import subprocess
    import sys

    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, bench.__file__, *args], capture_output=True, text=True, timeout=240,
                          env=e)


def test_gpus_n_starts_n_ranks_and_prints_one_line():
    """`bench.py --gpus 2` with no outer launcher starts 2 rank processes itself (gloo stand-in worker on
    CPU): both ranks join the timed region, rank 0 prints exactly one JSON line with n_gpus 2, dp2."""
    import json

    r = _bench_cmd("--gpus", "2", "--standin", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_joined"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["utterances_gathered"] == 8 and d["steps"] == 2


def test_launcher_parent_makes_no_hip_call(monkeypatch, capsys):
    """launch_ranks counts GPUs in a child process: with every torch entry that could reach the HIP runtime
    made to raise in this (parent) process, `--gpus 8` on a box with fewer GPUs (none here) still exits 2 with
    the message, and the parent's CUDA/HIP state stays uninitialised (bench.py:launch_ranks)."""
    import torch

    def boom(*a, **k):
        raise AssertionError("the launcher parent touched the GPU runtime")

    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    monkeypatch.setattr(torch.cuda, "init", boom)
    args = bench.parse_args(["--gpus", "8", "--steps", "1", "--warmup", "0"])
    rc = bench.launch_ranks(args, ["--gpus", "8", "--steps", "1", "--warmup", "0"])
    assert rc == 2
    assert "--gpus 8 but only" in capsys.readouterr().err
    assert not torch.cuda.is_initialized()


def test_outer_launcher_world_size_mismatch_fails():
    r = _bench_cmd("--gpus", "2", "--standin", "--steps", "1", "--warmup", "0",
                   env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_cpu_baseline_extrapolates_batch_configs():
    """C3/C4/C5 CPU baselines run a slice of the batch for 1 and 2 NFE steps and extrapolate x NFE x B/b
    (BASELINE.md §3); C1/C2 time the whole call. Tiny architecture, so it runs in seconds."""
    arch = configs.get_arch("DiT_tiny", text_num_embeds=64)
    case = dict(B=4, ref=[20, 30, 25, 40], total=[48, 64, 56, 80], nt=[8, 10, 9, 12], nfe=8, cfg=2.0, sway=-1.0)
    c = bench.cpu_baseline("c4", case, arch, threads=2)
    assert c["extrapolated"] is True and c["slice_utterances"] == 2 and c["value"] > 0
    assert c["seconds"] > c["per_step_s"] * 8  # (fixed + NFE x step) x B/b
    c = bench.cpu_baseline("c1", dict(case, B=1, ref=20, total=48, nt=8), arch, threads=2)
    assert c["extrapolated"] is False and c["value"] > 0


def test_pad_skip_prices_attention_and_out_on_live_rows():
    """With the pad-row skip (C3: mixed lengths) the attention class is priced on live query rows against all
    keys and the out-projection on live rows; QKV/FFN keep every row; equal lengths change nothing."""
    arch = configs.get_arch("F5TTS_v1_Base")
    q = [1876, 564, 1200, 900] * 2  # B = 4, CFG copies
    S, L = len(q), 1876
    a = bench.class_entry("attention", 1.0, 8, arch, S, L, 22, 100.0, qlens=q)
    assert a["flops_per_launch"] == 4.0 * 16 * 64 * L * sum(q)
    assert a["padded_flops_per_launch"] == bench.class_flops("attention", arch, S, L) > a["flops_per_launch"]
    o = bench.class_entry("out", 1.0, 8, arch, S, L, 22, 100.0, qlens=q)
    assert o["flops_per_launch"] == 2.0 * sum(q) * 1024 * 1024
    f = bench.class_entry("ffn1", 1.0, 8, arch, S, L, 22, 100.0, qlens=q)
    assert f["flops_per_launch"] == bench.class_flops("ffn1", arch, S, L) and "padded_flops_per_launch" not in f
    same = bench.class_entry("attention", 1.0, 8, arch, S, L, 22, 100.0, qlens=[L] * S)
    assert same["flops_per_launch"] == bench.class_flops("attention", arch, S, L)


def test_live_row_traffic_pricing_at_c3(fake_profiles):
    """With the pad-row skip (ragged C3 batch) attention reads K and V of every row but Q and O of the live
    query rows only, and the out-projection touches live rows only: their algorithmic bytes count those rows
    (round 4's C3 PMC summary measured 1.0-1.2x of them; 0.86x / 0.95x of the padded count)."""
    arch = configs.get_arch("F5TTS_v1_Base")
    tot = [564 + (i * 1312) // 31 for i in range(32)]
    q = tot * 2  # CFG copies
    c3 = {"S": 64, "L": 1876, "dim": 1024, "depth": 22, "config": "c3"}
    live_attn = 2 * 2 * 16 * 64 * (64 * 1876 + sum(q))
    live_out = 2 * (sum(q) * 1024 + 1024 * 1024) + 2 * 2 * sum(q) * 1024
    _summary(fake_profiles / "r05_pmc_classes_c3.json", c3,
             {"attention": {"hbm_bytes": 1.01 * live_attn}, "out": {"hbm_bytes": 1.2 * live_out}})
    at = bench.class_entry("attention", 1.058, 8, arch, 64, 1876, 704, 2262.0, 1, config="c3", qlens=q)
    assert at["algorithmic_bytes"] == 2 * 2 * 16 * 64 * (64 * 1876 + sum(q))
    out = bench.class_entry("out", 0.300, 8, arch, 64, 1876, 704, 2262.0, 1, config="c3", qlens=q)
    assert out["algorithmic_bytes"] == 2 * (sum(q) * 1024 + 1024 * 1024) + 2 * 2 * sum(q) * 1024
    for e in (at, out):
        assert e["traffic"] and 0.95 < e["traffic_over_algorithmic"] < 2.0


def test_visible_gpus_reads_kfd_topology(tmp_path, monkeypatch):
    """The launcher's GPU count comes from sysfs (KFD nodes with SIMDs) narrowed by the visibility variables;
    no torch/HIP entry is reached."""
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):
        (tmp_path / str(i)).mkdir()
        (tmp_path / str(i) / "properties").write_text(f"cpu_cores_count 4\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.kfd_gpu_nodes(str(tmp_path)) == 3
    assert bench.visible_gpus(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert bench.visible_gpus(str(tmp_path)) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert bench.visible_gpus(str(tmp_path)) == 1
    assert bench.kfd_gpu_nodes(str(tmp_path / "absent")) is None
