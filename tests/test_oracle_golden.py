"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs.

The golden .npz files were produced by running the reference implementation
(tests/golden/make_golden.py). A restatement that disagrees with them is not an
oracle, so every GPU parity claim rests on these tests.
"""

import numpy as np
import pytest
import torch

import golden_cases as gc
from f5_tts_amd import synthetic
from oracle import ref_cpu

SAMPLE_TOL = 2e-5  # fp32 vs fp32: only summation order differs


def _inputs(spec):
    return synthetic.make_case(**spec)


@pytest.mark.parametrize("name", [n for n in gc.FORWARD_CASES])
def test_oracle_forward_matches_reference(name, torch_threads):
    g = gc.load(name)
    assert g is not None, f"missing fixture {name}"
    tag, spec, opts = gc.FORWARD_CASES[name]
    arch = gc.arch_of(tag)
    W = synthetic.make_weights_torch(arch)
    inp = _inputs(spec)
    pre = ref_cpu.prepare(arch, inp["cond"], inp["text"], inp["duration"], inp["lens"])
    x = synthetic.reference_noise(pre["duration"], gc.SEED)
    fwd = ref_cpu.dit_forward if arch["backbone"] == "DiT" else ref_cpu.unett_forward
    with torch.no_grad():
        out = fwd(W, arch, x, pre["step_cond"], inp["text"], torch.tensor(opts.get("t", gc.FWD_T)), pre["mask"], {},
                  packed=opts.get("cfg_infer", True), drop_audio=opts.get("drop_audio", False),
                  drop_text=opts.get("drop_text", False))
    assert gc.max_rel(out.numpy(), g["out"]) < SAMPLE_TOL


@pytest.mark.parametrize("name", [n for n in gc.SAMPLE_CASES if not n.startswith("c2")])
def test_oracle_sample_matches_reference(name, torch_threads):
    g = gc.load(name)
    assert g is not None, f"missing fixture {name}"
    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES[name]
    arch = gc.arch_of(tag)
    W = synthetic.make_weights_torch(arch)
    inp = _inputs(spec)
    np.testing.assert_allclose(
        [float(inp["cond"].double().sum()), float(inp["text"].sum())], g["checksum"], rtol=1e-12
    )
    out, traj = ref_cpu.cfm_sample(W, arch, inp["cond"], inp["text"], inp["duration"], lens=inp["lens"],
                                   steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway, seed=gc.SEED)
    assert gc.max_rel(traj[1].numpy(), g["traj_1"]) < SAMPLE_TOL
    assert gc.max_rel(out.numpy(), g["out"]) < SAMPLE_TOL


@pytest.mark.parametrize("name", list(gc.EDGE_CASES))
def test_oracle_edge_sample_matches_reference(name, torch_threads):
    """cfg=0 single forward, edit mask, no_ref_audio, int duration, NFE 1, 5-frame sequence,
    linspace grid with positive sway: the reference's own outputs."""
    g = gc.load(name)
    assert g is not None, f"missing fixture {name}"
    tag, spec, nfe, sway, cfg, extra = gc.EDGE_CASES[name]
    arch = gc.arch_of(tag)
    W = synthetic.make_weights_torch(arch)
    inp = _inputs(spec)
    kw = gc.edge_sample_kwargs(inp, extra)
    out, traj = ref_cpu.cfm_sample(W, arch, kw.pop("cond"), kw.pop("text"), kw.pop("duration"), steps=nfe,
                                   cfg_strength=cfg, sway_sampling_coef=sway, seed=gc.SEED, **kw)
    assert out.shape == g["out"].shape
    assert gc.max_rel(traj[1].numpy(), g["traj_1"]) < SAMPLE_TOL
    assert gc.max_rel(out.numpy(), g["out"]) < SAMPLE_TOL


def test_time_grids_match_reference():
    g = gc.load("time_grids")
    for n in (4, 5, 6, 7, 10, 12, 16, 32):
        t = ref_cpu.epss_sway_grid(n, -1.0)
        np.testing.assert_array_equal(t.numpy(), g[f"nfe{n}"])
        np.testing.assert_array_equal(ref_cpu.epss_sway_grid(n, None).numpy(), g[f"nfe{n}_nosway"])
    # the NFE-16 EPSS+sway grid
    np.testing.assert_allclose(g["nfe16"][[1, 8, 12, 15]], [0.001205, 0.07612, 0.292893, 0.80491], atol=2e-6)


@pytest.mark.parametrize("tag", ["bf16", "fp16"])
def test_reference_c2_envelope_recorded(tag):
    """The reference's own reduced-precision error at C2 (same fp32 y0): the bar the engine's bf16 and
    fp16 modes are held to in the GPU tests (<= 1.5x of it)."""
    f32, lo = gc.load("c2_sample_fp32"), gc.load(f"c2_sample_{tag}")
    gen = slice(938, None)
    e = gc.rel_err(lo["out"][:, gen], f32["out"][:, gen])
    assert 1e-4 < e < 0.3, e


def test_reference_bf16_envelope_recorded():
    """the reference's own bf16 error vs its fp32 output at C1 (~4.5e-2 rel-L2)."""
    f32, b16, f16 = gc.load("c1_sample_fp32"), gc.load("c1_sample_bf16"), gc.load("c1_sample_fp16")
    gen = slice(282, None)
    e_b = gc.rel_err(b16["out"][:, gen], f32["out"][:, gen])
    e_h = gc.rel_err(f16["out"][:, gen], f32["out"][:, gen])
    assert 5e-3 < e_b < 0.2 and e_h < e_b


def test_oracle_c3_pair_matches_reference(torch_threads):
    """The C3 pair fixture (the shortest and the longest utterance of the C3 batch as a B=2 batch at 1876
    frames, Base, NFE 2; golden_cases.C3_PAIR): the oracle reproduces the reference's own output."""
    g = gc.load("c3_pair_sample_fp32")
    assert g is not None
    arch = gc.arch_of("c2")
    W = synthetic.make_weights_torch(arch)
    _, pair = gc.c3_pair_inputs()
    np.testing.assert_allclose([float(pair["cond"].double().sum()), float(pair["text"].sum())], g["checksum"],
                               rtol=1e-12)
    out, traj = ref_cpu.cfm_sample(W, arch, pair["cond"], pair["text"], pair["duration"], lens=pair["lens"],
                                   steps=gc.C3_PAIR_NFE, cfg_strength=2.0, sway_sampling_coef=-1.0, seed=gc.SEED)
    assert gc.max_rel(traj[1].numpy(), g["traj_1"]) < SAMPLE_TOL
    assert gc.max_rel(out.numpy(), g["out"]) < SAMPLE_TOL
