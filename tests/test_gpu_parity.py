"""GPU parity of the HIP engine (libf5h.so) against the reference's golden vectors and the
CPU oracle. Every call goes through the C ABI (ctypes) — no PyTorch compute on the path.

Tolerances (written here, BASELINE north star: "within 1e-3 rel fp32"):
  * fp32 engine mode vs reference fp32 output: max|diff| / max|ref| <= 1e-3.
  * bf16 / fp16 engine modes vs reference fp32: rel-L2 over the generated frames
    <= 1.5 x the reference's OWN bf16 / fp16 error vs its fp32 output.
"""

import os

import numpy as np
import pytest
import torch

import golden_cases as gc
from f5_tts_amd import synthetic
from f5_tts_amd.engine import gemm_force_config, op_attention, op_linear
from f5_tts_amd.model import CFM, DiT, UNetT

pytestmark = pytest.mark.gpu

FP32_TOL = 1e-3
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(arch, compute):
    cls = DiT if arch["backbone"] == "DiT" else UNetT
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = cls(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    m = CFM(transformer=net, num_channels=100, compute=compute).to(DEV)
    return m


def _sample(name, compute, keep_trajectory=True):
    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES[name]
    arch = gc.arch_of(tag)
    m = _model(arch, compute)
    inp = synthetic.make_case(**spec)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, gc.SEED)
    out, traj = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"].to(DEV),
                         lens=inp["lens"].to(DEV), steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway,
                         y0=y0.to(DEV), keep_trajectory=keep_trajectory)
    torch.cuda.synchronize()
    return out.float().cpu().numpy(), (None if traj is None else traj.float().cpu().numpy()), inp


# ---------------------------------------------------------------- ops
@pytest.mark.parametrize("compute,tol", [("fp32", 1e-5), ("bf16", 2e-2), ("fp16", 4e-3)])
@pytest.mark.parametrize("M,N,K", [(3752, 3072, 1024), (77, 100, 1024), (130, 2048, 512), (1, 128, 64)])
def test_op_linear(compute, tol, M, N, K):
    _need_gpu()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    C = op_linear(A, W, b, compute=compute)
    ref = A.double() @ W.double().t() + b.double()
    err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < tol, err


GEMM_CONFIGS = [0, 1, 5, 11, 12, 13]  # 11: ping-pong 8-wave 256x256; 12: 8-phase 256x256; 13: persistent ping-pong
if os.environ.get("F5H_TEST_GEMM_CFGS"):  # tuning runs: check extra configurations too
    GEMM_CONFIGS = [int(c) for c in os.environ["F5H_TEST_GEMM_CFGS"].split(",")]


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
@pytest.mark.parametrize("M,N,K", [(3752, 3072, 1024), (77, 100, 1024), (3752, 1024, 2048), (700, 2048, 128),
                                   (16384, 4096, 1024)])
def test_op_linear_every_tile_config(M, N, K, compute):
    """Every 16-bit tile configuration meets the fp64 reference and all of them agree bit for
    bit (same per-element K order: one lane, k-steps in sequence). 16384 x 4096: 1,024 tiles of
    256 x 256, the large-batch size class that picks cfg 11 by default."""
    _need_gpu()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    ref = A.double() @ W.double().t() + b.double()
    outs = []
    try:
        for cfg in GEMM_CONFIGS:
            gemm_force_config(cfg)
            C = op_linear(A, W, b, compute=compute)
            err = (C.double() - ref).abs().max().item() / ref.abs().max().item()
            assert err < 2e-2, (cfg, err)
            outs.append(C)
    finally:
        gemm_force_config(-1)
    for cfg, C in zip(GEMM_CONFIGS, outs):
        assert torch.equal(C, outs[0]), cfg


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
def test_sample_bitwise_identical_across_tile_configs(compute):
    """All GEMM epilogues (QKV+RoPE, gated residual, GELU, input projection) under every tile
    configuration: a Base-architecture sample is bitwise identical. fp16 also pins the epilogue
    rounding: no config may fold a product into its fp16 conversion (v_fma_mix) where another rounds
    it to fp32 first."""
    _need_gpu()
    from f5_tts_amd import configs

    arch = configs.get_arch("F5TTS_v1_Base")
    m = _model(arch, compute)
    inp = synthetic.make_case(B=2, ref_frames=[200, 150], total_frames=[700, 610], n_text=[90, 70])
    dur = torch.tensor([700, 610])
    y0 = synthetic.reference_noise(dur, 5)
    kw = dict(steps=2, cfg_strength=2.0, sway_sampling_coef=-1.0, keep_trajectory=False)
    outs = []
    try:
        for cfg in GEMM_CONFIGS:
            gemm_force_config(cfg)
            out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=dur.to(DEV),
                              lens=inp["lens"].to(DEV), y0=y0.to(DEV), **kw)
            outs.append(out)
    finally:
        gemm_force_config(-1)
    assert torch.isfinite(outs[0]).all()
    for cfg, o in zip(GEMM_CONFIGS, outs):
        assert torch.equal(o, outs[0]), cfg


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
@pytest.mark.parametrize("preset,depth", [("F5TTS_v1_Base", 2), ("F5TTS_v1_Small_4L", 2)])
def test_ln_fold_bitwise_identical_across_tile_configs(compute, preset, depth):
    """The LayerNorm fold (single-utterance DiT calls; DESIGN.md §3 'LayerNorm fold') under every tile configuration:
    bitwise identical. The consumers combine the producers' 64-column strip statistics either once per block row
    (gemm_kernel configurations 0/1/5) or per chunk row in the strip epilogue (the 256x256 kernels; 12 and 13 run
    the fold as 11), with every rounding written out so both forms give the same bits; d = 1024 (16 strips) and
    d = 768 (12: lanes holding one partial or none). Against the unfolded launches the result moves by the
    statistics' summation order only (rel-L2 well under the bf16 / fp16 rounding of the output)."""
    _need_gpu()
    from f5_tts_amd import configs

    arch = configs.get_arch(preset, depth=depth)
    m = _model(arch, compute)
    eng = m.transformer.get_engine(compute, m.device)
    inp = synthetic.make_case(B=1, ref_frames=[300], total_frames=[777], n_text=[90])
    dur = torch.tensor([777])
    y0 = synthetic.reference_noise(dur, 7)
    kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=dur.to(DEV), lens=inp["lens"].to(DEV),
              y0=y0.to(DEV), steps=3, cfg_strength=2.0, sway_sampling_coef=-1.0, keep_trajectory=False)
    outs = []
    try:
        eng.set_ln_fold(True)
        sup, p0 = eng.ln_fold_stats()
        assert sup, "the fold should be supported for this architecture"
        for cfg in GEMM_CONFIGS:
            gemm_force_config(cfg)
            outs.append(m.sample(**kw)[0].clone())
        _, p1 = eng.ln_fold_stats()
        assert p1 > p0, "no backbone pass ran with the fold"
        eng.set_ln_fold(False)
        gemm_force_config(-1)
        plain = m.sample(**kw)[0]
    finally:
        gemm_force_config(-1)
        eng.set_ln_fold(os.environ.get("F5H_LNFOLD", "1") != "0")
    assert torch.isfinite(outs[0]).all()
    for cfg, o in zip(GEMM_CONFIGS, outs):
        assert torch.equal(o, outs[0]), cfg
    rel = float((outs[0].float() - plain.float()).norm() / plain.float().norm())
    assert rel < (1e-2 if compute == "bf16" else 2e-3), rel


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
@pytest.mark.parametrize("preset,depth,spec", [
    ("E2TTS_Base", 4, dict(B=2, ref_frames=[100, 60], total_frames=[300, 220], n_text=[50, 40])),
    ("UNetT_tiny", 4, dict(B=1, ref_frames=[70], total_frames=[190], n_text=[30], vocab=64))])
def test_rms_fold_unett(compute, preset, depth, spec):
    """The UNetT RMSNorm fold (x_transformers RMSNorm, unett.py:300-301: the FFN-norms and the first half's
    attention-norms inside the GEMMs around them; the consumers read the residual stream with W diag(g)): on a masked
    batch with ragged lengths and on one utterance, bitwise identical under every tile configuration, and against
    the RMSNorm launches only the rounding moves (W diag(g) rounded once per weight instead of the normalised
    activations per element; rel-L2 well under the 16-bit output rounding's order)."""
    _need_gpu()
    from f5_tts_amd import configs

    over = {"depth": depth} if preset == "E2TTS_Base" else {"text_num_embeds": 64}
    arch = configs.get_arch(preset, **over)
    m = _model(arch, compute)
    eng = m.transformer.get_engine(compute, m.device)
    inp = synthetic.make_case(**spec)
    dur = torch.tensor(spec["total_frames"])
    y0 = synthetic.reference_noise(dur, 9)
    kw = dict(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=dur.to(DEV), lens=inp["lens"].to(DEV),
              y0=y0.to(DEV), steps=3, cfg_strength=2.0, sway_sampling_coef=-1.0, keep_trajectory=False)
    outs = []
    try:
        eng.set_ln_fold(True)
        sup, p0 = eng.ln_fold_stats()
        assert sup, "the RMSNorm fold should be supported for this architecture"
        for cfg in GEMM_CONFIGS:
            gemm_force_config(cfg)
            outs.append(m.sample(**kw)[0].clone())
        _, p1 = eng.ln_fold_stats()
        assert p1 > p0, "no backbone pass ran with the fold"
        gemm_force_config(-1)
        eng.set_ln_fold(False)
        plain = m.sample(**kw)[0]
    finally:
        gemm_force_config(-1)
        eng.set_ln_fold(os.environ.get("F5H_LNFOLD") == "1")  # UNetT engines: off unless asked for
    assert torch.isfinite(outs[0]).all()
    for cfg, o in zip(GEMM_CONFIGS, outs):
        assert torch.equal(o, outs[0]), cfg
    rel = float((outs[0].float() - plain.float()).norm() / plain.float().norm())
    assert rel < (1e-2 if compute == "bf16" else 2e-3), rel


@pytest.mark.parametrize("compute,tol", [("fp32", 1e-5), ("bf16", 2e-2), ("fp16", 4e-3)])
@pytest.mark.parametrize("S,H,N,masked", [(2, 16, 1876, False), (3, 2, 150, True), (1, 1, 65, False),
                                          (2, 4, 577, True)])
def test_op_attention(compute, tol, S, H, N, masked):
    _need_gpu()
    g = torch.Generator(device="cpu").manual_seed(S * 1000 + N)
    Q, K, V = (torch.randn(S, H, N, 64, generator=g).to(DEV) for _ in range(3))
    kv = torch.tensor([max(1, N - 37 * i) for i in range(S)], dtype=torch.int32) if masked else None
    O = op_attention(Q, K, V, kv, compute=compute)
    am = None
    if masked:
        am = (torch.arange(N)[None, :] < kv[:, None].long()).to(DEV)[:, None, None, :]
    ref = torch.nn.functional.scaled_dot_product_attention(Q.double(), K.double(), V.double(), attn_mask=am)
    ref = ref.transpose(1, 2).reshape(S, N, H * 64)
    err = (O.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < tol, err


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
@pytest.mark.parametrize("N", [577, 65, 1876])
def test_op_attention_ragged_tile_reads_no_foreign_rows(compute, N):
    """N % 64 != 0: the last K/V tile's rows past N must read as zero, not as the next (sequence, head)'s keys
    or the memory after V (the O buffer). The workspace is filled with NaN bits before the call:
    any foreign row that reaches the P.V MFMA (0 * NaN) makes the output NaN."""
    _need_gpu()
    S, H = 2, 4
    g = torch.Generator(device="cpu").manual_seed(N)
    Q, K, V = (torch.randn(S, H, N, 64, generator=g).to(DEV) for _ in range(3))
    O = op_attention(Q, K, V, None, compute=compute, poison=True)
    assert torch.isfinite(O).all()
    ref = torch.nn.functional.scaled_dot_product_attention(Q.double(), K.double(), V.double())
    ref = ref.transpose(1, 2).reshape(S, N, H * 64)
    err = (O.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (2e-2 if compute == "bf16" else 4e-3), err


@pytest.mark.parametrize("compute", ["bf16", "fp16"])
@pytest.mark.parametrize("spike", [0.0, 12.0, 20.0, 70.0, 160.0])
@pytest.mark.parametrize("safe", [False, True])
def test_op_attention_rare_branches(compute, spike, safe):
    """The 16-bit attention kernel against an fp64 softmax of the SAME rounded operands (the
    engine's layout: q pre-multiplied by (1/8)*log2(e), scores in log2 units), with inputs that
    force the rare branches (cdna_hip_programming.md rule 26): one key row at a late tile is
    aligned with a few query rows so their scores jump far above the first tile's. Against the first
    tile's max, P reaches ~2^spike: spike 12 stays in the fast path in both dtypes (P carried above 1),
    20 passes fp16's bound (2^15: the workgroup reruns in the lazy-max form), 70 bf16's (2^64), 160 both.
    safe=True forces that rerun everywhere (the lazy-max form alone, incl. its re-base past 2^8)."""
    _need_gpu()
    from f5_tts_amd.engine import attn_force_safe

    attn_force_safe(safe)
    try:
        _rare_branch_case(compute, spike)
    finally:
        attn_force_safe(False)


def _rare_branch_case(compute, spike):
    S, H, N = 2, 2, 700
    g = torch.Generator(device="cpu").manual_seed(11)
    Q, K, V = (torch.randn(S, H, N, 64, generator=g) for _ in range(3))
    Q = Q * (0.125 * 1.4426950408889634)
    if spike:
        for key, qs in ((650, (5, 6, 7)), (400, (300,))):
            for qi in qs:
                K[:, :, key] += spike * Q[:, :, qi] / Q[:, :, qi].pow(2).sum(-1, keepdim=True)
    dt = torch.bfloat16 if compute == "bf16" else torch.float16
    Q, K, V = (x.to(dt).float() for x in (Q, K, V))
    sc = Q.double() @ K.double().transpose(-1, -2)
    p = torch.exp2(sc - sc.amax(-1, keepdim=True))
    ref = (p / p.sum(-1, keepdim=True)) @ V.double()
    ref = ref.transpose(1, 2).reshape(S, N, H * 64)
    O = op_attention(Q.to(DEV), K.to(DEV), V.to(DEV), None, compute=compute, q_prescaled=True).cpu()
    assert torch.isfinite(O).all()
    err = ((O.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < (1e-2 if compute == "bf16" else 2e-3), err


# ---------------------------------------------------------------- backbone forward vs reference
@pytest.mark.parametrize("name", list(gc.FORWARD_CASES))
def test_forward_fp32_matches_reference(name):
    _need_gpu()
    g = gc.load(name)
    tag, spec, opts = gc.FORWARD_CASES[name]
    arch = gc.arch_of(tag)
    m = _model(arch, "fp32")
    inp = synthetic.make_case(**spec)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    N = int(dur.max())
    B = dur.shape[0]
    cond = torch.nn.functional.pad(inp["cond"], (0, 0, 0, N - inp["cond"].shape[1]))
    cmask = (torch.arange(N)[None] < inp["lens"][:, None])[..., None]
    step_cond = torch.where(cmask, cond, torch.zeros_like(cond))
    x = synthetic.reference_noise(dur, gc.SEED)
    mask = (torch.arange(N)[None] < dur[:, None]) if B > 1 else None
    pred = m.transformer(x=x.to(DEV), cond=step_cond.to(DEV), text=inp["text"].to(DEV),
                         time=torch.tensor(opts.get("t", gc.FWD_T)), mask=None if mask is None else mask.to(DEV),
                         cfg_infer=opts.get("cfg_infer", True), drop_audio_cond=opts.get("drop_audio", False),
                         drop_text=opts.get("drop_text", False), cache=True, compute="fp32")
    assert pred.shape == g["out"].shape
    err = gc.max_rel(pred.cpu().numpy(), g["out"])
    assert err < FP32_TOL, err


# ---------------------------------------------------------------- full CFM.sample vs reference
FP32_SAMPLE_CASES = [n for n in gc.SAMPLE_CASES]


@pytest.mark.parametrize("name", FP32_SAMPLE_CASES)
def test_sample_fp32_matches_reference(name):
    _need_gpu()
    g = gc.load(name)
    if g is None:
        pytest.skip(f"fixture {name} not generated")
    out, traj, inp = _sample(name, "fp32")
    np.testing.assert_allclose([float(inp["cond"].double().sum()), float(inp["text"].sum())], g["checksum"],
                               rtol=1e-12)
    e1 = gc.max_rel(traj[1], g["traj_1"])
    e = gc.max_rel(out, g["out"])
    assert e1 < FP32_TOL, e1
    assert e < FP32_TOL, e


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
@pytest.mark.parametrize("name", list(gc.EDGE_CASES))
def test_edge_sample_matches_reference(name, compute):
    """Edge paths of CFM.sample against the reference's own outputs: cfg=0 (one conditional forward,
    S=B), edit mask, no_ref_audio, int duration lifted by the duration rule, NFE 1, a 5-frame
    sequence, linspace grid with positive sway. fp32: max-rel <= 1e-3; bf16: rel-L2 <= 5e-2."""
    _need_gpu()
    g = gc.load(name)
    tag, spec, nfe, sway, cfg, extra = gc.EDGE_CASES[name]
    arch = gc.arch_of(tag)
    m = _model(arch, compute)
    inp = synthetic.make_case(**spec)
    kw = gc.edge_sample_kwargs(inp, extra)
    dur = torch.as_tensor(kw["duration"]).expand(inp["lens"].shape[0])
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, dur)
    y0 = synthetic.reference_noise(dur, gc.SEED)
    kw = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    out, traj = m.sample(**kw, steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway, y0=y0.to(DEV))
    torch.cuda.synchronize()
    out = out.float().cpu().numpy()
    assert out.shape == g["out"].shape
    if compute == "fp32":
        assert gc.max_rel(traj[1].float().cpu().numpy(), g["traj_1"]) < FP32_TOL
        assert gc.max_rel(out, g["out"]) < FP32_TOL
    else:
        assert gc.rel_err(out, g["out"]) < 5e-2


# (bf16/fp16 envelopes of C1/C2/C3/C5: tests/test_gpu_envelope.py)


# ---------------------------------------------------------------- size-independent properties
def test_deterministic_and_cond_region_exact():
    """Two runs are bitwise identical; the prompt region is exactly the cond (cfm.py:223)."""
    _need_gpu()
    a, _, inp = _sample("dit_tiny_sample_b3", "bf16", keep_trajectory=False)
    b, _, _ = _sample("dit_tiny_sample_b3", "bf16", keep_trajectory=False)
    assert np.array_equal(a, b)
    for i, L in enumerate(inp["lens"].tolist()):
        assert np.array_equal(a[i, :L], inp["cond"][i, :L].numpy())


@pytest.mark.parametrize("masked", [False, True])
def test_batch_permutation_equivariance_at_c3_shape(masked):
    """C3 shape (Base, B=32 mixed lengths padded to 1876): permuting the utterances of a batch
    permutes the outputs bit for bit (rows, sequences and masks are independent in the engine,
    as in the reference). Steps reduced to 3: the property does not depend on NFE."""
    _need_gpu()
    from f5_tts_amd import configs

    arch = configs.get_arch("F5TTS_v1_Base", attn_mask_enabled=masked)
    m = _model(arch, "bf16")
    c3 = synthetic.c3_case()
    inp = synthetic.make_case(B=c3["B"], ref_frames=c3["ref"], total_frames=c3["total"], n_text=c3["nt"])
    dur = torch.tensor(c3["total"])
    y0 = synthetic.reference_noise(dur, 11)
    kw = dict(steps=3, cfg_strength=2.0, sway_sampling_coef=-1.0, keep_trajectory=False)
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=dur.to(DEV),
                      lens=inp["lens"].to(DEV), y0=y0.to(DEV), **kw)
    perm = torch.randperm(c3["B"], generator=torch.Generator().manual_seed(0))
    outp, _ = m.sample(cond=inp["cond"][perm].to(DEV), text=inp["text"][perm].to(DEV), duration=dur[perm].to(DEV),
                       lens=inp["lens"][perm].to(DEV), y0=y0[perm].to(DEV), **kw)
    assert torch.isfinite(out).all()
    assert torch.equal(outp, out[perm.to(DEV)])
    for i in range(c3["B"]):
        L = int(inp["lens"][i])
        assert torch.equal(out[i, :L].cpu(), inp["cond"][i, :L])


@pytest.mark.parametrize("name", ["dit_tiny_sample_b3", "dit_tiny_sample_b3_masked", "unett_tiny_sample_b3"])
def test_step_graph_bitwise_equals_eager(name):
    """The hipGraph-replayed NFE step (default) and the eager launch sequence give bitwise
    identical outputs and trajectories. The first call of a shape captures the step graph and runs
    the prologue eagerly; the second captures the prologue graph (the shape repeats); the third
    replays both (no new capture); a different cfg strength captures its own step graph only."""
    _need_gpu()
    if name not in gc.SAMPLE_CASES:
        pytest.skip(f"{name} not a sample case")
    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES[name]
    arch = gc.arch_of(tag)
    m = _model(arch, "bf16")
    inp = synthetic.make_case(**spec)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, gc.SEED)
    eng = m.transformer.get_engine("bf16", m.device)

    def run(cfg_strength=cfg):
        out, traj = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"].to(DEV),
                             lens=inp["lens"].to(DEV), steps=nfe, cfg_strength=cfg_strength,
                             sway_sampling_coef=sway, y0=y0.to(DEV), keep_trajectory=True)
        torch.cuda.synchronize()
        return out.clone(), traj.clone()

    eng.set_graph_mode(False)
    o_e, t_e = run()
    eng.set_graph_mode(True)
    s0 = eng.graph_stats()
    o_g, t_g = run()
    s1 = eng.graph_stats()
    o_g2, t_g2 = run()
    s2 = eng.graph_stats()
    o_g3, t_g3 = run()
    s3 = eng.graph_stats()
    assert torch.equal(o_g, o_e) and torch.equal(t_g, t_e)
    assert torch.equal(o_g2, o_e) and torch.equal(t_g2, t_e)
    assert torch.equal(o_g3, o_e) and torch.equal(t_g3, t_e)
    assert s1["captures"] == s0["captures"] + 1  # the step graph; a new shape's prologue runs eagerly
    assert s2["captures"] == s1["captures"] + 1  # the shape repeats: its prologue graph
    assert s3["captures"] == s2["captures"], "third call on the same shape must replay"
    assert s3["replays"] - s2["replays"] == t_e.shape[0]  # nfe step replays + one prologue replay
    o_c, _ = run(cfg_strength=cfg + 0.5)
    assert eng.graph_stats()["captures"] == s3["captures"] + 1  # the prologue does not depend on cfg
    assert not torch.equal(o_c, o_e)


def test_concurrent_samples_on_two_streams_match_sequential():
    """The reference samples from a ThreadPoolExecutor (utils_infer.py:540-541). Two host threads,
    each on its own stream and with its own inputs, sampling repeatedly through one engine (step
    graphs on): every result equals the sequential one bit for bit."""
    _need_gpu()
    import threading

    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES["dit_tiny_sample_b3"]
    arch = gc.arch_of(tag)
    m = _model(arch, "bf16")
    cases = []
    for seed in (1, 2):
        inp = synthetic.make_case(**spec, seed=seed)
        dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
        cases.append((inp, synthetic.reference_noise(dur, seed)))

    def run(inp, y0):
        out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"].to(DEV),
                          lens=inp["lens"].to(DEV), steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway,
                          y0=y0.to(DEV), keep_trajectory=False)
        return out

    ref = [run(*c).clone() for c in cases]
    torch.cuda.synchronize()
    results, errors = [[], []], []

    def worker(i):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(4):
                    results[i].append(run(*cases[i]).clone())
            s.synchronize()
        except Exception as ex:  # surfaced below
            errors.append(ex)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(2):
        assert len(results[i]) == 4
        for r in results[i]:
            assert torch.equal(r, ref[i])


def test_maximum_length_matches_oracle_and_beyond_raises():
    """N = 8192, the reference's text position table (precompute_max_pos, dit.py:47): fp32 engine
    vs the CPU oracle within 1e-3 (DiT_tiny, 2 Euler steps); one frame more raises, as the
    reference's freqs_cis[:N] broadcast would."""
    _need_gpu()
    from oracle import ref_cpu

    arch = gc.arch_of("tiny")
    W = synthetic.make_weights_torch(arch)
    m = _model(arch, "fp32")
    inp = synthetic.make_case(B=1, ref_frames=4000, total_frames=8192, n_text=900, vocab=64)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, gc.SEED)
    kw = dict(steps=2, cfg_strength=2.0, sway_sampling_coef=-1.0)
    with torch.no_grad():
        ref, _ = ref_cpu.cfm_sample(W, arch, inp["cond"], inp["text"], inp["duration"], lens=inp["lens"], y0=y0, **kw)
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"].to(DEV),
                      lens=inp["lens"].to(DEV), y0=y0.to(DEV), keep_trajectory=False, **kw)
    torch.cuda.synchronize()
    assert out.shape == (1, 8192, 100)
    assert gc.max_rel(out.float().cpu().numpy(), ref.numpy()) < FP32_TOL
    with pytest.raises(RuntimeError):
        m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=8193, lens=inp["lens"].to(DEV),
                 keep_trajectory=False, **kw)


def _sample_pad_skip(m, compute, inp, y0, dur, steps, on, keep_trajectory=False):
    eng = m.transformer.get_engine(compute, torch.device(DEV))
    eng.set_pad_skip(on)
    try:
        out, traj = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=dur.to(DEV),
                             lens=inp["lens"].to(DEV), steps=steps, cfg_strength=2.0, sway_sampling_coef=-1.0,
                             y0=y0.to(DEV), keep_trajectory=keep_trajectory)
        torch.cuda.synchronize()
    finally:
        eng.set_pad_skip(True)
    return out.clone(), (None if traj is None else traj.clone())


@pytest.mark.parametrize("compute", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("name", ["base_batch_sample_b4", "base_batch_sample_b4_masked", "dit_tiny_sample_b3",
                                  "unett_tiny_sample_b3"])
def test_pad_row_skip_bitwise(name, compute):
    """The batch path's dead pad-row work (attention query blocks wholly past a sequence's length and
    out-proj row tiles of padding only, modules.py:551-553) is skipped by default; with and without the
    skip the outputs and whole trajectories are bitwise identical: valid rows, and pad rows, whose
    residual feeds later layers' keys/values when the attention mask is off."""
    _need_gpu()
    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES[name]
    m = _model(gc.arch_of(tag), compute)
    inp = synthetic.make_case(**spec)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, gc.SEED)
    a, ta = _sample_pad_skip(m, compute, inp, y0, dur, nfe, False, keep_trajectory=True)
    b, tb = _sample_pad_skip(m, compute, inp, y0, dur, nfe, True, keep_trajectory=True)
    assert torch.isfinite(b).all()
    assert torch.equal(a, b) and torch.equal(ta, tb)


@pytest.mark.parametrize("masked", [False, True])
def test_pad_row_skip_bitwise_at_c3_shape(masked):
    """C3 shape (Base, B=32, 564..1876 frames padded to 1876, 35 % padding): skip on == skip off, bit for
    bit, over the whole trajectory (3 steps: the property does not depend on NFE)."""
    _need_gpu()
    from f5_tts_amd import configs

    m = _model(configs.get_arch("F5TTS_v1_Base", attn_mask_enabled=masked), "bf16")
    c3 = synthetic.c3_case()
    inp = synthetic.make_case(B=c3["B"], ref_frames=c3["ref"], total_frames=c3["total"], n_text=c3["nt"])
    dur = torch.tensor(c3["total"])
    y0 = synthetic.reference_noise(dur, 11)
    a, ta = _sample_pad_skip(m, "bf16", inp, y0, dur, 3, False, keep_trajectory=True)
    b, tb = _sample_pad_skip(m, "bf16", inp, y0, dur, 3, True, keep_trajectory=True)
    assert torch.isfinite(b).all()
    assert torch.equal(a, b) and torch.equal(ta, tb)


@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_c3_full_batch_pinned_through_the_reference_pair(compute):
    """C3 at full size (Base, B=32, 564..1876 frames padded to 1876, batch-mask path), pinned to the reference:
    the shortest and the longest utterance of the batch, run by the reference as a B=2 batch at 1876 frames
    (tests/golden/c3_pair_sample_fp32.npz), match the fp32 engine <= 1e-3 (max-rel); and in both modes the
    full B=32 batch's rows of those utterances equal the engine's B=2 run bit for bit (sequences of one padded
    length never interact, in the reference as here: cfm.py:155-158, modules.py:511-553)."""
    _need_gpu()
    from f5_tts_amd import configs

    m = _model(configs.get_arch("F5TTS_v1_Base"), compute)
    full, pair = gc.c3_pair_inputs()
    kw = dict(steps=gc.C3_PAIR_NFE, cfg_strength=2.0, sway_sampling_coef=-1.0, keep_trajectory=False)

    def run(inp):
        y0 = synthetic.reference_noise(inp["duration"], gc.SEED)
        out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"],
                          lens=inp["lens"], y0=y0.to(DEV), **kw)
        torch.cuda.synchronize()
        return out

    out_pair = run(pair)
    out_full = run(full)
    assert torch.isfinite(out_full).all()
    assert torch.equal(out_full[list(gc.C3_PAIR)], out_pair)
    if compute == "fp32":
        ref = gc.load("c3_pair_sample_fp32")
        assert ref is not None
        got = out_pair.float().cpu().numpy()
        err = np.abs(got - ref["out"]).max() / np.abs(ref["out"]).max()
        assert err <= FP32_TOL, err
