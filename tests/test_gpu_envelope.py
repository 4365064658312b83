"""Reduced-precision envelopes in the configs' own dtype, one test per path:

  C2  F5 v1 Base, B=1, NFE 16, 938+938 frames            (c2_sample_{fp32,bf16,fp16})
  C3  F5 v1 Base batch path, B=4 mixed 260-520 frames     (base_batch_sample_b4{,_bf16}), with and
      without the attention mask (base_batch_sample_b4_masked{,_bf16}): the batch mask of
      cfm.py:155-158 and the pad-row zeroing of modules.py:548-554
  C5  E2 Base UNetT, B=2                                  (e2_base_sample_b2{,_bf16}): unett.py:244-307
  C1  F5 v1 Small 4L                                      (c1_sample_{fp32,bf16,fp16})

Every fixture was produced by the reference itself (tests/golden/make_golden.py) from the same fp32
y0. Metric: rel-L2 over the generated frames of every utterance ([lens_i, dur_i)). Tolerance written
here: the engine's error vs the reference fp32 output is at most 1.5x the reference's OWN bf16 /
fp16 error vs its fp32 output. Each test prints e_ours / e_ref (and appends them to the file named
by F5H_ENVELOPE_LOG when set), so a regression inside the envelope is visible; DESIGN.md §4 records
the measured values, and every case carries an absolute bound at its measured value + 25 %.
"""

import json
import os

import numpy as np
import pytest
import torch

import golden_cases as gc
from f5_tts_amd import synthetic
from f5_tts_amd.model import CFM, DiT, UNetT

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
MARGIN = 1.5
# The engine's own error per case as measured on MI355X (round 3; the kernels are
# deterministic, so every box reproduces it): each case must stay within that value + 25 %, so a
# regression far inside the reference's envelope still fails.
MEASURED = {
    ("c2_sample_fp32", "bf16"): 0.010403,
    ("c2_sample_fp32", "fp16"): 0.0012941,
    ("base_batch_sample_b4", "bf16"): 0.019751,
    ("base_batch_sample_b4_masked", "bf16"): 0.018786,
    ("e2_base_sample_b2", "bf16"): 0.010949,  # 16-bit residual stream on UNetT (0.00824 with fp32)
    ("c1_sample_fp32", "bf16"): 0.0080304,
    ("c1_sample_fp32", "fp16"): 0.0010028,
    # round 4 (gpurun_out/r04a/envelopes.jsonl): reference fp16 errors 0.00191 and 0.1046
    ("e2_base_sample_b2", "fp16"): 0.0013136,
    ("base_batch_sample_b4_masked", "fp16"): 0.0023377,
}


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(arch, compute):
    cls = DiT if arch["backbone"] == "DiT" else UNetT
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = cls(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute=compute).to(DEV)


def _gen_frames(x, lens, dur):
    """Concatenated generated frames [lens_i, dur_i) of every utterance (the region the ODE writes)."""
    return np.concatenate([x[i, int(lens[i]):int(dur[i])] for i in range(x.shape[0])], axis=0)


def _record(name, compute, e_ours, e_ref):
    print(f"envelope {name} [{compute}]: e_ours={e_ours:.5f} e_ref={e_ref:.5f} ratio={e_ours / e_ref:.3f}")
    path = os.environ.get("F5H_ENVELOPE_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(dict(case=name, compute=compute, e_ours=e_ours, e_ref=e_ref)) + "\n")


def _envelope(case, lo_fixture, compute):
    f32, lo = gc.load(case), gc.load(lo_fixture)
    assert f32 is not None and lo is not None, (case, lo_fixture)
    tag, spec, nfe, sway, cfg = gc.SAMPLE_CASES[case]
    m = _model(gc.arch_of(tag), compute)
    eng = m.transformer.get_engine(compute, m.device)
    inp = synthetic.make_case(**spec)
    dur = torch.maximum(torch.maximum((inp["text"] != -1).sum(-1), inp["lens"]) + 1, inp["duration"])
    y0 = synthetic.reference_noise(dur, gc.SEED)
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"].to(DEV),
                      lens=inp["lens"].to(DEV), steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway,
                      y0=y0.to(DEV), keep_trajectory=False)
    out = out.float().cpu().numpy()
    # no phase-chain wait gave up (the chain is off by default; F5H_CHAIN=1 runs these cases through it)
    assert eng.chain_stats()[1] == 0, case
    assert out.shape == f32["out"].shape
    assert np.isfinite(out).all()
    ref32 = _gen_frames(f32["out"], inp["lens"], dur)
    e_ours = gc.rel_err(_gen_frames(out, inp["lens"], dur), ref32)
    e_ref = gc.rel_err(_gen_frames(lo["out"], inp["lens"], dur), ref32)
    _record(case, compute, e_ours, e_ref)
    return e_ours, e_ref


CASES = [
    ("c2_sample_fp32", "c2_sample_bf16", "bf16"),
    ("c2_sample_fp32", "c2_sample_fp16", "fp16"),
    ("base_batch_sample_b4", "base_batch_sample_b4_bf16", "bf16"),
    ("base_batch_sample_b4_masked", "base_batch_sample_b4_masked_bf16", "bf16"),
    ("e2_base_sample_b2", "e2_base_sample_b2_bf16", "bf16"),
    ("c1_sample_fp32", "c1_sample_bf16", "bf16"),
    ("c1_sample_fp32", "c1_sample_fp16", "fp16"),
    # round 4: fp16 (the reference's default GPU dtype) on the UNetT path and the masked batch path
    ("e2_base_sample_b2", "e2_base_sample_b2_fp16", "fp16"),
    ("base_batch_sample_b4_masked", "base_batch_sample_b4_masked_fp16", "fp16"),
]


@pytest.mark.parametrize("case,lo,compute", CASES, ids=[f"{c}-{m}" for c, _, m in CASES])
def test_within_reference_envelope(case, lo, compute):
    _need_gpu()
    e_ours, e_ref = _envelope(case, lo, compute)
    assert e_ours <= MARGIN * e_ref, (e_ours, e_ref)
    measured = MEASURED.get((case, compute))
    assert measured is not None, f"record the measured e_ours={e_ours:.6g} of {case} [{compute}] in MEASURED"
    assert e_ours <= 1.25 * measured, (e_ours, measured)
