"""Golden-vector case table shared by the oracle tests and the GPU parity tests.

Each case names: the arch, the synthetic input spec, and the sampler settings
that tests/golden/make_golden.py ran the reference with. Fixtures are float32 .npz.
"""

from __future__ import annotations

import os

import numpy as np

from f5_tts_amd import configs

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

B1 = dict(B=1, ref_frames=60, total_frames=150, n_text=30, vocab=64)
B3 = dict(B=3, ref_frames=[40, 60, 25], total_frames=[90, 150, 70], n_text=[20, 30, 12], vocab=64)
C1 = dict(B=1, ref_frames=282, total_frames=564, n_text=90)
C2 = dict(B=1, ref_frames=938, total_frames=1876, n_text=300)
# Base-size cases (fp32 fixtures, reduced NFE/frames): E2 UNetT Base (the C5 architecture, its skip-proj
# GEMMs and ff 4096) and the F5 v1 Base batch path (C3's mask semantics at Base dimensions).
E2B2 = dict(B=2, ref_frames=[100, 60], total_frames=[300, 220], n_text=[50, 40])
BASE_B4 = dict(B=4, ref_frames=[120, 200, 80, 150], total_frames=[400, 520, 260, 450], n_text=[60, 90, 40, 70])


# C3 at full length (round 4): the shortest and the longest utterance of the C3 batch (synthetic.c3_case,
# make_case seed 1234), sliced out of the B=32 inputs, run by the reference as a B=2 batch padded to 1876
# frames (the batch-mask path). The GPU tests pin the engine on this pair against the reference and then the
# full B=32 C3 batch to the pair bit for bit (sequences of one padded length are independent).
C3_PAIR = (0, 31)
C3_PAIR_NFE = 2


def c3_pair_inputs():
    """The C3 batch inputs (B=32) and the pair slice: (full, pair) dicts of cond/text/lens/duration."""
    from f5_tts_amd import synthetic

    c3 = synthetic.c3_case()
    full = synthetic.make_case(B=c3["B"], ref_frames=c3["ref"], total_frames=c3["total"], n_text=c3["nt"])
    idx = list(C3_PAIR)
    pair = {k: v[idx] for k, v in full.items()}
    return full, pair


def arch_of(tag):
    if tag == "tiny":
        return configs.get_arch("DiT_tiny", text_num_embeds=64)
    if tag == "tiny_v0":
        return configs.get_arch("DiT_tiny", text_num_embeds=64, text_mask_padding=False, pe_attn_head=1)
    if tag == "tiny_masked":
        return configs.get_arch("DiT_tiny", text_num_embeds=64, attn_mask_enabled=True)
    if tag == "utiny":
        return configs.get_arch("UNetT_tiny", text_num_embeds=64)
    if tag == "c1":
        return configs.get_arch("F5TTS_v1_Small_4L")
    if tag == "c2":
        return configs.get_arch("F5TTS_v1_Base")
    if tag == "c2_masked":
        return configs.get_arch("F5TTS_v1_Base", attn_mask_enabled=True)
    if tag == "e2":
        return configs.get_arch("E2TTS_Base")
    raise KeyError(tag)


# name -> (arch tag, input spec, nfe, sway, cfg)
SAMPLE_CASES = {
    "dit_tiny_sample_b1": ("tiny", B1, 4, -1.0, 2.0),
    "dit_tiny_sample_b3": ("tiny", B3, 6, -1.0, 2.0),
    "dit_tiny_sample_b3_masked": ("tiny_masked", B3, 6, -1.0, 2.0),
    "dit_v0_tiny_sample_b3": ("tiny_v0", B3, 5, None, 2.0),
    "dit_tiny_sample_b1_lin32": ("tiny", B1, 32, -1.0, 2.0),
    "unett_tiny_sample_b1": ("utiny", B1, 4, -1.0, 2.0),
    "unett_tiny_sample_b3": ("utiny", B3, 4, -1.0, 2.0),
    "c1_sample_fp32": ("c1", C1, 4, -1.0, 2.0),
    "c2_sample_fp32": ("c2", C2, 16, -1.0, 2.0),
    "e2_base_sample_b2": ("e2", E2B2, 2, -1.0, 2.0),
    "base_batch_sample_b4": ("c2", BASE_B4, 2, -1.0, 2.0),
    "base_batch_sample_b4_masked": ("c2_masked", BASE_B4, 2, -1.0, 2.0),
}

# Backbone-plugin forwards (DiT.forward / UNetT.forward, dit.py:319-370): name -> (arch tag, input
# spec, options). Options: cfg_infer (default True: packed cond/uncond), drop_audio / drop_text (single
# branch), t (scalar or one value per sample; default FWD_T).
FORWARD_CASES = {
    "dit_tiny_fwd_b1": ("tiny", B1, {}),
    "dit_tiny_fwd_b3": ("tiny", B3, {}),
    "unett_tiny_fwd_b1": ("utiny", B1, {}),
    "unett_tiny_fwd_b3": ("utiny", B3, {}),
    "dit_tiny_fwd_b3_single": ("tiny", B3, {"cfg_infer": False}),
    "dit_tiny_fwd_b3_dropaudio": ("tiny", B3, {"cfg_infer": False, "drop_audio": True}),
    "dit_tiny_fwd_b3_droptext": ("tiny", B3, {"cfg_infer": False, "drop_text": True}),
    "dit_tiny_fwd_b1_dropboth": ("tiny", B1, {"cfg_infer": False, "drop_audio": True, "drop_text": True}),
    "dit_tiny_fwd_b3_tvec": ("tiny", B3, {"t": [0.1, 0.7, 0.1]}),
    "unett_tiny_fwd_b3_droptext": ("utiny", B3, {"cfg_infer": False, "drop_text": True}),
    "unett_tiny_fwd_b3_tvec_single": ("utiny", B3, {"cfg_infer": False, "t": [0.9, 0.2, 0.5]}),
}


SEED = 7
FWD_T = 0.3


def forward_ref_kwargs(opts):
    """make_golden.run_forward keyword arguments of a FORWARD_CASES option dict."""
    return dict(t_val=opts.get("t", FWD_T), cfg_infer=opts.get("cfg_infer", True),
                drop_audio_cond=opts.get("drop_audio", False), drop_text=opts.get("drop_text", False))


def load(name):
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        return None
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def max_rel(a, b):
    """max |a-b| / max |b|  (the '≤1e-3 rel' figure used throughout)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


# Edge cases of CFM.sample's host preamble and ODE loop (reference cfm.py:83-229), each produced by
# the reference itself (tests/golden/make_golden.py --only edge):
# name -> (arch tag, input spec, nfe, sway, cfg, extra)
#   extra: edit     -> edit_mask [B, cond_len] with a False span [lens//3, lens//2) (speech_edit.py path)
#          no_ref   -> no_ref_audio=True (cfm.py:146-147)
#          int_dur  -> duration passed as a python int (cfm.py:132-139 rule then lifts it per utterance)
#          epss     -> use_epss flag
#          dup      -> duplicate_test=True with t_inter = value (cfm.py:141-143, 205-209)
SHORT = dict(B=1, ref_frames=3, total_frames=5, n_text=2, vocab=64)
EDGE_CASES = {
    "edge_dit_nocfg_b1": ("tiny", B1, 4, -1.0, 0.0, {}),
    "edge_dit_nocfg_b3": ("tiny", B3, 3, -1.0, 0.0, {}),
    "edge_unett_nocfg_b3": ("utiny", B3, 3, -1.0, 0.0, {}),
    "edge_dit_edit_b3": ("tiny", B3, 4, -1.0, 2.0, {"edit": True}),
    "edge_dit_noref_b1": ("tiny", B1, 4, -1.0, 2.0, {"no_ref": True}),
    "edge_dit_intdur_b3": ("tiny", B3, 2, -1.0, 2.0, {"int_dur": 10}),
    "edge_dit_nfe1_b1": ("tiny", B1, 1, None, 2.0, {}),
    "edge_dit_short_b1": ("tiny", SHORT, 3, -1.0, 2.0, {}),
    "edge_dit_lin7_b3": ("tiny", B3, 7, 0.5, 1.5, {"epss": False}),
    "edge_dit_duptest_b1": ("tiny", B1, 8, -1.0, 2.0, {"dup": 0.1}),
    "edge_dit_duptest_b3": ("tiny", dict(B3, total_frames=[90, 150, 130]), 6, None, 2.0, {"dup": 0.25}),
}


def edit_mask_for(lens, cond_len):
    """[B, cond_len] bool: True except [lens//3, lens//2) per utterance."""
    import torch

    ar = torch.arange(cond_len)[None]
    lo, hi = (lens // 3)[:, None], (lens // 2)[:, None]
    return ~((ar >= lo) & (ar < hi))


def edge_sample_kwargs(inp, extra):
    """The CFM.sample keyword arguments of an edge case (inputs from synthetic.make_case)."""
    kw = dict(cond=inp["cond"], text=inp["text"], lens=inp["lens"],
              duration=extra.get("int_dur", inp["duration"]))
    if extra.get("edit"):
        kw["edit_mask"] = edit_mask_for(inp["lens"], inp["cond"].shape[1])
    if extra.get("no_ref"):
        kw["no_ref_audio"] = True
    if "epss" in extra:
        kw["use_epss"] = extra["epss"]
    if "dup" in extra:
        kw["duplicate_test"] = True
        kw["t_inter"] = extra["dup"]
    return kw
