"""Generate the golden vectors in tests/golden/ by running the REFERENCE implementation.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py [--skip-c2]

The reference's own `f5_tts.model.{CFM, DiT, UNetT}` are imported from
/root/reference/src with third-party pieces that are absent from this image
restated here:
  * x_transformers RotaryEmbedding / apply_rotary_pos_emb / RMSNorm (x_transformers>=1.31.14,
    pyproject.toml:44) — restated from the library's published algorithm: interleaved
    `(d r)` frequency layout, rotate_half on adjacent pairs, fp32 math cast back;
    RMSNorm = F.normalize(x)*sqrt(d)*g.
  * torchdiffeq.odeint(method="euler") — fixed grid, y1 = y0 + (t1-t0)*f(t0,y0).
  * torchaudio / librosa / rjieba / pypinyin / f5_tts.model.trainer — empty stubs
    (mel front end, tokenizers and training are off the sampling path).
Weights are the hash-PRNG weights of f5_tts_amd.synthetic (regenerable anywhere);
inputs come from seeded torch CPU generators. Only OUTPUTS (plus small input
checksums) are stored, as float32 .npz.
"""

from __future__ import annotations

import argparse
import os
import sys
import time
import types

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "f5-tts_amd"))
sys.dont_write_bytecode = True  # /root/reference is read-only

from f5_tts_amd import configs, synthetic  # noqa: E402

REF_SRC = "/root/reference/src"


# ----------------------------------------------------------------- third-party restatements
class RotaryEmbedding(nn.Module):
    def __init__(self, dim, use_xpos=False, scale_base=512, interpolation_factor=1.0, base=10000,
                 base_rescale_factor=1.0):
        super().__init__()
        base *= base_rescale_factor ** (dim / (dim - 2))
        inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2).float() / dim))
        self.register_buffer("inv_freq", inv_freq)
        self.interpolation_factor = interpolation_factor

    def forward_from_seq_len(self, seq_len):
        t = torch.arange(seq_len, device=self.inv_freq.device)
        return self.forward(t)

    def forward(self, t):
        if t.ndim == 1:
            t = t[None, :]
        freqs = torch.einsum("bi,j->bij", t.type_as(self.inv_freq), self.inv_freq) / self.interpolation_factor
        freqs = torch.stack((freqs, freqs), dim=-1).flatten(-2)
        return freqs, 1.0


def _rotate_half(x):
    x = x.unflatten(-1, (-1, 2))
    x1, x2 = x.unbind(dim=-1)
    return torch.stack((-x2, x1), dim=-1).flatten(-2)


def apply_rotary_pos_emb(t, freqs, scale=1):
    rot_dim, seq_len, orig_dtype = freqs.shape[-1], t.shape[-2], t.dtype
    freqs = freqs[:, -seq_len:, :]
    if t.ndim == 4 and freqs.ndim == 3:
        freqs = freqs[:, None]
    t, t_unrot = t[..., :rot_dim], t[..., rot_dim:]
    t = (t * freqs.cos() * scale) + (_rotate_half(t) * freqs.sin() * scale)
    return torch.cat((t, t_unrot), dim=-1).type(orig_dtype)


class RMSNorm(nn.Module):
    def __init__(self, dim, unit_offset=False):
        super().__init__()
        self.unit_offset = unit_offset
        self.scale = dim ** 0.5
        self.g = nn.Parameter(torch.ones(dim) * (1.0 - float(unit_offset)))

    def forward(self, x):
        return F.normalize(x, dim=-1) * self.scale * (self.g + float(self.unit_offset))


def odeint(func, y0, t, method="euler", **kw):
    assert method == "euler"
    ys = [y0]
    y = y0
    for t0, t1 in zip(t[:-1], t[1:]):
        y = y + (t1 - t0) * func(t0, y)
        ys.append(y)
    return torch.stack(ys)


def install_shims():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    xt = mod("x_transformers", RMSNorm=RMSNorm)
    xt.x_transformers = mod("x_transformers.x_transformers", RotaryEmbedding=RotaryEmbedding,
                            apply_rotary_pos_emb=apply_rotary_pos_emb)
    mod("torchdiffeq", odeint=odeint)
    mod("torchaudio", transforms=types.SimpleNamespace())
    lib = mod("librosa")
    lib.filters = mod("librosa.filters", mel=lambda **k: None)
    mod("rjieba", cut=lambda s: list(s))
    mod("pypinyin", Style=types.SimpleNamespace(TONE3=3), lazy_pinyin=lambda *a, **k: [])
    mod("f5_tts.model.trainer", Trainer=object)
    sys.path.insert(0, REF_SRC)


# ----------------------------------------------------------------- reference model helpers
def build_ref(arch):
    from f5_tts.model import CFM, DiT, UNetT

    kw = {k: arch[k] for k in ("dim", "depth", "heads", "dim_head", "ff_mult", "text_dim", "text_mask_padding",
                                "conv_layers", "pe_attn_head", "attn_mask_enabled", "qk_norm")}
    kw["text_num_embeds"] = arch["text_num_embeds"]
    kw["mel_dim"] = arch["mel_dim"]
    if arch["backbone"] == "DiT":
        net = DiT(**kw)
    else:
        net = UNetT(**kw)
    ident = nn.Identity()
    ident.n_mel_channels = 100
    model = CFM(transformer=net, mel_spec_module=ident, num_channels=100)
    sd = {"transformer." + k: v for k, v in synthetic.make_weights_torch(arch).items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    bad = [m for m in missing if not (m.endswith("inv_freq") or m.endswith("freqs_cis"))]
    assert not bad and not unexpected, (bad, unexpected)
    return model.eval()


class fp32_noise:
    """Make the reference's y0 recipe draw fp32 noise and cast (same y0 for every dtype)."""

    def __enter__(self):
        self.orig = torch.randn

        def randn(*a, dtype=None, device=None, **k):
            return self.orig(*a, **k).to(dtype=dtype or torch.float32)

        torch.randn = randn

    def __exit__(self, *e):
        torch.randn = self.orig


def run_sample(arch, case, nfe, cfg=2.0, sway=-1.0, dtype=torch.float32, seed=7, use_epss=True):
    model = build_ref(arch).to(dtype)
    inp = synthetic.make_case(**case)
    with fp32_noise(), torch.no_grad():
        out, traj = model.sample(cond=inp["cond"], text=inp["text"], duration=inp["duration"], lens=inp["lens"],
                                 steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway, seed=seed,
                                 use_epss=use_epss)
    return out.float().numpy(), traj.float().numpy(), inp


def run_edge(name, seed=7):
    """One golden_cases.EDGE_CASES entry through the reference CFM.sample."""
    import golden_cases as gc

    tag, case, nfe, sway, cfg, extra = gc.EDGE_CASES[name]
    model = build_ref(gc.arch_of(tag))
    inp = synthetic.make_case(**case)
    kw = gc.edge_sample_kwargs(inp, extra)
    with fp32_noise(), torch.no_grad():
        out, traj = model.sample(**kw, steps=nfe, cfg_strength=cfg, sway_sampling_coef=sway, seed=seed)
    return dict(out=out.float().numpy(), traj_last=traj[-1].float().numpy(), traj_1=traj[1].float().numpy(),
                checksum=checksum(inp))


def run_forward(arch, case, t_val=0.3, seed=7, cfg_infer=True, drop_audio_cond=False, drop_text=False):
    """One backbone forward at time t (dit.py:319-370): packed cond/uncond (cfg_infer=True) or one
    branch with the drop flags; t_val a scalar or one value per sample."""
    model = build_ref(arch)
    inp = synthetic.make_case(**case)
    B = inp["cond"].shape[0]
    dur = inp["duration"]
    N = int(dur.max())
    cond = F.pad(inp["cond"], (0, 0, 0, N - inp["cond"].shape[1]))
    cmask = (torch.arange(N)[None] < inp["lens"][:, None])[..., None]
    step_cond = torch.where(cmask, cond, torch.zeros_like(cond))
    x = synthetic.reference_noise(dur, seed)
    mask = (torch.arange(N)[None] < dur[:, None]) if B > 1 else None
    with torch.no_grad():
        out = model.transformer(x=x, cond=step_cond, text=inp["text"], time=torch.tensor(t_val), mask=mask,
                                cfg_infer=cfg_infer, drop_audio_cond=drop_audio_cond, drop_text=drop_text,
                                cache=True)
        model.transformer.clear_cache()
    return out.float().numpy()


def checksum(inp):
    return np.array([float(inp["cond"].double().sum()), float(inp["text"].sum())], dtype=np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-c2", action="store_true")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    install_shims()
    torch.set_num_threads(8)

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tests/
    import golden_cases as gc

    tiny = configs.get_arch("DiT_tiny", text_num_embeds=64)
    tiny_v0 = configs.get_arch("DiT_tiny", text_num_embeds=64, text_mask_padding=False, pe_attn_head=1)
    tiny_masked = configs.get_arch("DiT_tiny", text_num_embeds=64, attn_mask_enabled=True)
    utiny = configs.get_arch("UNetT_tiny", text_num_embeds=64)
    c1 = configs.get_arch("F5TTS_v1_Small_4L")
    b1 = dict(B=1, ref_frames=60, total_frames=150, n_text=30, vocab=64)
    b3 = dict(B=3, ref_frames=[40, 60, 25], total_frames=[90, 150, 70], n_text=[20, 30, 12], vocab=64)

    jobs = {}
    for name, (tag, spec, opts) in gc.FORWARD_CASES.items():
        jobs[name] = (lambda a, sp, o: (lambda: dict(out=run_forward(a, sp, **gc.forward_ref_kwargs(o)))))(
            gc.arch_of(tag), spec, opts)

    def sample_job(arch, case, nfe, **kw):
        def f():
            out, traj, inp = run_sample(arch, case, nfe, **kw)
            return dict(out=out, traj_last=traj[-1], traj_1=traj[1], checksum=checksum(inp))
        return f

    jobs["dit_tiny_sample_b1"] = sample_job(tiny, b1, 4)
    jobs["dit_tiny_sample_b3"] = sample_job(tiny, b3, 6)
    jobs["dit_tiny_sample_b3_masked"] = sample_job(tiny_masked, b3, 6)
    jobs["dit_v0_tiny_sample_b3"] = sample_job(tiny_v0, b3, 5, sway=None)
    jobs["dit_tiny_sample_b1_lin32"] = sample_job(tiny, b1, 32, cfg=2.0, sway=-1.0)
    jobs["unett_tiny_sample_b1"] = sample_job(utiny, b1, 4)
    jobs["unett_tiny_sample_b3"] = sample_job(utiny, b3, 4)
    c1_case = dict(B=1, ref_frames=282, total_frames=564, n_text=90)
    for dt, tag in ((torch.float32, "fp32"), (torch.bfloat16, "bf16"), (torch.float16, "fp16")):
        jobs[f"c1_sample_{tag}"] = sample_job(c1, c1_case, 4, dtype=dt)
    for name in gc.EDGE_CASES:
        jobs[name] = (lambda n: (lambda: run_edge(n)))(name)
    # Base-size cases (round 2): E2 UNetT Base (C5 architecture) and the F5 v1 Base batch path, both at
    # reduced NFE and frame counts so the CPU reference finishes in seconds; fp32.
    e2 = configs.get_arch("E2TTS_Base")
    base = configs.get_arch("F5TTS_v1_Base")
    base_masked = configs.get_arch("F5TTS_v1_Base", attn_mask_enabled=True)
    jobs["e2_base_sample_b2"] = sample_job(e2, gc.E2B2, 2)
    jobs["base_batch_sample_b4"] = sample_job(base, gc.BASE_B4, 2)
    jobs["base_batch_sample_b4_masked"] = sample_job(base_masked, gc.BASE_B4, 2)
    # round 3: the same three cases run by the reference in bf16 (same fp32 y0), i.e. the reference's
    # own reduced-precision envelope for the C3 batch-mask path and the C5 (UNetT) path
    jobs["e2_base_sample_b2_bf16"] = sample_job(e2, gc.E2B2, 2, dtype=torch.bfloat16)
    jobs["base_batch_sample_b4_bf16"] = sample_job(base, gc.BASE_B4, 2, dtype=torch.bfloat16)
    jobs["base_batch_sample_b4_masked_bf16"] = sample_job(base_masked, gc.BASE_B4, 2, dtype=torch.bfloat16)
    # round 4: the reference in fp16 (its default GPU dtype, utils_infer.py:190-199) on the UNetT path
    # (16-bit residual stream) and the masked batch path
    jobs["e2_base_sample_b2_fp16"] = sample_job(e2, gc.E2B2, 2, dtype=torch.float16)
    jobs["base_batch_sample_b4_masked_fp16"] = sample_job(base_masked, gc.BASE_B4, 2, dtype=torch.float16)
    def c3_pair_job():
        # the C3 pair (golden_cases.C3_PAIR): sliced out of the B=32 C3 inputs, reference B=2 batch at 1876 frames
        model = build_ref(base)
        _, pair = gc.c3_pair_inputs()
        with fp32_noise(), torch.no_grad():
            out, traj = model.sample(cond=pair["cond"], text=pair["text"], duration=pair["duration"],
                                     lens=pair["lens"], steps=gc.C3_PAIR_NFE, cfg_strength=2.0,
                                     sway_sampling_coef=-1.0, seed=7)
        return dict(out=out.float().numpy(), traj_1=traj[1].float().numpy(), checksum=checksum(pair))

    jobs["c3_pair_sample_fp32"] = c3_pair_job
    if not args.skip_c2:
        c2 = configs.get_arch("F5TTS_v1_Base")
        jobs["c2_sample_fp32"] = sample_job(c2, gc.C2, 16)
        # the reference's own reduced-precision envelopes at C2 (same fp32 y0)
        jobs["c2_sample_bf16"] = sample_job(c2, gc.C2, 16, dtype=torch.bfloat16)
        jobs["c2_sample_fp16"] = sample_job(c2, gc.C2, 16, dtype=torch.float16)

    # time grids (model/utils.py:205-218 + cfm.py:215-216), computed by the reference itself
    from f5_tts.model.utils import get_epss_timesteps

    grids = {}
    for n in (4, 5, 6, 7, 10, 12, 16, 32):
        t = get_epss_timesteps(n, "cpu", torch.float32)
        grids[f"nfe{n}"] = (t + -1.0 * (torch.cos(torch.pi / 2 * t) - 1 + t)).numpy()
        grids[f"nfe{n}_nosway"] = t.numpy()
    np.savez(os.path.join(HERE, "time_grids.npz"), **grids)

    for name, fn in jobs.items():
        if args.only and args.only not in name:
            continue
        t0 = time.time()
        res = fn()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **{k: np.asarray(v) for k, v in res.items()})
        print(f"{name}: {time.time() - t0:.1f}s  out{tuple(res['out'].shape)} absmax {np.abs(res['out']).max():.3f}",
              flush=True)


if __name__ == "__main__":
    main()
