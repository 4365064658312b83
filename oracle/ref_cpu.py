"""ORACLE — test infrastructure only. CPU restatement of the reference CFM sampling path.

This module is the checker for the HIP engine, never part of the product path:
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg import it.

What it restates (fp32, PyTorch-CPU, written from scratch against the reference's
semantics; file:line refer to /root/reference/src/f5_tts):

  cfm_sample ........ CFM.sample                      model/cfm.py:83-229
  epss_sway_grid .... get_epss_timesteps + sway       model/utils.py:205-218, model/cfm.py:211-216
  euler ............. torchdiffeq odeint(method=euler) (third-party; call cfm.py:218)
  dit_forward ....... DiT.forward (cfg pack)          model/backbones/dit.py:319-370
  text_embed_dit .... TextEmbedding (v1, per-sample)  model/backbones/dit.py:86-139
  convnext .......... ConvNeXtV2Block + GRN           model/modules.py:236-280
  input_embed ....... InputEmbedding + ConvPosEmbed   model/backbones/dit.py:145-164, model/modules.py:175-201
  time_embed ........ TimestepEmbedding + sinus       model/modules.py:157-169, 852-862
  rope .............. x_transformers RotaryEmbedding / apply_rotary_pos_emb
                      (third-party x_transformers>=1.31.14, pyproject.toml:44; interleaved pairs,
                      cross-checked by runtime/triton_trtllm/patch/f5tts/modules.py:210-276)
  dit_block ......... DiTBlock / AdaLayerNorm / Attention / AttnProcessor / FeedForward
                      model/modules.py:312-364, 451-556, 711-757
  unett_forward ..... UNetT.forward                   model/backbones/unett.py:244-307
  rms_norm .......... x_transformers RMSNorm: F.normalize(x)*sqrt(d)*g

Parity pin: tests/golden/*.npz were produced by importing the reference itself in the
build container (tests/golden/make_golden.py); tests/test_oracle_golden.py checks this
restatement against them. The third-party pieces (rotary, RMSNorm, Euler) are pinned
only through the generator's own restatement of them ("parity unpinned"
for those by the reference's tests; the in-tree TRT restatement agrees on rotary layout
and Euler form).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPSS = {  # model/utils.py:207-214
    5: [0, 2, 4, 8, 16, 32],
    6: [0, 2, 4, 6, 8, 16, 32],
    7: [0, 2, 4, 6, 8, 16, 24, 32],
    10: [0, 2, 4, 6, 8, 12, 16, 20, 24, 28, 32],
    12: [0, 2, 4, 6, 8, 10, 12, 14, 16, 20, 24, 28, 32],
    16: [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32],
}


def epss_sway_grid(steps: int, sway, use_epss=True, dtype=torch.float32, t_start=0.0):
    """Time grid (cfm.py:211-216): EPSS table /32 when t_start == 0 (else linspace(t_start, 1)),
    then t += s*(cos(pi/2 t) - 1 + t)."""
    if t_start == 0 and use_epss and steps in EPSS:
        t = (1 / 32) * torch.tensor(EPSS[steps], dtype=dtype)
    else:
        t = torch.linspace(t_start, 1, steps + 1, dtype=dtype)
    if sway is not None:
        t = t + sway * (torch.cos(torch.pi / 2 * t) - 1 + t)
    return t


def lens_to_mask(lens, length=None):
    length = int(lens.max()) if length is None else length
    return torch.arange(length)[None, :] < lens[:, None]


# ------------------------------------------------------------------ small blocks

def time_embed(W, t):
    """sinus(256, scale 1000) -> Linear -> SiLU -> Linear. t: [b]."""
    half = 128
    k = math.log(10000) / (half - 1)
    freq = torch.exp(torch.arange(half).float() * -k)
    e = 1000.0 * t.float()[:, None] * freq[None, :]
    e = torch.cat((e.sin(), e.cos()), -1).to(t.dtype)
    h = F.linear(e, W["time_embed.time_mlp.0.weight"], W["time_embed.time_mlp.0.bias"])
    return F.linear(F.silu(h), W["time_embed.time_mlp.2.weight"], W["time_embed.time_mlp.2.bias"])


def freqs_cis_table(dim, end, theta=10000.0):
    f = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].float() / dim))
    p = torch.outer(torch.arange(end).float(), f)
    return torch.cat([torch.cos(p), torch.sin(p)], -1)


def grn(x, gamma, beta):
    g = torch.linalg.vector_norm(x, ord=2, dim=1, keepdim=True)  # over TIME (dim=1)
    n = g / (g.mean(dim=-1, keepdim=True) + 1e-6)
    return gamma * (x * n) + beta + x


def convnext(W, p, x):
    r = x
    y = F.conv1d(x.transpose(1, 2), W[p + "dwconv.weight"], W[p + "dwconv.bias"], padding=3,
                 groups=x.shape[-1]).transpose(1, 2)
    y = F.layer_norm(y, (y.shape[-1],), W[p + "norm.weight"], W[p + "norm.bias"], eps=1e-6)
    y = F.gelu(F.linear(y, W[p + "pwconv1.weight"], W[p + "pwconv1.bias"]))  # erf GELU
    y = grn(y, W[p + "grn.gamma"], W[p + "grn.beta"])
    y = F.linear(y, W[p + "pwconv2.weight"], W[p + "pwconv2.bias"])
    return r + y


def text_embed_dit(W, arch, text, seq_len, drop_text):
    """TextEmbedding.forward of the v1 DiT. seq_len: int, or LongTensor [b] (batched path)."""
    text = text + 1
    per_sample = torch.is_tensor(seq_len)
    n = int(seq_len.max()) if per_sample else int(seq_len)
    text = text[:, :n]
    text = F.pad(text, (0, n - text.shape[1]), value=0)
    valid = None
    if per_sample:
        valid = torch.arange(n)[None, :] < seq_len[:, None]
        text = text.masked_fill(~valid, 0)
    fill = text == 0  # taken BEFORE drop_text (dit.py:103-107)
    if drop_text:
        text = torch.zeros_like(text)
    e = W["text_embed.text_embed.weight"][text]
    if valid is not None:
        e = e.masked_fill(~valid[..., None], 0.0)
    if arch["conv_layers"] > 0:
        fc = freqs_cis_table(arch["text_dim"], 8192)[:n]
        if valid is not None:
            fc = fc[None] * valid[..., None].float()
        e = e + fc
        if arch["text_mask_padding"]:
            e = e.masked_fill(fill[..., None], 0.0)
            for i in range(arch["conv_layers"]):
                e = convnext(W, f"text_embed.text_blocks.{i}.", e)
                e = e.masked_fill(fill[..., None], 0.0)
        else:
            for i in range(arch["conv_layers"]):
                e = convnext(W, f"text_embed.text_blocks.{i}.", e)
    return e


def conv_pos(W, x, mask):
    """ConvPositionEmbedding: [mask] conv(k31,g16) [mask] Mish conv [mask] Mish."""
    m = None if mask is None else mask[:, None, :]
    y = x.transpose(1, 2)
    if m is not None:
        y = y.masked_fill(~m, 0.0)
    for j in (0, 2):
        y = F.conv1d(y, W[f"input_embed.conv_pos_embed.conv1d.{j}.weight"],
                     W[f"input_embed.conv_pos_embed.conv1d.{j}.bias"], padding=15, groups=16)
        if m is not None:
            y = y.masked_fill(~m, 0.0)
        y = F.mish(y)
    return y.transpose(1, 2)


def input_embed(W, x, cond, text_e, drop_audio, mask):
    if drop_audio:
        cond = torch.zeros_like(cond)
    h = F.linear(torch.cat((x, cond, text_e), -1), W["input_embed.proj.weight"], W["input_embed.proj.bias"])
    return conv_pos(W, h, mask) + h


def rope_cos_sin(n, dh=64):
    inv = 1.0 / (10000 ** (torch.arange(0, dh, 2).float() / dh))
    f = torch.arange(n).float()[:, None] * inv[None, :]
    f = torch.stack((f, f), -1).flatten(-2)  # interleaved (d r)
    return f.cos(), f.sin()


def apply_rope(t, cos, sin):
    """t·cos + rotate_half(t)·sin with rotate_half on interleaved pairs (a,b)->(-b,a)."""
    a, b = t[..., 0::2], t[..., 1::2]
    rot = torch.stack((-b, a), -1).flatten(-2)
    return (t.float() * cos + rot.float() * sin).to(t.dtype)


def attention(W, p, arch, x, mask, rope):
    S, N, _ = x.shape
    H, Dh = arch["heads"], arch["dim_head"]
    q = F.linear(x, W[p + "to_q.weight"], W[p + "to_q.bias"]).view(S, N, H, Dh).transpose(1, 2)
    k = F.linear(x, W[p + "to_k.weight"], W[p + "to_k.bias"]).view(S, N, H, Dh).transpose(1, 2)
    v = F.linear(x, W[p + "to_v.weight"], W[p + "to_v.bias"]).view(S, N, H, Dh).transpose(1, 2)
    cos, sin = rope
    pn = arch["pe_attn_head"]
    if pn is None:
        q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
    else:
        q = torch.cat((apply_rope(q[:, :pn], cos, sin), q[:, pn:]), 1)
        k = torch.cat((apply_rope(k[:, :pn], cos, sin), k[:, pn:]), 1)
    am = None
    if arch["attn_mask_enabled"] and mask is not None:
        am = mask[:, None, None, :].expand(S, H, N, N)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=am)
    o = o.transpose(1, 2).reshape(S, N, H * Dh)
    o = F.linear(o, W[p + "to_out.0.weight"], W[p + "to_out.0.bias"])
    if mask is not None:
        o = o.masked_fill(~mask[..., None], 0.0)
    return o


def ffn(W, p, x):
    h = F.gelu(F.linear(x, W[p + "ff.0.0.weight"], W[p + "ff.0.0.bias"]), approximate="tanh")
    return F.linear(h, W[p + "ff.2.weight"], W[p + "ff.2.bias"])


def ln(x):
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6)


def dit_block(W, i, arch, x, t_emb, mask, rope):
    p = f"transformer_blocks.{i}."
    e = F.linear(F.silu(t_emb), W[p + "attn_norm.linear.weight"], W[p + "attn_norm.linear.bias"])
    sh1, sc1, g1, sh2, sc2, g2 = torch.chunk(e, 6, dim=1)
    a = ln(x) * (1 + sc1[:, None]) + sh1[:, None]
    x = x + g1[:, None] * attention(W, p + "attn.", arch, a, mask, rope)
    f = ln(x) * (1 + sc2[:, None]) + sh2[:, None]
    return x + g2[:, None] * ffn(W, p + "ff.", f)


def dit_forward(W, arch, x, cond, text, t, mask, text_cache, packed=True, drop_audio=False, drop_text=False):
    """Packed cond/uncond DiT forward (cfg_infer=True, cache=True). Returns [2b,n,mel].
    `packed=False`: one branch (dit.py:347-350) honouring drop_audio / drop_text -> [b,n,mel]
    (the forward of `cfm.py:167-178` is the one with both flags False)."""
    b, n = x.shape[:2]
    t = t.reshape(-1).expand(b) if t.numel() == 1 else t
    te = time_embed(W, t)
    if "cond" not in text_cache:
        seq = n if mask is None else mask.sum(1)
        text_cache["cond"] = text_embed_dit(W, arch, text, seq, False)
        text_cache["uncond"] = text_embed_dit(W, arch, text, seq, True)
    if packed:
        xc = input_embed(W, x, cond, text_cache["cond"], False, mask)
        xu = input_embed(W, x, cond, text_cache["uncond"], True, mask)
        h = torch.cat((xc, xu), 0)
        te = torch.cat((te, te), 0)
        m2 = None if mask is None else torch.cat((mask, mask), 0)
    else:
        h = input_embed(W, x, cond, text_cache["uncond" if drop_text else "cond"], drop_audio, mask)
        m2 = mask
    rope = rope_cos_sin(n, arch["dim_head"])
    for i in range(arch["depth"]):
        h = dit_block(W, i, arch, h, te, m2, rope)
    e = F.linear(F.silu(te), W["norm_out.linear.weight"], W["norm_out.linear.bias"])
    sc, sh = torch.chunk(e, 2, dim=1)  # scale first (modules.py:343)
    h = ln(h) * (1 + sc[:, None]) + sh[:, None]
    return F.linear(h, W["proj_out.weight"], W["proj_out.bias"])


# ------------------------------------------------------------------ UNetT (E2)

def rms_norm(x, g):
    return F.normalize(x, dim=-1) * (x.shape[-1] ** 0.5) * g


def text_embed_unett(W, arch, text, n, drop_text):
    text = text + 1
    text = text[:, :n]
    text = F.pad(text, (0, n - text.shape[1]), value=0)
    if drop_text:
        text = torch.zeros_like(text)
    return W["text_embed.text_embed.weight"][text]  # conv_layers=0 for E2 Base


def unett_forward(W, arch, x, cond, text, t, mask, text_cache, packed=True, drop_audio=False, drop_text=False):
    b, n = x.shape[:2]
    t = t.reshape(-1).expand(b) if t.numel() == 1 else t
    te = time_embed(W, t)
    if "cond" not in text_cache:
        text_cache["cond"] = text_embed_unett(W, arch, text, n, False)
        text_cache["uncond"] = text_embed_unett(W, arch, text, n, True)
    if packed:  # InputEmbedding takes no mask (unett.py:90-102)
        xc = input_embed(W, x, cond, text_cache["cond"], False, None)
        xu = input_embed(W, x, cond, text_cache["uncond"], True, None)
        h = torch.cat((xc, xu), 0)
        te = torch.cat((te, te), 0)
        m2 = None if mask is None else torch.cat((mask, mask), 0)
    else:
        h = input_embed(W, x, cond, text_cache["uncond" if drop_text else "cond"], drop_audio, None)
        m2 = mask
    h = torch.cat((te[:, None], h), 1)
    if m2 is not None:
        m2 = F.pad(m2, (1, 0), value=True)
    rope = rope_cos_sin(n + 1, arch["dim_head"])
    depth = arch["depth"]
    skips = []
    for i in range(depth):
        p = f"layers.{i}."
        if i < depth // 2:
            skips.append(h)
        else:
            h = F.linear(torch.cat((h, skips.pop()), -1), W[p + "0.weight"])
        h = attention(W, p + "2.", arch, rms_norm(h, W[p + "1.g"]), m2, rope) + h
        h = ffn(W, p + "4.", rms_norm(h, W[p + "3.g"])) + h
    h = rms_norm(h, W["norm_out.g"])[:, 1:]
    return F.linear(h, W["proj_out.weight"], W["proj_out.bias"])


# ------------------------------------------------------------------ sampler

def prepare(arch, cond, text, duration, lens=None, max_duration=65536, edit_mask=None, no_ref_audio=False):
    """The host-side preamble of CFM.sample (cfm.py:111-158). Returns a dict."""
    B, cond_len = cond.shape[:2]
    if lens is None:
        lens = torch.full((B,), cond_len, dtype=torch.long)
    cond_mask = lens_to_mask(lens)
    if edit_mask is not None:
        cond_mask = cond_mask & edit_mask
    if isinstance(duration, int):
        duration = torch.full((B,), duration, dtype=torch.long)
    duration = torch.maximum(torch.maximum((text != -1).sum(-1), lens) + 1, duration)
    duration = duration.clamp(max=max_duration)
    N = int(duration.max())
    cond = F.pad(cond, (0, 0, 0, N - cond_len), value=0.0)
    if no_ref_audio:  # cfm.py:146-147
        cond = torch.zeros_like(cond)
    cond_mask = F.pad(cond_mask, (0, N - cond_mask.shape[-1]), value=False)[..., None]
    step_cond = torch.where(cond_mask, cond, torch.zeros_like(cond))
    mask = lens_to_mask(duration) if B > 1 else None
    return dict(cond=cond, cond_mask=cond_mask, step_cond=step_cond, mask=mask, duration=duration, N=N)


@torch.no_grad()
def cfm_sample(W, arch, cond, text, duration, *, lens=None, steps=32, cfg_strength=1.0,
               sway_sampling_coef=None, y0=None, seed=None, use_epss=True, edit_mask=None,
               max_steps=None, no_ref_audio=False, duplicate_test=False, t_inter=0.1):
    """fp32 restatement of CFM.sample. `y0` overrides the noise recipe (cfm.py:196-201).
    `max_steps` truncates the Euler loop (used only for bounded CPU-baseline timing).
    duplicate_test (cfm.py:141-143, 205-209): start at t_inter from a mix of the noise and the prompt
    shifted by its own length, over int(steps * (1 - t_inter)) linspace steps."""
    cond_len = cond.shape[1]
    pre = prepare(arch, cond.float(), text, duration, lens, edit_mask=edit_mask, no_ref_audio=no_ref_audio)
    if y0 is None:
        from torch.nn.utils.rnn import pad_sequence
        ys = []
        for d in pre["duration"]:
            if seed is not None:
                torch.manual_seed(seed)
            ys.append(torch.randn(int(d), cond.shape[-1]))
        y0 = pad_sequence(ys, padding_value=0, batch_first=True)
    fwd = dit_forward if arch["backbone"] == "DiT" else unett_forward
    cache = {}

    def fn(t, x):
        if cfg_strength < 1e-5:  # cfm.py:167-178: one conditional forward, no guidance
            return fwd(W, arch, x, pre["step_cond"], text, t, pre["mask"], cache, packed=False)
        p = fwd(W, arch, x, pre["step_cond"], text, t, pre["mask"], cache)
        pc, pu = torch.chunk(p, 2, 0)
        return pc + (pc - pu) * cfg_strength

    t_start = 0.0
    if duplicate_test:
        test_cond = F.pad(cond.float(), (0, 0, cond_len, pre["N"] - 2 * cond_len), value=0.0)
        t_start = t_inter
        y0 = (1 - t_start) * y0.float() + t_start * test_cond
        steps = int(steps * (1 - t_start))
    t = epss_sway_grid(steps, sway_sampling_coef, use_epss, t_start=t_start)
    y = y0.float()
    traj = [y]
    n_run = steps if max_steps is None else min(steps, max_steps)
    for k in range(n_run):
        y = y + (t[k + 1] - t[k]) * fn(t[k], y)
        traj.append(y)
    out = torch.where(pre["cond_mask"], pre["cond"], y)
    return out, torch.stack(traj)
