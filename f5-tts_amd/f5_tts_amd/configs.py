"""Model architecture presets for the CFM sampling engine.

The hyper-parameters mirror the reference's Hydra configs
(`src/f5_tts/configs/F5TTS_v1_Base.yaml:24-37`, `F5TTS_v1_Small.yaml:24-37`,
`F5TTS_Base.yaml:24-35`, `E2TTS_Base.yaml:24-31`) and the constructor defaults of
`DiT.__init__` (`src/f5_tts/model/backbones/dit.py:171-192`) and
`UNetT.__init__` (`src/f5_tts/model/backbones/unett.py:108-129`).

Only the keys that change the arithmetic of `CFM.sample()` are kept; the
training/Hydra keys (dropout, checkpoint_activations, attn_backend) have no
effect on inference numerics.
"""

from __future__ import annotations

import copy

# vocab.txt in the reference has 2545 entries -> text_num_embeds=2545
VOCAB_SIZE = 2545
MEL_DIM = 100

_DIT_DEFAULTS = dict(
    backbone="DiT",
    dim=1024,
    depth=22,
    heads=16,
    dim_head=64,
    ff_mult=2,
    text_dim=512,
    text_mask_padding=True,
    conv_layers=4,
    pe_attn_head=None,
    attn_mask_enabled=False,
    qk_norm=None,
    long_skip_connection=False,
    text_embedding_average_upsampling=False,
)

_UNETT_DEFAULTS = dict(
    backbone="UNetT",
    dim=1024,
    depth=24,
    heads=16,
    dim_head=64,
    ff_mult=4,
    text_dim=None,  # -> mel_dim (unett.py:131-132)
    text_mask_padding=False,
    conv_layers=0,
    pe_attn_head=1,
    attn_mask_enabled=False,
    qk_norm=None,
    skip_connect_type="concat",
)

PRESETS = {
    # F5TTS_v1_Base.yaml:24-37
    "F5TTS_v1_Base": dict(_DIT_DEFAULTS),
    # F5TTS_v1_Small.yaml:24-37
    "F5TTS_v1_Small": dict(_DIT_DEFAULTS, dim=768, depth=18, heads=12),
    # the v1 Small architecture with depth overridden to 4 (not a shipped config)
    "F5TTS_v1_Small_4L": dict(_DIT_DEFAULTS, dim=768, depth=4, heads=12),
    # F5TTS_Base.yaml:24-35 (v0: no text mask padding, rope on head 0 only)
    "F5TTS_Base": dict(_DIT_DEFAULTS, text_mask_padding=False, pe_attn_head=1),
    # E2TTS_Base.yaml:24-31
    "E2TTS_Base": dict(_UNETT_DEFAULTS),
    # tiny configs used for golden vectors / quick parity (head dim stays 64: the engine's attention is Dh=64)
    "DiT_tiny": dict(_DIT_DEFAULTS, dim=128, depth=2, heads=2, text_dim=64, conv_layers=1),
    "UNetT_tiny": dict(_UNETT_DEFAULTS, dim=128, depth=4, heads=2),
}


def get_arch(name_or_arch, **overrides) -> dict:
    """Return a full arch dict (preset name or partial dict) with overrides applied."""
    if isinstance(name_or_arch, str):
        if name_or_arch not in PRESETS:
            raise KeyError(f"unknown preset {name_or_arch!r}; known: {sorted(PRESETS)}")
        arch = copy.deepcopy(PRESETS[name_or_arch])
    else:
        base = _UNETT_DEFAULTS if name_or_arch.get("backbone", "DiT") == "UNetT" else _DIT_DEFAULTS
        arch = dict(base)
        arch.update(name_or_arch)
    arch.update(overrides)
    arch.setdefault("text_num_embeds", VOCAB_SIZE)
    arch.setdefault("mel_dim", MEL_DIM)
    if arch.get("text_dim") is None:
        arch["text_dim"] = arch["mel_dim"]
    return arch


def param_shapes(arch: dict) -> "dict[str, tuple]":
    """Ordered parameter names/shapes, using the reference's state-dict names
    (without the `transformer.` prefix that `CFM` adds).

    Names follow `dit.py:145-226`, `modules.py:175-201,252-280,312-364,371-441,711-757,852-862`
    and `unett.py:37-183`; the TRT converter's key map (`convert_checkpoint.py:129-145`)
    enumerates the same keys for the DiT.
    """
    d = arch["dim"]
    H, Dh = arch["heads"], arch["dim_head"]
    inner = H * Dh
    F = int(d * arch["ff_mult"])
    mel = arch["mel_dim"]
    td = arch["text_dim"]
    V = arch["text_num_embeds"] + 1
    s = {}
    s["time_embed.time_mlp.0.weight"] = (d, 256)
    s["time_embed.time_mlp.0.bias"] = (d,)
    s["time_embed.time_mlp.2.weight"] = (d, d)
    s["time_embed.time_mlp.2.bias"] = (d,)
    s["text_embed.text_embed.weight"] = (V, td)
    for i in range(arch["conv_layers"]):
        p = f"text_embed.text_blocks.{i}."
        s[p + "dwconv.weight"] = (td, 1, 7)
        s[p + "dwconv.bias"] = (td,)
        s[p + "norm.weight"] = (td,)
        s[p + "norm.bias"] = (td,)
        s[p + "pwconv1.weight"] = (2 * td, td)
        s[p + "pwconv1.bias"] = (2 * td,)
        s[p + "grn.gamma"] = (1, 1, 2 * td)
        s[p + "grn.beta"] = (1, 1, 2 * td)
        s[p + "pwconv2.weight"] = (td, 2 * td)
        s[p + "pwconv2.bias"] = (td,)
    s["input_embed.proj.weight"] = (d, 2 * mel + td)
    s["input_embed.proj.bias"] = (d,)
    for j in (0, 2):
        s[f"input_embed.conv_pos_embed.conv1d.{j}.weight"] = (d, d // 16, 31)
        s[f"input_embed.conv_pos_embed.conv1d.{j}.bias"] = (d,)

    def attn(p):
        for n in ("to_q", "to_k", "to_v"):
            s[p + f"{n}.weight"] = (inner, d)
            s[p + f"{n}.bias"] = (inner,)
        s[p + "to_out.0.weight"] = (d, inner)
        s[p + "to_out.0.bias"] = (d,)

    def ff(p):
        s[p + "ff.0.0.weight"] = (F, d)
        s[p + "ff.0.0.bias"] = (F,)
        s[p + "ff.2.weight"] = (d, F)
        s[p + "ff.2.bias"] = (d,)

    if arch["backbone"] == "DiT":
        for i in range(arch["depth"]):
            p = f"transformer_blocks.{i}."
            s[p + "attn_norm.linear.weight"] = (6 * d, d)
            s[p + "attn_norm.linear.bias"] = (6 * d,)
            attn(p + "attn.")
            ff(p + "ff.")
        s["norm_out.linear.weight"] = (2 * d, d)
        s["norm_out.linear.bias"] = (2 * d,)
    elif arch["backbone"] == "UNetT":
        for i in range(arch["depth"]):
            p = f"layers.{i}."
            if i >= arch["depth"] // 2:
                s[p + "0.weight"] = (d, 2 * d)  # skip_proj, no bias (unett.py:174)
            s[p + "1.g"] = (d,)  # x_transformers RMSNorm gain
            attn(p + "2.")
            s[p + "3.g"] = (d,)
            ff(p + "4.")
        s["norm_out.g"] = (d,)
    else:
        raise ValueError(f"unsupported backbone {arch['backbone']!r}")
    s["proj_out.weight"] = (mel, d)
    s["proj_out.bias"] = (mel,)
    return s
