"""E2-TTS flat-UNet transformer backbone plugin (engine-backed).

Same constructor signature and state-dict names as the reference UNetT
(`src/f5_tts/model/backbones/unett.py:108-183`): time token prepended, RMSNorm
(x_transformers, gain `g`), concat skips + bias-free Linear, GELU-tanh FFN.
"""

from __future__ import annotations

from .base import EngineBackbone


class UNetT(EngineBackbone):
    backbone_name = "UNetT"

    def __init__(self, *, dim, depth=8, heads=8, dim_head=64, dropout=0.1, ff_mult=4, mel_dim=100,
                 text_num_embeds=256, text_dim=None, text_mask_padding=True, qk_norm=None, conv_layers=0,
                 pe_attn_head=None, attn_backend="torch", attn_mask_enabled=False, skip_connect_type="concat"):
        super().__init__()
        del dropout, attn_backend
        if skip_connect_type != "concat":
            raise NotImplementedError("only the default concat skips (unett.py:129) are implemented")
        if conv_layers:
            raise NotImplementedError("UNetT text ConvNeXt blocks are not used by E2TTS_Base (conv_layers 0)")
        self._setup(dict(
            backbone="UNetT", dim=dim, depth=depth, heads=heads, dim_head=dim_head, ff_mult=ff_mult, mel_dim=mel_dim,
            text_num_embeds=text_num_embeds, text_dim=text_dim if text_dim is not None else mel_dim,
            text_mask_padding=text_mask_padding, qk_norm=qk_norm, conv_layers=0, pe_attn_head=pe_attn_head,
            attn_mask_enabled=attn_mask_enabled, skip_connect_type="concat",
        ))
