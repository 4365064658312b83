"""F5-TTS DiT backbone plugin (engine-backed).

Same constructor signature and state-dict names as the reference DiT
(`src/f5_tts/model/backbones/dit.py:170-226`); the forward pass is the HIP engine
(ConvNeXt-V2 text embed, conv position embedding, AdaLN-Zero DiT blocks with RoPE
attention and GELU-tanh FFN, final AdaLN + projection).
"""

from __future__ import annotations

from .base import EngineBackbone


class DiT(EngineBackbone):
    backbone_name = "DiT"

    def __init__(self, *, dim, depth=8, heads=8, dim_head=64, dropout=0.1, ff_mult=4, mel_dim=100,
                 text_num_embeds=256, text_dim=None, text_mask_padding=True, text_embedding_average_upsampling=False,
                 qk_norm=None, conv_layers=0, pe_attn_head=None, attn_backend="torch", attn_mask_enabled=False,
                 long_skip_connection=False, checkpoint_activations=False):
        super().__init__()
        del dropout, attn_backend, checkpoint_activations  # no effect on inference arithmetic
        self._setup(dict(
            backbone="DiT", dim=dim, depth=depth, heads=heads, dim_head=dim_head, ff_mult=ff_mult, mel_dim=mel_dim,
            text_num_embeds=text_num_embeds, text_dim=text_dim if text_dim is not None else mel_dim,
            text_mask_padding=text_mask_padding, text_embedding_average_upsampling=text_embedding_average_upsampling,
            qk_norm=qk_norm, conv_layers=conv_layers, pe_attn_head=pe_attn_head,
            attn_mask_enabled=attn_mask_enabled, long_skip_connection=long_skip_connection,
        ))
