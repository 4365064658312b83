"""Parameter-tree construction shared by the backbone plugins.

The backbones are weight containers whose state-dict names equal the reference's
(so reference checkpoints load unchanged, `utils_infer.py:190-232`); the arithmetic
lives in the HIP engine. The tree is generated from `configs.param_shapes`, the single
source of truth for names and shapes.
"""

from __future__ import annotations

import torch
from torch import nn


def build_param_tree(root: nn.Module, shapes: dict, dtype=torch.float32):
    for name, shape in shapes.items():
        parts = name.split(".")
        mod = root
        for p in parts[:-1]:
            child = mod._modules.get(p)
            if child is None:
                child = nn.Module()
                mod.add_module(p, child)
            mod = child
        mod.register_parameter(parts[-1], nn.Parameter(torch.zeros(shape, dtype=dtype)))


def rotary_inv_freq(dim_head: int) -> torch.Tensor:
    # x_transformers RotaryEmbedding keeps inv_freq as a persistent buffer; real checkpoints carry it
    return 1.0 / (10000 ** (torch.arange(0, dim_head, 2).float() / dim_head))
