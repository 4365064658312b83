from .backbones.dit import DiT
from .backbones.unett import UNetT
from .cfm import CFM

__all__ = ["CFM", "DiT", "UNetT"]
