"""Common machinery of the engine-backed backbone plugins (DiT, UNetT).

Contract kept from the reference (SURVEY §1 "Public interface of L2"):
  * `__init__(**arch, text_num_embeds, mel_dim)`       utils_infer.py:258
  * `.dim`                                             cfm.py:67
  * `forward(x, cond, text, time, mask, drop_audio_cond, drop_text, cfg_infer, cache)`  dit.py:319-330
  * `clear_cache()`                                    dit.py:316-317 (no-op: the engine keeps no
    cross-call state, so the reference's thread-local text cache, dit.py:237-262, is not needed)
"""

from __future__ import annotations

import threading

import torch
from torch import nn

from ... import configs
from ._params import build_param_tree, rotary_inv_freq


class EngineBackbone(nn.Module):
    backbone_name = "DiT"

    def _setup(self, arch: dict):
        self.arch = configs.get_arch(arch)
        self.dim = self.arch["dim"]
        self.depth = self.arch["depth"]
        build_param_tree(self, configs.param_shapes(self.arch))
        # persistent buffer of x_transformers.RotaryEmbedding (present in reference checkpoints)
        rot = nn.Module()
        rot.register_buffer("inv_freq", rotary_inv_freq(self.arch["dim_head"]))
        self.add_module("rotary_embed", rot)
        self.__dict__["_engines"] = {}
        self.__dict__["_engine_lock"] = threading.Lock()

    # ------------------------------------------------------------------ engine cache
    def _weights_version(self):
        return tuple(p._version for p in self.parameters()) + (id(self),)

    def engine_weights(self) -> dict:
        return {k: v for k, v in self.state_dict().items() if not k.endswith("inv_freq")}

    def get_engine(self, compute: str, device):
        """The packed HIP engine for this backbone's current weights (rebuilt if they changed)."""
        from ...engine import Engine

        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("the f5h engine runs on a ROCm GPU (cuda:N); got device " + str(device))
        key = (compute, device.index if device.index is not None else torch.cuda.current_device())
        ver = self._weights_version()
        with self._engine_lock:
            hit = self._engines.get(key)
            if hit is not None and hit[0] == ver:
                return hit[1]
            eng = Engine(self.arch, self.engine_weights(), compute=compute, device=torch.device("cuda", key[1]))
            self._engines[key] = (ver, eng)
            return eng

    def __deepcopy__(self, memo):  # EMA-style deepcopy stays possible (cf. dit.py:237-238)
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        import copy

        for k, v in self.__dict__.items():
            if k in ("_engines", "_engine_lock"):
                continue
            new.__dict__[k] = copy.deepcopy(v, memo)
        new.__dict__["_engines"] = {}
        new.__dict__["_engine_lock"] = threading.Lock()
        return new

    def clear_cache(self):
        pass

    # ------------------------------------------------------------------ plugin forward
    def forward(self, x, cond, text, time, mask=None, drop_audio_cond=False, drop_text=False, cfg_infer=False,
                cache=False, compute: str | None = None):
        """Packed cond/uncond forward through the engine (the path CFM.sample uses, cfm.py:181-191).
        `cond` must already be the masked step_cond; returns [2B, N, mel]."""
        if not cfg_infer:
            raise NotImplementedError("engine backbones implement the packed CFG forward (cfg_infer=True); "
                                      "single-branch sampling runs inside CFM.sample")
        B, N = x.shape[:2]
        if torch.is_tensor(time) and time.numel() > 1:
            if not bool((time == time.reshape(-1)[0]).all()):
                raise NotImplementedError("per-sample time values are not used by CFM.sample")
        t = float(time.reshape(-1)[0]) if torch.is_tensor(time) else float(time)
        compute = compute or ("fp32" if next(self.parameters()).dtype == torch.float32 else "bf16")
        eng = self.get_engine(compute, x.device)
        dur = mask.sum(1) if mask is not None else torch.full((B,), N, device=x.device)
        ones = torch.ones(B, N, dtype=torch.uint8, device=x.device)
        pred = eng.forward(x, cond, ones, text, dur, t, use_batch_mask=mask is not None)
        return pred.to(x.dtype)
