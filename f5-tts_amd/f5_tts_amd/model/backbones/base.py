"""Common machinery of the engine-backed backbone plugins (DiT, UNetT).

Contract kept from the reference (SURVEY §1 "Public interface of L2"):
  * `__init__(**arch, text_num_embeds, mel_dim)`       utils_infer.py:258
  * `.dim`                                             cfm.py:67
  * `forward(x, cond, text, time, mask, drop_audio_cond, drop_text, cfg_infer, cache)`  dit.py:319-330
  * `clear_cache()`                                    dit.py:316-317
  * `forward(..., cache=True)` keeps the text embedding of the first call in a per-thread session
    workspace (the reference's thread-local text_cond / text_uncond cache, dit.py:237-262, 294-317)
    and reuses it until `clear_cache()`; the backbone step of a session replays as a hipGraph
"""

from __future__ import annotations

import threading

import torch
from torch import nn

from ... import configs
from ._params import build_param_tree, rotary_inv_freq


def compute_for_dtype(dtype: torch.dtype) -> str:
    """Engine compute mode for a parameter dtype: fp32 -> exact-f32 parity mode, fp16 -> fp16 MFMA
    operands (the reference's GPU default, utils_infer.py:190-199), bf16 -> bf16 MFMA operands."""
    if dtype == torch.float16:
        return "fp16"
    if dtype == torch.bfloat16:
        return "bf16"
    return "fp32"


# bumped whenever any module in the process registers a submodule (torch's global registration hook)
_STRUCT_GEN = [0]


def _bump_struct_gen(module, name, submodule):
    _STRUCT_GEN[0] += 1


torch.nn.modules.module.register_module_module_registration_hook(_bump_struct_gen)


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
        self.__dict__["_tls"] = threading.local()

    # ------------------------------------------------------------------ engine cache
    def _weights_version(self):
        # _version misses writes through .data (p.data.copy_); the storage pointer and dtype catch
        # re-assigned / re-cast parameters, so a stale packed engine is never reused. The module list
        # is cached (walking the ~300-module tree per call cost ~1 ms of host time) and rebuilt when
        # any module registers a submodule; each module's own parameter dict is read every call, so a
        # replaced Parameter object is seen too.
        mods = self.__dict__.get("_mods")
        if mods is None or mods[0] != _STRUCT_GEN[0]:
            mods = (_STRUCT_GEN[0], tuple(self.modules()))
            self.__dict__["_mods"] = mods
        return tuple((p._version, p.data_ptr(), p.dtype) for m in mods[1] for p in m._parameters.values()
                     if p is not None) + (id(self),)

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
            if k in ("_engines", "_engine_lock", "_mods", "_tls"):
                continue
            new.__dict__[k] = copy.deepcopy(v, memo)
        new.__dict__.pop("_mods", None)
        new.__dict__["_engines"] = {}
        new.__dict__["_engine_lock"] = threading.Lock()
        new.__dict__["_tls"] = threading.local()
        return new

    # kept text-embedding sessions per thread (LRU); the reference keeps one (dit.py:294-317)
    MAX_SESSIONS = 2

    def _sessions(self) -> dict:
        tls = self.__dict__["_tls"]
        if not hasattr(tls, "sessions"):
            tls.sessions = {}
        return tls.sessions

    def clear_cache(self):
        """Drop this thread's kept text embeddings (dit.py:316-317)."""
        self._sessions().clear()

    # ------------------------------------------------------------------ plugin forward
    def forward(self, x, cond, text, time, mask=None, drop_audio_cond=False, drop_text=False, cfg_infer=False,
                cache=False, compute: str | None = None):
        """DiT.forward / UNetT.forward through the engine (dit.py:319-370, unett.py:244-307).

        cfg_infer=True: the packed cond/uncond forward of CFM.sample (cfm.py:181-191) -> [2B, N, mel];
        cfg_infer=False: one branch (cfm.py:167-178) -> [B, N, mel], honouring drop_audio_cond and
        drop_text. `cond` is the already-masked step_cond; `time` a scalar or one value per sample
        (dit.py:332-333 repeats a scalar; distinct values run as groups of equal t, which is exact
        because sequences of equal padded length N are independent in the backbone). A scalar device
        `time` is read on the stream (no host sync). `cache=True`: the first call of this thread's
        session computes the text embedding (both branches) and keeps it, later calls reuse it until
        clear_cache(), as dit.py:294-317 does; sessions are keyed by shape, the MAX_SESSIONS most recently
        used per thread are kept."""
        B, N = x.shape[:2]
        compute = compute or compute_for_dtype(next(self.parameters()).dtype)
        eng = self.get_engine(compute, x.device)
        dur = mask.sum(1) if mask is not None else torch.full((B,), N, device=x.device)
        ones = torch.ones(B, N, dtype=torch.uint8, device=x.device)
        use_mask = mask is not None
        flags = dict(cfg_infer=cfg_infer, drop_audio_cond=drop_audio_cond, drop_text=drop_text)
        if not torch.is_tensor(time) or time.numel() == 1:
            tval = time if torch.is_tensor(time) else float(time)
            text_cache, ws = 0, None
            if cache:
                key = (compute, eng.device.index, B, N, text.shape[1], bool(cfg_infer), use_mask)
                sess = self._sessions()
                ws = sess.pop(key, None)
                text_cache = 2 if ws is not None else 1
                if ws is None:
                    ws = eng.forward_workspace(B, N, text.shape[1], cfg_infer)
                sess[key] = ws  # most recently used last
                while len(sess) > self.MAX_SESSIONS:  # bounded: a forward workspace can be hundreds of MB
                    sess.pop(next(iter(sess)))
            pred = eng.forward(x, cond, ones, text, dur, tval, use_mask, text_cache=text_cache, workspace=ws, **flags)
            return pred.to(x.dtype)
        tv = time.reshape(-1).float().cpu()
        if tv.numel() != B:
            raise ValueError(f"time must be a scalar or have one value per sample ({B}), got {tv.numel()}")
        values = torch.unique(tv)
        if values.numel() == 1:
            pred = eng.forward(x, cond, ones, text, dur, float(values[0]), use_mask, **flags)
            return pred.to(x.dtype)
        S = 2 * B if cfg_infer else B
        pred = torch.empty(S, N, x.shape[2], dtype=torch.float32, device=x.device)
        for v in values.tolist():
            idx = torch.nonzero(tv == v).flatten().to(x.device)
            p = eng.forward(x[idx], cond[idx], ones[idx], text[idx], dur[idx], v, use_mask, **flags)
            nb = idx.numel()
            pred[idx] = p[:nb]
            if cfg_infer:
                pred[idx + B] = p[nb:]
        return pred.to(x.dtype)
