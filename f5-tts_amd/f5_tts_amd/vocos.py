"""Host mirror of vocos' `Vocos` decoder on the HIP engine.

The reference decodes generated mels with `vocoder.decode(mel)` (src/f5_tts/infer/utils_infer.py:
506-511; runtime/triton_trtllm/benchmark.py:432-435), `vocoder` being vocos' mel-24khz model
loaded by `load_vocoder` (utils_infer.py:106-128: `Vocos.from_hparams` + `load_state_dict` of the
checkpoint). This class keeps that surface: construct, `load_state_dict(state_dict)` with vocos'
parameter names (feature-extractor buffers are ignored, as they are not on the decode path),
`.to(device)` / `.eval()`, and `decode(features_input)` mapping mel [B, 100, T] fp32 to audio
[B, (T - 1) * 256] (torch.istft center=True length). The work runs in libf5h.so
(`f5h_vocos_decode`, include/f5h.h); there is no PyTorch fallback.
"""

from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib

VOCOS_MEL_24KHZ = dict(input_channels=100, dim=512, intermediate_dim=1536, num_layers=8, n_fft=1024, hop_length=256)


class Vocos:
    def __init__(self, input_channels=100, dim=512, intermediate_dim=1536, num_layers=8, n_fft=1024,
                 hop_length=256, compute: str = "fp32"):
        self.arch = dict(input_channels=input_channels, dim=dim, intermediate_dim=intermediate_dim,
                         num_layers=num_layers, n_fft=n_fft, hop_length=hop_length)
        if compute not in ("fp32", "bf16"):
            raise ValueError("compute must be 'fp32' or 'bf16'")
        self.compute = compute
        self.device = torch.device("cpu")
        self._state = None
        self._h = None
        self._lock = threading.Lock()
        self._create_lock = threading.Lock()
        self._ws = {}

    # ------------------------------------------------------------------ nn.Module-like surface
    def load_state_dict(self, state_dict, strict: bool = True):
        sd = {k: v for k, v in state_dict.items() if not k.startswith("feature_extractor.")
              and not k.startswith("head.istft.")}
        self._state = {k: (v.detach().to("cpu", torch.float32).contiguous().numpy() if isinstance(v, torch.Tensor)
                           else np.ascontiguousarray(v, dtype=np.float32)) for k, v in sd.items()}
        self._destroy()
        return self

    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("the HIP Vocos runs on a GPU device")
        if device != self.device:
            self._destroy()
        self.device = torch.device("cuda", device.index if device.index is not None else torch.cuda.current_device())
        return self

    def eval(self):
        return self

    def _engine(self):
        # decode() is called from the reference's thread pool (utils_infer.py:540-547): create the engine
        # under a lock so concurrent first calls build (and upload weights for) exactly one
        with self._create_lock:
            return self._engine_locked()

    def _engine_locked(self):
        if self._h is not None:
            return self._h
        if self._state is None:
            raise RuntimeError("Vocos: load_state_dict() first")
        if self.device.type != "cuda":
            raise RuntimeError("Vocos: call .to('cuda:N') first")
        L = _lib.lib()
        names = [k.encode() for k in self._state]
        arr = (_lib.Weight * len(self._state))()
        for i, (k, v) in enumerate(self._state.items()):
            arr[i].name = names[i]
            arr[i].data = v.ctypes.data
            arr[i].numel = v.size
        a = _lib.VocosArch(*[self.arch[k] for k in ("input_channels", "dim", "intermediate_dim", "num_layers",
                                                    "n_fft", "hop_length")],
                           _lib.F5H_BF16 if self.compute == "bf16" else _lib.F5H_FP32)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.f5h_vocos_create(ctypes.byref(a), arr, len(self._state), self.device.index, ctypes.byref(h)),
                       "f5h_vocos_create")
        self._h = h
        return h

    def _destroy(self):
        if self._h is not None and self._h.value:
            try:
                _lib.lib().f5h_vocos_destroy(self._h)
            except Exception:
                pass
        self._h = None
        self._ws = {}

    def __del__(self):
        self._destroy()

    # ------------------------------------------------------------------ decode
    def decode(self, features_input: torch.Tensor) -> torch.Tensor:
        """mel [B, C, T] (or [C, T]) -> audio [B, (T-1)*hop] fp32 on this device."""
        mel = features_input
        if mel.dim() == 2:
            mel = mel[None]
        B, C, T = mel.shape
        if C != self.arch["input_channels"]:
            raise ValueError(f"expected {self.arch['input_channels']} mel channels, got {C}")
        h = self._engine()
        mel = mel.to(self.device, torch.float32).contiguous()
        audio = torch.empty(B, (T - 1) * self.arch["hop_length"], dtype=torch.float32, device=self.device)
        L = _lib.lib()
        need = int(L.f5h_vocos_workspace_size(h, B, T))
        stream = _lib.stream_handle(self.device)
        with self._lock:
            ws = self._ws.get((stream, need))
            if ws is None:
                ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
                self._ws = {(stream, need): ws}
            with torch.cuda.device(self.device):
                _lib.check(L.f5h_vocos_decode(h, stream, B, T, mel.data_ptr(), audio.data_ptr(), ws.data_ptr(),
                                              ws.numel()), "f5h_vocos_decode")
        return audio

    __call__ = decode


def param_shapes(arch: dict = VOCOS_MEL_24KHZ) -> "dict[str, tuple]":
    """vocos state-dict names/shapes on the decode path (backbone + head)."""
    C, d, I, nf = arch["input_channels"], arch["dim"], arch["intermediate_dim"], arch["n_fft"]
    s = {"backbone.embed.weight": (d, C, 7), "backbone.embed.bias": (d,),
         "backbone.norm.weight": (d,), "backbone.norm.bias": (d,)}
    for i in range(arch["num_layers"]):
        p = f"backbone.convnext.{i}."
        s.update({p + "dwconv.weight": (d, 1, 7), p + "dwconv.bias": (d,), p + "norm.weight": (d,),
                  p + "norm.bias": (d,), p + "pwconv1.weight": (I, d), p + "pwconv1.bias": (I,),
                  p + "pwconv2.weight": (d, I), p + "pwconv2.bias": (d,), p + "gamma": (d,)})
    s.update({"backbone.final_layer_norm.weight": (d,), "backbone.final_layer_norm.bias": (d,),
              "head.out.weight": (nf + 2, d), "head.out.bias": (nf + 2,)})
    return s


def make_weights(arch: dict = VOCOS_MEL_24KHZ, seed: int = 0) -> "dict[str, torch.Tensor]":
    """Synthetic vocos state dict from the hash PRNG (checkpoints are network-only): unit-variance
    linear/conv maps, norm gains around 1, layer scale gamma around 1/num_layers (vocos' default
    init), small biases."""
    import math

    from .synthetic import hash_uniform

    sq3 = math.sqrt(3.0)
    out = {}
    for name, shape in param_shapes(arch).items():
        n = int(np.prod(shape))
        if name.endswith("gamma"):
            off, a = 1.0 / max(1, arch["num_layers"]), 0.02 * sq3
        elif name.endswith("norm.weight") or name.endswith("final_layer_norm.weight"):
            off, a = 1.0, 0.1 * sq3
        elif len(shape) >= 2:
            off, a = 0.0, sq3 / math.sqrt(int(np.prod(shape[1:])))
        else:
            off, a = 0.0, 0.02 * sq3
        w = hash_uniform("vocos." + name, n, seed) * np.float32(a) + np.float32(off)
        out[name] = torch.from_numpy(w.reshape(shape).copy())
    return out
