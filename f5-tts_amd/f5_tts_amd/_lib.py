"""ctypes binding of the C ABI in include/f5h.h (libf5h.so, gfx950).

torch is imported first on purpose: torch ships its own libamdhip64.so (SONAME
libamdhip64.so.7); libf5h.so's NEEDED entry then resolves to that already-loaded
runtime, so torch's device pointers and streams are valid inside the engine.

There is no fallback: if the library is missing or cannot load, every engine
entry point raises (the product path never drops to PyTorch or to the oracle).
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("F5H_LIB", os.path.join(_HERE, "lib", "libf5h.so"))

F5H_DIT, F5H_UNETT = 0, 1
F5H_FP32, F5H_BF16, F5H_FP16 = 0, 1, 2
COMPUTE = {"fp32": F5H_FP32, "bf16": F5H_BF16, "fp16": F5H_FP16}
F5H_DT_F32, F5H_DT_BF16, F5H_DT_F16 = 0, 1, 2

# exported symbols, checked by tests/test_boundary.py against include/f5h.h
EXPORTS = (
    "f5h_engine_create_views",
    "f5h_engine_create",
    "f5h_engine_destroy",
    "f5h_release_pending",
    "f5h_workspace_size",
    "f5h_sample",
    "f5h_forward",
    "f5h_probe_enable",
    "f5h_probe_read",
    "f5h_probe_timeline",
    "f5h_set_graph_mode",
    "f5h_set_cfg_streams",
    "f5h_graph_stats",
    "f5h_last_call_host_ms",
    "f5h_set_pad_skip",
    "f5h_set_chain",
    "f5h_chain_stats",
    "f5h_chain_debug_spin_limit",
    "f5h_set_ln_fold",
    "f5h_ln_fold_stats",
    "f5h_op_linear",
    "f5h_op_attention",
    "f5h_gemm_force_config",
    "f5h_attn_force_safe",
    "f5h_debug_tile_live",
    "f5h_vocos_create",
    "f5h_vocos_destroy",
    "f5h_vocos_workspace_size",
    "f5h_vocos_decode",
    "f5h_mel_create",
    "f5h_mel_destroy",
    "f5h_mel_workspace_size",
    "f5h_mel_forward",
    "f5h_last_error",
    "f5h_version",
)

KCLASS = {"ffn1": 0, "attention": 1, "qkv": 2, "ffn2": 3, "conv": 4, "out": 5, "norm": 6, "chain": 7}


class Arch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "backbone", "dim", "depth", "heads", "dim_head", "ff_dim", "text_dim", "text_num_embeds", "mel_dim",
        "conv_layers", "text_mask_padding", "pe_attn_head", "attn_mask_enabled", "compute")]


class VocosArch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "input_channels", "dim", "intermediate_dim", "num_layers", "n_fft", "hop_length", "compute")]


class MelArch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("n_fft", "hop_length", "n_mels", "sample_rate")]


class Weight(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class TensorView(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("dtype", ctypes.c_int32),
                ("on_device", ctypes.c_int32), ("numel", ctypes.c_int64)]


class SampleArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("N", ctypes.c_int32), ("nt", ctypes.c_int32), ("nfe", ctypes.c_int32),
        ("cond", ctypes.c_void_p), ("cond_mask", ctypes.c_void_p), ("text", ctypes.c_void_p),
        ("duration", ctypes.c_void_p), ("y0", ctypes.c_void_p), ("t_grid", ctypes.c_void_p),
        ("cfg_strength", ctypes.c_float), ("use_batch_mask", ctypes.c_int32),
        ("out", ctypes.c_void_p), ("trajectory", ctypes.c_void_p),
    ]


class ForwardArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("N", ctypes.c_int32), ("nt", ctypes.c_int32),
        ("x", ctypes.c_void_p), ("cond", ctypes.c_void_p), ("cond_mask", ctypes.c_void_p),
        ("text", ctypes.c_void_p), ("duration", ctypes.c_void_p), ("t", ctypes.c_float),
        ("use_batch_mask", ctypes.c_int32), ("pred", ctypes.c_void_p),
        ("cfg_infer", ctypes.c_int32), ("drop_audio_cond", ctypes.c_int32), ("drop_text", ctypes.c_int32),
        ("t_dev", ctypes.c_void_p), ("text_cache", ctypes.c_int32),
    ]


_lib = None
_load_error = None


def lib():
    """Load libf5h.so once; raise a clear error if it is absent (no silent fallback)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RuntimeError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libf5h.so not found at {LIB_PATH}: build it with `python -c \"import __graft_entry__ as g; "
                       f"g.build()\"` or `make -C f5-tts_amd/csrc`")
        raise RuntimeError(_load_error)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
    L.f5h_engine_create.argtypes = [ctypes.POINTER(Arch), ctypes.POINTER(Weight), i32, i32, ctypes.POINTER(vp)]
    L.f5h_engine_create.restype = ctypes.c_int
    L.f5h_engine_create_views.argtypes = [ctypes.POINTER(Arch), ctypes.POINTER(TensorView), i32, i32,
                                          ctypes.POINTER(vp)]
    L.f5h_engine_create_views.restype = ctypes.c_int
    L.f5h_engine_destroy.argtypes = [vp]
    L.f5h_engine_destroy.restype = None
    L.f5h_release_pending.argtypes = [i32]
    L.f5h_release_pending.restype = ctypes.c_int
    L.f5h_workspace_size.argtypes = [vp, i32, i32, i32, i32, i32]
    L.f5h_workspace_size.restype = sz
    L.f5h_sample.argtypes = [vp, vp, ctypes.POINTER(SampleArgs), vp, sz]
    L.f5h_sample.restype = ctypes.c_int
    L.f5h_forward.argtypes = [vp, vp, ctypes.POINTER(ForwardArgs), vp, sz]
    L.f5h_forward.restype = ctypes.c_int
    L.f5h_probe_enable.argtypes = [vp, i32, i32]
    L.f5h_probe_enable.restype = ctypes.c_int
    L.f5h_probe_read.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double)]
    L.f5h_probe_read.restype = ctypes.c_int
    L.f5h_probe_timeline.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), i32, ctypes.POINTER(i32),
                                     ctypes.POINTER(ctypes.c_double)]
    L.f5h_probe_timeline.restype = ctypes.c_int
    L.f5h_set_graph_mode.argtypes = [vp, i32]
    L.f5h_set_graph_mode.restype = ctypes.c_int
    L.f5h_set_cfg_streams.argtypes = [vp, i32]
    L.f5h_set_cfg_streams.restype = ctypes.c_int
    L.f5h_graph_stats.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i32)]
    L.f5h_graph_stats.restype = ctypes.c_int
    if hasattr(L, "f5h_last_call_host_ms"):
        L.f5h_last_call_host_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i32]
        L.f5h_last_call_host_ms.restype = ctypes.c_int
    L.f5h_set_pad_skip.argtypes = [vp, i32]
    L.f5h_set_pad_skip.restype = ctypes.c_int
    L.f5h_op_linear.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, sz]
    L.f5h_op_linear.restype = ctypes.c_int
    L.f5h_op_attention.argtypes = [vp, i32, i32, i32, i32, vp, vp, vp, vp, i32, vp, vp, sz]
    L.f5h_op_attention.restype = ctypes.c_int
    L.f5h_gemm_force_config.argtypes = [i32]
    L.f5h_gemm_force_config.restype = ctypes.c_int
    # test hooks: bound when present, so an older build loaded through F5H_LIB (one-box A/Bs) still loads
    if hasattr(L, "f5h_attn_force_safe"):
        L.f5h_attn_force_safe.argtypes = [i32]
        L.f5h_attn_force_safe.restype = ctypes.c_int
    if hasattr(L, "f5h_set_chain"):
        L.f5h_set_chain.argtypes = [vp, i32]
        L.f5h_set_chain.restype = ctypes.c_int
        L.f5h_chain_stats.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.POINTER(i64)]
        L.f5h_chain_stats.restype = ctypes.c_int
    if hasattr(L, "f5h_set_ln_fold"):
        L.f5h_set_ln_fold.argtypes = [vp, i32]
        L.f5h_set_ln_fold.restype = ctypes.c_int
        L.f5h_ln_fold_stats.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i64)]
        L.f5h_ln_fold_stats.restype = ctypes.c_int
    if hasattr(L, "f5h_chain_debug_spin_limit"):
        L.f5h_chain_debug_spin_limit.argtypes = [i64]
        L.f5h_chain_debug_spin_limit.restype = ctypes.c_int
    if hasattr(L, "f5h_debug_tile_live"):
        L.f5h_debug_tile_live.argtypes = [vp, i32, i32, i32, i32]
        L.f5h_debug_tile_live.restype = ctypes.c_int
    L.f5h_vocos_create.argtypes = [ctypes.POINTER(VocosArch), ctypes.POINTER(Weight), i32, i32, ctypes.POINTER(vp)]
    L.f5h_vocos_create.restype = ctypes.c_int
    L.f5h_vocos_destroy.argtypes = [vp]
    L.f5h_vocos_destroy.restype = None
    L.f5h_vocos_workspace_size.argtypes = [vp, i32, i32]
    L.f5h_vocos_workspace_size.restype = sz
    L.f5h_vocos_decode.argtypes = [vp, vp, i32, i32, vp, vp, vp, sz]
    L.f5h_vocos_decode.restype = ctypes.c_int
    L.f5h_mel_create.argtypes = [ctypes.POINTER(MelArch), i32, ctypes.POINTER(vp)]
    L.f5h_mel_create.restype = ctypes.c_int
    L.f5h_mel_destroy.argtypes = [vp]
    L.f5h_mel_destroy.restype = None
    L.f5h_mel_workspace_size.argtypes = [vp, i32, i32]
    L.f5h_mel_workspace_size.restype = sz
    L.f5h_mel_forward.argtypes = [vp, vp, i32, i32, vp, vp, vp, sz]
    L.f5h_mel_forward.restype = ctypes.c_int
    L.f5h_last_error.argtypes = []
    L.f5h_last_error.restype = ctypes.c_char_p
    L.f5h_version.argtypes = []
    L.f5h_version.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc: int, what: str = "f5h"):
    if rc != 0:
        msg = lib().f5h_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
