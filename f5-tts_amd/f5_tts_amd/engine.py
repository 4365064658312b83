"""Python handle on the HIP engine (libf5h.so). Plumbing only: device memory and the
current stream come from PyTorch; every FLOP runs in the engine's kernels."""

from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib


_VIEW_DT = {torch.float32: _lib.F5H_DT_F32, torch.bfloat16: _lib.F5H_DT_BF16, torch.float16: _lib.F5H_DT_F16}


def _arch_struct(arch: dict, compute: str) -> _lib.Arch:
    a = _lib.Arch()
    a.backbone = _lib.F5H_DIT if arch["backbone"] == "DiT" else _lib.F5H_UNETT
    a.dim = arch["dim"]
    a.depth = arch["depth"]
    a.heads = arch["heads"]
    a.dim_head = arch.get("dim_head", 64)
    a.ff_dim = int(arch["dim"] * arch["ff_mult"])
    a.text_dim = arch["text_dim"] if arch.get("text_dim") is not None else arch["mel_dim"]
    a.text_num_embeds = arch["text_num_embeds"]
    a.mel_dim = arch["mel_dim"]
    a.conv_layers = arch.get("conv_layers", 0)
    a.text_mask_padding = int(bool(arch.get("text_mask_padding", True)))
    a.pe_attn_head = int(arch.get("pe_attn_head") or 0)
    a.attn_mask_enabled = int(bool(arch.get("attn_mask_enabled", False)))
    a.compute = _lib.COMPUTE[compute]
    if arch.get("qk_norm"):
        raise NotImplementedError("qk_norm is not used by any shipped config (F5TTS_*.yaml qk_norm: null)")
    if arch.get("long_skip_connection") or arch.get("text_embedding_average_upsampling"):
        raise NotImplementedError("long_skip_connection / average upsampling are off in every shipped config")
    return a


class Engine:
    """One packed model on one device. Immutable after construction, so one instance may
    serve concurrent `sample` calls from several host threads (each call allocates its own
    workspace from the torch caching allocator)."""

    def __init__(self, arch: dict, weights: dict, compute: str = "bf16", device=None):
        L = _lib.lib()
        self.arch = dict(arch)
        self.compute = compute
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        # typed views of the parameters in their own dtype and placement (utils_infer.py:190-232 leaves
        # them fp16/bf16/fp32 on the device): the engine packs from them on the device, no host copy
        keep, views = [], []
        for k, v in weights.items():
            k = k[len("transformer."):] if k.startswith("transformer.") else k
            t = v.detach() if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
            if t.dtype not in _VIEW_DT:
                t = t.to(torch.float32)
            if t.is_cuda and t.device != self.device:
                t = t.to(self.device)
            t = t.contiguous()
            keep.append(t)
            views.append((k.encode(), t))
        arr = (_lib.TensorView * len(views))()
        for i, (name, t) in enumerate(views):
            arr[i].name = name
            arr[i].data = t.data_ptr()
            arr[i].dtype = _VIEW_DT[t.dtype]
            arr[i].on_device = int(t.is_cuda)
            arr[i].numel = t.numel()
        a = _arch_struct(self.arch, compute)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            # device views are read on the engine's internal stream: the producers must be done
            if any(t.is_cuda for t in keep):
                torch.cuda.current_stream(self.device).synchronize()
            _lib.check(L.f5h_engine_create_views(ctypes.byref(a), arr, len(views), self.device.index,
                                                 ctypes.byref(h)), "f5h_engine_create_views")
        del keep
        self._h = h
        self._lock = threading.Lock()
        # per-(stream, size) workspaces kept across calls: the engine's NFE-step hipGraph is keyed
        # by the workspace address, so a stable workspace makes every call after the first a replay.
        # A call holds its workspace's lock while it enqueues, so calls sharing a stream serialise
        # in stream order and calls on different streams never share a workspace.
        self._ws_cache: dict = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().f5h_engine_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ workspace
    def workspace_bytes(self, B, N, nt, nfe, use_cfg=True) -> int:
        return int(_lib.lib().f5h_workspace_size(self._h, B, N, nt, nfe, int(use_cfg)))

    def _workspace(self, nbytes):
        return torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.device)

    def _cached_workspace(self, nbytes, stream):
        with self._lock:
            ent = self._ws_cache.get((stream, nbytes))
            if ent is None:
                if len(self._ws_cache) >= 4:
                    self._ws_cache.pop(next(iter(self._ws_cache)))
                ent = (self._workspace(nbytes), threading.Lock())
                self._ws_cache[(stream, nbytes)] = ent
            return ent

    def set_graph_mode(self, on: bool):
        """True: the NFE loop replays one captured hipGraph step (default); False: eager launches."""
        _lib.check(_lib.lib().f5h_set_graph_mode(self._h, int(bool(on))), "set_graph_mode")

    def set_cfg_streams(self, n: int):
        """2: the captured step runs the two CFG branches as parallel launch chains; 1: one chain;
        0: automatic (the default; currently one chain, the faster form at C2, C3 and C5)."""
        _lib.check(_lib.lib().f5h_set_cfg_streams(self._h, int(n)), "set_cfg_streams")

    def set_pad_skip(self, on: bool):
        """Skip the batch path's dead pad-row work (attention query blocks and out-proj row tiles of
        padding only; default on). Results are bitwise identical either way."""
        _lib.check(_lib.lib().f5h_set_pad_skip(self._h, int(bool(on))), "set_pad_skip")

    def set_chain(self, on: bool):
        """Run each DiT layer's row-local seams (out-proj .. next QKV) as one phase-chain launch (16-bit DiT
        path without row masks; f5h_set_chain; default on). Results are bitwise identical either way."""
        _lib.check(_lib.lib().f5h_set_chain(self._h, int(bool(on))), "set_chain")

    def set_ln_fold(self, on: bool):
        """Run the AdaLN LayerNorms between the residual GEMMs and their consumers inside those GEMMs (16-bit DiT
        path without row masks; f5h_set_ln_fold; default on). Not bitwise the separate launches."""
        _lib.check(_lib.lib().f5h_set_ln_fold(self._h, int(bool(on))), "set_ln_fold")

    def ln_fold_stats(self):
        """(the engine can fold, backbone passes enqueued with the fold)."""
        sup, n = ctypes.c_int32(), ctypes.c_int64()
        _lib.check(_lib.lib().f5h_ln_fold_stats(self._h, ctypes.byref(sup), ctypes.byref(n)), "ln_fold_stats")
        return bool(sup.value), int(n.value)

    def chain_stats(self):
        """(phase-chain launches this engine enqueued, 1 if one of its chain waits gave up and the engine has not
        reported it yet, chained calls of this process that the per-device concurrency rule sent to the separate
        launches). Synchronous; call after the engine's work has completed (f5h_chain_stats)."""
        n, f, r = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int64()
        _lib.check(_lib.lib().f5h_chain_stats(self._h, ctypes.byref(n), ctypes.byref(f), ctypes.byref(r)),
                   "chain_stats")
        return int(n.value), int(f.value), int(r.value)

    HOST_PHASES = ("total", "prologue", "cache_lock", "reap", "capture", "instantiate", "launch", "final")

    def last_call_host_ms(self):
        """Host milliseconds of this engine's newest sample call by phase (f5h_last_call_host_ms)."""
        buf = (ctypes.c_double * 8)()
        _lib.check(_lib.lib().f5h_last_call_host_ms(self._h, buf, 8), "last_call_host_ms")
        return {k: round(buf[i], 4) for i, k in enumerate(self.HOST_PHASES)}

    def graph_stats(self):
        cap, rep, n = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        _lib.check(_lib.lib().f5h_graph_stats(self._h, ctypes.byref(cap), ctypes.byref(rep), ctypes.byref(n)),
                   "graph_stats")
        return {"captures": cap.value, "replays": rep.value, "cached": n.value}

    # ------------------------------------------------------------------ calls
    def sample(self, cond, cond_mask, text, duration, y0, t_grid, cfg_strength, use_batch_mask,
               out=None, keep_trajectory=True, workspace=None):
        """Run the CFM ODE loop. Tensors on this engine's device:
        cond f32 [B,N,mel], cond_mask bool/u8 [B,N], text int64 [B,nt], duration int [B],
        y0 f32 [B,N,mel]; t_grid: host sequence of nfe+1 floats."""
        B, N, mel = cond.shape
        nt = text.shape[1]
        tg = np.ascontiguousarray(np.asarray(t_grid, dtype=np.float32))
        nfe = tg.shape[0] - 1
        cond = cond.to(self.device, torch.float32).contiguous()
        cmask = cond_mask.to(self.device, torch.uint8).contiguous()
        text = text.to(self.device, torch.int64).contiguous()
        dur = duration.to(self.device, torch.int32).contiguous()
        y0 = y0.to(self.device, torch.float32).contiguous()
        if out is None:
            out = torch.empty(B, N, mel, dtype=torch.float32, device=self.device)
        traj = (torch.empty(nfe + 1, B, N, mel, dtype=torch.float32, device=self.device)
                if keep_trajectory else None)
        use_cfg = cfg_strength >= 1e-5
        need = self.workspace_bytes(B, N, nt, nfe, use_cfg)
        stream = _lib.stream_handle(self.device)
        if workspace is not None and workspace.numel() >= need:
            ws, wlock = workspace, threading.Lock()
        else:
            ws, wlock = self._cached_workspace(need, stream)
        a = _lib.SampleArgs()
        a.B, a.N, a.nt, a.nfe = B, N, nt, nfe
        a.cond, a.cond_mask, a.text, a.duration, a.y0 = (cond.data_ptr(), cmask.data_ptr(), text.data_ptr(),
                                                         dur.data_ptr(), y0.data_ptr())
        a.t_grid = tg.ctypes.data
        a.cfg_strength = float(cfg_strength)
        a.use_batch_mask = int(bool(use_batch_mask))
        a.out = out.data_ptr()
        a.trajectory = traj.data_ptr() if traj is not None else None
        with torch.cuda.device(self.device), wlock:
            _lib.check(_lib.lib().f5h_sample(self._h, stream, ctypes.byref(a), ws.data_ptr(), ws.numel()),
                       "f5h_sample")
        return out, traj

    def forward_workspace(self, B, N, nt, cfg_infer=True):
        """A workspace for `forward`; one kept across calls carries the text cache (text_cache=1/2)."""
        return self._workspace(self.workspace_bytes(B, N, nt, 1, cfg_infer))

    def forward(self, x, cond, cond_mask, text, duration, t, use_batch_mask, cfg_infer=True,
                drop_audio_cond=False, drop_text=False, text_cache=0, workspace=None):
        """One backbone forward at time t (DiT.forward / UNetT.forward, dit.py:319-370).
        cfg_infer: packed cond/uncond -> pred [2B,N,mel]; else one branch -> [B,N,mel] honouring
        drop_audio_cond / drop_text. t: a python float, or a one-element device tensor (read on the
        stream, no host sync). text_cache: 0 = compute the text embedding for this call, 1 = compute
        and keep it in `workspace`, 2 = reuse the one kept there (dit.py:294-317)."""
        B, N, mel = x.shape
        nt = text.shape[1]
        x = x.to(self.device, torch.float32).contiguous()
        cond = cond.to(self.device, torch.float32).contiguous()
        cmask = cond_mask.to(self.device, torch.uint8).contiguous()
        text = text.to(self.device, torch.int64).contiguous()
        dur = duration.to(self.device, torch.int32).contiguous()
        S = 2 * B if cfg_infer else B
        pred = torch.empty(S, N, mel, dtype=torch.float32, device=self.device)
        need = self.workspace_bytes(B, N, nt, 1, cfg_infer)
        if text_cache and (workspace is None or workspace.numel() < need):
            raise ValueError("text_cache needs a kept workspace of workspace_bytes(B, N, nt, 1, cfg_infer) bytes")
        ws = workspace if workspace is not None and workspace.numel() >= need else self._workspace(need)
        t_dev = None
        if torch.is_tensor(t):
            t_dev = t.reshape(-1)[:1].to(self.device, torch.float32).contiguous()
        a = _lib.ForwardArgs()
        a.B, a.N, a.nt = B, N, nt
        a.x, a.cond, a.cond_mask, a.text, a.duration = (x.data_ptr(), cond.data_ptr(), cmask.data_ptr(),
                                                        text.data_ptr(), dur.data_ptr())
        a.t = 0.0 if t_dev is not None else float(t)
        a.t_dev = t_dev.data_ptr() if t_dev is not None else None
        a.text_cache = int(text_cache)
        a.use_batch_mask = int(bool(use_batch_mask))
        a.pred = pred.data_ptr()
        a.cfg_infer = int(bool(cfg_infer))
        a.drop_audio_cond = int(bool(drop_audio_cond))
        a.drop_text = int(bool(drop_text))
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().f5h_forward(self._h, _lib.stream_handle(self.device), ctypes.byref(a),
                                              ws.data_ptr(), ws.numel()), "f5h_forward")
        return pred

    # ------------------------------------------------------------------ kernel probe
    def probe(self, kclass: str | None):
        L = _lib.lib()
        if kclass is None:
            _lib.check(L.f5h_probe_enable(self._h, 0, 0), "probe")
        else:
            _lib.check(L.f5h_probe_enable(self._h, _lib.KCLASS[kclass], 1), "probe")

    def probe_timeline(self, max_wg: int = 8192):
        """Per-workgroup [entry, loop entered, loop done, exit] stamps (microseconds from the earliest
        entry) of the probed class's first launch in the first probed step, as a [n_wg, 4] array."""
        buf = (ctypes.c_uint64 * (4 * max_wg))()
        n, khz = ctypes.c_int32(), ctypes.c_double()
        _lib.check(_lib.lib().f5h_probe_timeline(self._h, buf, max_wg, ctypes.byref(n), ctypes.byref(khz)),
                   "probe_timeline")
        a = np.frombuffer(buf, dtype=np.uint64, count=4 * n.value).reshape(n.value, 4).astype(np.float64)
        if n.value == 0 or khz.value <= 0:
            return a
        t0 = a[:, 0][a[:, 0] > 0].min()
        return np.where(a > 0, (a - t0) * 1e3 / khz.value, np.nan)

    def probe_read(self):
        n = ctypes.c_int64()
        ms = ctypes.c_double()
        _lib.check(_lib.lib().f5h_probe_read(self._h, ctypes.byref(n), ctypes.byref(ms)), "probe_read")
        return n.value, ms.value


# ---------------------------------------------------------------- op-level helpers (tests)
def op_linear(A, W, bias=None, compute="bf16"):
    M, K = A.shape
    N = W.shape[0]
    C = torch.empty(M, N, dtype=torch.float32, device=A.device)
    ws = torch.empty(((N + 127) // 128 * 128) * K * 4 + 512 + M * K * 4, dtype=torch.uint8, device=A.device)
    _lib.check(_lib.lib().f5h_op_linear(_lib.stream_handle(A.device), _lib.COMPUTE[compute], M, N, K,
                                        A.contiguous().data_ptr(), W.contiguous().data_ptr(), _lib.ptr(bias),
                                        C.data_ptr(), ws.data_ptr(), ws.numel()), "f5h_op_linear")
    return C


def op_attention(Q, K, V, kv_len=None, compute="bf16", q_prescaled=False, poison=False):
    """O[S,N,H*64] = softmax(Q K^T/8) V; q_prescaled: Q already carries (1/8)*log2(e). poison: fill the
    workspace (16-bit q | k | v | o, back to back) with NaN bits first, so a kernel that reads key rows past N
    (the next (sequence, head)'s rows, or past V into O) turns its output NaN."""
    S, H, N, D = Q.shape
    assert D == 64
    O = torch.empty(S, N, H * 64, dtype=torch.float32, device=Q.device)
    ws = torch.empty(Q.numel() * 8 + 1024, dtype=torch.uint8, device=Q.device)
    if poison:
        ws.fill_(0xFF)
    kv = None if kv_len is None else kv_len.to(Q.device, torch.int32).contiguous()
    _lib.check(_lib.lib().f5h_op_attention(_lib.stream_handle(Q.device), _lib.COMPUTE[compute], S, H, N,
                                           Q.contiguous().data_ptr(), K.contiguous().data_ptr(),
                                           V.contiguous().data_ptr(), _lib.ptr(kv), int(bool(q_prescaled)),
                                           O.data_ptr(), ws.data_ptr(), ws.numel()), "f5h_op_attention")
    return O


def attn_force_safe(on: bool):
    """Test hook: every later 16-bit attention launch reruns its key loop in the lazy-running-max form."""
    _lib.check(_lib.lib().f5h_attn_force_safe(int(bool(on))), "attn_force_safe")


def gemm_force_config(cfg: int = -1):
    """Pin the 16-bit GEMM tile configuration (0, 1, 5, 11, 12, 13) for this process; -1 = automatic."""
    _lib.check(_lib.lib().f5h_gemm_force_config(int(cfg)), "gemm_force_config")


def chain_debug_spin_limit(limit: int = -1):
    """Test hook: polls before a phase-chain wait gives up (0: at the first poll that finds its rows not yet
    produced); -1 restores the default (~0.3 s). Applies to launches and graph captures made afterwards."""
    _lib.check(_lib.lib().f5h_chain_debug_spin_limit(int(limit)), "chain_debug_spin_limit")
