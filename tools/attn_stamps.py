"""Cycle anatomy of the v5 attention K loop (diagnostic variant 6): per-segment cycles per tile."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import torch  # noqa: E402

from f5_tts_amd import _lib  # noqa: E402
from f5_tts_amd.engine import attn_force_variant, op_attention  # noqa: E402

S, H, N = 2, 16, 1876
g = torch.Generator(device="cpu").manual_seed(0)
Q, K, V = (torch.randn(S, H, N, 64, generator=g).cuda() for _ in range(3))
VAR = int(sys.argv[1]) if len(sys.argv) > 1 else 6
attn_force_variant(VAR)
for _ in range(5):
    op_attention(Q, K, V, None, compute="bf16")
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * 256)()
_lib.check(_lib.lib().f5h_debug_attn_stamps(ctypes.cast(buf, ctypes.c_void_p), 256), "stamps")
names = (["qk issue", "pv issue", "exp+cvt", "vmcnt", "barrier", "dma+reads+lds wait"] if VAR == 6 else
         ["X: qk issue", "X: exp+cvt", "X: barrier", "Y: pv+dma+reads+lds wait", "Y: vmcnt", "Y: barrier"])
rows = []
for w in range(32):
    grp = (w % 8) // 4
    v = buf[w * 8:(w + 1) * 8]
    nt = v[6]
    if nt:
        rows.append((grp, [v[k] / (nt - 1) for k in range(6)]))
for gsel in (0, 1):
    sel = [r for gg, r in rows if gg == gsel]
    print(f"group {gsel}")
    for k, n in enumerate(names):
        vals = [r[k] for r in sel]
        print(f"  {n:26s} mean {sum(vals) / len(vals):8.1f}  min {min(vals):8.1f}  max {max(vals):8.1f} cycles/tile")
    print(f"  total {sum(sum(r) for r in sel) / len(sel):8.1f} cycles/tile (s_memtime ticks)")
attn_force_variant(-1)
