"""Reads the phase stamps of a F5H_PW_STAMPS build of attn_pw_kernel (tile 12 of every wave, C2
shape): python tools/attn_stamps_pw.py   (needs the diagnostic libf5h.so)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import torch  # noqa: E402

from f5_tts_amd.engine import op_attention  # noqa: E402

S, H, N = 2, 16, 1876
g = torch.Generator(device="cpu").manual_seed(0)
Q, K, V = (torch.randn(S, H, N, 64, generator=g).cuda() for _ in range(3))
Q = Q * (0.125 * 1.4426950408889634)
for _ in range(5):
    O = op_attention(Q, K, V, None, compute="bf16", q_prescaled=True)
torch.cuda.synchronize()
nw = 8 * S * H * 4
raw = O.flatten()[: nw * 8].to(torch.bfloat16).view(torch.int16).to(torch.int64).cpu().view(nw, 8)
names = ["alpha QK(B)+max(A)", "alpha P.V(B)+exp(A)", "vmcnt+barrier", "beta P.V(A)c0-1+max(B)",
         "beta rebase+P.V(A)c2", "beta P.V(A)c3", "beta QK(A)+exp(B)"]
med = raw.median(0).values
print("per-phase median cycles (tile 12):")
for i, n in enumerate(names):
    print(f"  {n:28s} {int(med[i + 1] - med[i]) if i < 7 else 0:6d}")
tot = raw[:, 7]
print(f"tile total: median {int(tot.median())}  min {int(tot.min())}  max {int(tot.max())}")
