import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "f5-tts_amd")]
import torch
from f5_tts_amd.engine import op_attention
torch.manual_seed(0)
S, H, N = 1, 1, 64
Q, K, V = (torch.randn(S, H, N, 64, device="cuda") for _ in range(3))
O = op_attention(Q, K, V, None, compute="bf16").reshape(N, 64)
q, k, v = Q[0, 0], K[0, 0], V[0, 0]
def attn(q, k, v, scale):
    return torch.softmax(q @ k.t() * scale, -1) @ v
cands = {
    "ref": attn(q, k, v, 0.125),
    "noscale": attn(q, k, v, 1.0),
    "scale^2": attn(q, k, v, 0.125 * 0.125 * 1.4427),
    "scale*log2e(no conv)": attn(q, k, v, 0.125 * 1.4427),
    "uniform": v.mean(0).expand(N, 64),
    "kv swapped": attn(q, v, k, 0.125),
    "q as k": attn(k, q, v, 0.125),
}
for name, c in cands.items():
    print(f"{name:24s} maxerr {(O - c).abs().max().item():.4f}")
print("O[0,:8]", O[0, :8].tolist())
print("ref[0,:8]", cands["ref"][0, :8].tolist())
print("O row norms", O.norm(dim=1)[:6].tolist(), "ref", cands["ref"].norm(dim=1)[:6].tolist())
P = torch.softmax(q @ k.t() * 0.125, -1).double()
Veff = torch.linalg.solve(P, O.double())
# match each effective row to the closest true V row
d = torch.cdist(Veff.float(), v)
best = d.argmin(1)
print("row map (eff row -> V row):", best.tolist())
print("match dist", d.min(1).values.max().item())
# also try columns: maybe dh permuted
dc = torch.cdist(Veff.float().t(), v.t())
print("col map:", dc.argmin(1).tolist(), dc.min(1).values.max().item())
