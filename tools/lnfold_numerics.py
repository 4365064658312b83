"""Numerics of folding AdaLN LayerNorm into the consuming GEMM, on the CPU.

Reference path (bf16 model, as the reference runs it): a = bf16(LN(h) * (1 + s) + shift), y = a . W^T.
Folded path: y = (h . W'^T - mu * c) * rstd + b',  W' = bf16(W * (1 + s)),  c = rowsum(W'),
b' = W . shift (fp32), mu / rstd from h.  Both against an fp64 evaluation of the same formula on the
same bf16 h and W. Rows carry a per-row offset of k sigmas (a large row mean is the folded form's
weak spot: u - mu*c cancels).  python tools/lnfold_numerics.py"""
import torch

torch.manual_seed(0)
d, n, rows = 1024, 2048, 512
W = (torch.randn(n, d) / d ** 0.5).bfloat16()
s = 0.3 * torch.randn(d)
shift = 0.1 * torch.randn(d)


def ln(x, eps=1e-6):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps), mu, 1 / torch.sqrt(var + eps)


print(f"{'mean/sigma':>10s} {'ref-path err':>13s} {'folded err':>11s}  (max|y - y64| / max|y64|)")
for k in (0, 1, 3, 10, 30, 100):
    h = (torch.randn(rows, d) + k * torch.randn(rows, 1).sign()).bfloat16()  # per-row offset of k sigma
    h64, W64 = h.double(), W.double()
    y64 = (ln(h64)[0] * (1 + s.double()) + shift.double()) @ W64.T
    a = (ln(h.float())[0] * (1 + s) + shift).bfloat16()
    y_ref = a.float() @ W.float().T
    Wp = (W.float() * (1 + s)).bfloat16()
    c = Wp.float().sum(-1)
    bp = shift @ W.float().T
    _, mu, rstd = ln(h.float())
    u = h.float() @ Wp.float().T
    y_fold = (u - mu * c) * rstd + bp
    e = lambda y: ((y.double() - y64).abs().max() / y64.abs().max()).item()  # noqa: E731
    print(f"{k:10d} {e(y_ref):13.2e} {e(y_fold):11.2e}")
