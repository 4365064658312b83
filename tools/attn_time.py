"""Times the 16-bit attention kernel at the C2 shape (S=2, H=16, N=1876, q prescaled).
  rocprofv3 --kernel-trace --stats -d gpurun_out/at -o run -- python tools/attn_time.py
Also checks the variant against an fp64 softmax of the same rounded operands."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import torch  # noqa: E402

from f5_tts_amd.engine import op_attention  # noqa: E402

S, H, N = 2, 16, int(os.environ.get("ATTN_N", "1876"))
g = torch.Generator(device="cpu").manual_seed(0)
Q, K, V = (torch.randn(S, H, N, 64, generator=g) for _ in range(3))
Q = Q * (0.125 * 1.4426950408889634)
Q, K, V = (x.to(torch.bfloat16) for x in (Q, K, V))
Qd, Kd, Vd = (x.float().cuda() for x in (Q, K, V))
for _ in range(int(os.environ.get("ATTN_REPS", "50"))):
    O = op_attention(Qd, Kd, Vd, None, compute="bf16", q_prescaled=True)
torch.cuda.synchronize()
sc = Q.double() @ K.double().transpose(-1, -2)
p = torch.exp2(sc - sc.amax(-1, keepdim=True))
ref = ((p / p.sum(-1, keepdim=True)) @ V.double()).transpose(1, 2).reshape(S, N, H * 64)
err = ((O.cpu().double() - ref).abs().max() / ref.abs().max()).item()
print(f"N={N} max-rel err {err:.3e}")
assert err < 1e-2
