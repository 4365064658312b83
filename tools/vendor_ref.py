"""Vendor-library yardstick for the path's shapes (not on the product path): hipBLASLt GEMMs via
torch.mm (bf16) and torch SDPA (bf16) at C2/C3 shapes. Run under rocprofv3 --kernel-trace --stats
and read per-kernel averages; prints wall-clock per op as well."""
import torch
import torch.nn.functional as F

dev = "cuda:0"
SH = {"c2_qkv": (3752, 3072, 1024), "c2_ffn1": (3752, 2048, 1024), "c2_out": (3752, 1024, 1024),
      "c2_ffn2": (3752, 1024, 2048), "c3_qkv": (120064, 3072, 1024), "c3_ffn2": (120064, 1024, 2048)}
for name, (M, N, K) in SH.items():
    A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        C = A @ W.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    R = 20
    for _ in range(R):
        C = A @ W.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / R
    print(f"{name}: {ms*1e3:.1f} us  {2*M*N*K/ms/1e9:.0f} TF/s", flush=True)
for S, H, N in ((2, 16, 1876), (64, 16, 1876)):
    q, k, v = (torch.randn(S, H, N, 64, device=dev, dtype=torch.bfloat16) for _ in range(3))
    for _ in range(3):
        o = F.scaled_dot_product_attention(q, k, v)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        o = F.scaled_dot_product_attention(q, k, v)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"sdpa S={S}: {ms*1e3:.1f} us  {4*S*H*N*N*64/ms/1e9:.0f} TF/s", flush=True)
