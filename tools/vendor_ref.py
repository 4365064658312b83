"""Vendor-library yardstick for the path's shapes (not on the product path): hipBLASLt GEMMs via torch.mm
(bf16, no epilogue) and torch SDPA (bf16, head dim 64, non-causal) at the C2 (S = 2) and C4-per-rank / C3
(S = 64, padded to 1876 frames) shapes of every kernel class. Run under `rocprofv3 --kernel-trace --stats` to
get the per-kernel averages; also prints / writes event-timed averages per op (20 back-to-back launches).

  python tools/vendor_ref.py [out.json]

VENDOR_GEMM_ONLY=1 skips SDPA and VENDOR_REPS=n fixes the timed launches per op (3 warm + n each, in SH order:
tools/vendor_pmc.py maps counter-pass dispatches to ops by that order).
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

dev = "cuda:0"
N_FR, D, F_DIM = 1876, 1024, 2048
SH = {}
for cfg, S in (("c2", 2), ("c4", 64)):
    M = S * N_FR
    SH[f"{cfg}_qkv"] = (M, 3 * D, D)
    SH[f"{cfg}_out"] = (M, D, D)
    SH[f"{cfg}_ffn1"] = (M, F_DIM, D)
    SH[f"{cfg}_ffn2"] = (M, D, F_DIM)


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


res = {"device": torch.cuda.get_device_name(0), "torch": torch.__version__, "ops": {}}
g = torch.Generator(device=dev).manual_seed(0)
for name, (M, N, K) in SH.items():
    A = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
    reps = int(os.environ.get("VENDOR_REPS", "0")) or (20 if M < 10000 else 5)
    us = timed(lambda: A @ W.t(), reps)
    tf = 2 * M * N * K / us / 1e6
    res["ops"][name] = {"kind": "hipBLASLt torch.mm bf16", "M": M, "N": N, "K": K, "us": us, "tflops": tf,
                        "frac": tf / 2500.0}
    print(f"{name}: {us:.1f} us  {tf:.0f} TF/s", flush=True)
    del A, W
for cfg, S in (() if os.environ.get("VENDOR_GEMM_ONLY") == "1" else (("c2", 2), ("c4", 64))):
    q, k, v = (torch.randn(S, 16, N_FR, 64, device=dev, dtype=torch.bfloat16, generator=g) for _ in range(3))
    us = timed(lambda: F.scaled_dot_product_attention(q, k, v), 10 if S < 10 else 3)
    tf = 4 * S * 16 * N_FR * N_FR * 64 / us / 1e6
    res["ops"][f"{cfg}_attention"] = {"kind": "torch SDPA bf16", "S": S, "H": 16, "N": N_FR, "us": us,
                                      "tflops": tf, "frac": tf / 2500.0}
    print(f"sdpa {cfg} S={S}: {us:.1f} us  {tf:.0f} TF/s", flush=True)
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
