"""GEMM timing probe for tile configs and ablation builds (F5H_GEMM_ABL, read once per process:
1 no DMA, 2 no MFMA, 4 no LDS reads in the K loop). Run under rocprofv3, then report:
  F5H_GEMM_ABL=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ga1 -o run -- python tools/gemm_abl.py 10 12
  python tools/gemm_abl.py --report gpurun_out/ga1/run_kernel_trace.csv 10 12"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))

SHAPES = {"c2_qkv": (3752, 3072, 1024), "c2_ffn1": (3752, 2048, 1024), "c2_out": (3752, 1024, 1024),
          "c2_ffn2": (3752, 1024, 2048), "c3_ffn2": (120064, 1024, 2048)}
REPS = 20


def shapes():
    only = os.environ.get("SHAPES")
    return {k: v for k, v in SHAPES.items() if not only or k in only.split(",")}


def run(cfgs):
    import torch
    from f5_tts_amd.engine import gemm_force_config, op_linear
    for name, (M, N, K) in shapes().items():
        A = torch.randn(M, K, device="cuda")
        W = torch.randn(N, K, device="cuda") / K ** 0.5
        for cfg in cfgs:
            gemm_force_config(cfg)
            for _ in range(REPS):
                op_linear(A, W, None, compute="bf16")
        torch.cuda.synchronize()
    gemm_force_config(-1)


def report(path, cfgs):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "gemm_" in r["Kernel_Name"]]
    sh = shapes()
    assert len(ts) == len(sh) * len(cfgs) * REPS, len(ts)
    k = 0
    for name, (M, N, K) in sh.items():
        line = []
        for cfg in cfgs:
            t = sorted(ts[k:k + REPS])[: REPS * 3 // 4]
            k += REPS
            us = sum(t) / len(t)
            line.append(f"cfg{cfg:<2d} {us:8.2f}us {2 * M * N * K / us / 1e6:5.0f}TF")
        print(f"{os.path.basename(os.path.dirname(path)):6s} {name:8s} " + " | ".join(line))


if __name__ == "__main__":
    if sys.argv[1] == "--report":
        report(sys.argv[2], [int(c) for c in sys.argv[3:]])
    else:
        run([int(c) for c in sys.argv[1:]])
