"""Time every bf16 GEMM tile configuration on the path's GEMM shapes.

Run under rocprofv3 (kernel trace), then report from the trace:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -o run -- python tools/gemm_tune.py
  python tools/gemm_tune.py --report gpurun_out/gt/run_kernel_trace.csv
Dispatches are keyed by (tile template, grid), which is unique per (shape, config) here.
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))

SHAPES = {  # name: (M, N, K); C2 = 2 x 1876 rows, C3 = 64 x 1876 rows
    "c2_qkv": (3752, 3072, 1024), "c2_ffn1": (3752, 2048, 1024), "c2_out": (3752, 1024, 1024),
    "c2_ffn2": (3752, 1024, 2048), "c3_qkv": (120064, 3072, 1024), "c3_ffn2": (120064, 1024, 2048),
    "c3_ffn1": (120064, 2048, 1024), "c3_out": (120064, 1024, 1024), "c5_qkv": (30032, 3072, 1024),
}
for _k in (128, 256, 512, 2048, 4096):  # K sweeps at the C2 output shapes: fixed cost per launch = intercept
    SHAPES[f"c2_out_k{_k}"] = (3752, 1024, _k)
    SHAPES[f"c2_qkv_k{_k}"] = (3752, 3072, _k)
CFGS = {0: (64, 128, 256), 1: (128, 128, 256), 5: (192, 128, 256), 11: (256, 256, 512), 12: (256, 256, 512),
        13: (256, 256, 512)}  # 13: persistent (one block per CU)
# round 5 also timed one-block-per-CU ping-pong tiles at the C2 shapes (128x128, 256x128, 192x256 as cfg 14-16):
# slower than the picks on every C2 GEMM (profiles/r05_gemm_tune_c2_pp.txt), removed
# round 3 also timed register-staged intake (cfg 40-45) and K32-stage deeper rings for 192x128 / 128x128
# (cfg 6-8): slower on every C2 and C3 shape (profiles/r03_gemm_tune_rs_c2.txt, r03_gemm_tune_k32.txt)
# round 2 also timed 8-wave one-block-per-CU tiles (128x256, 192x256, 256x128, 128x128, 256x256, 256x192),
# K32-stage deep rings (64x128..128x256) and DMA issue interleaved with the MFMAs; all slower at C2
# (profiles/r02_gemm_tune_c2*.txt), so they are no longer built.
REPS = 20
if os.environ.get("GT_CFGS"):  # e.g. GT_CFGS=5,11 GT_SHAPES=c3_qkv,c3_ffn2
    CFGS = {int(c): CFGS[int(c)] for c in os.environ["GT_CFGS"].split(",")}
if os.environ.get("GT_SHAPES"):
    SHAPES = {k: SHAPES[k] for k in os.environ["GT_SHAPES"].split(",")}


def grid_threads(M, N, cfg):
    bm, bn, th = CFGS[cfg]
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    return (min(tiles, 256) if cfg == 13 else tiles) * th


ROUNDS, PER = 5, REPS // 5  # interleaved rounds per shape (MI355X_MICROARCH DVFS: compare within one process)
MODES = [-1]  # round 2 also A/B'd a tile -> XCD rectangle grouping here: no gain (profiles/r02_gemm_tune_c2_xcd.txt)


def run():
    import torch
    from f5_tts_amd.engine import gemm_force_config, op_linear

    dev = "cuda:0"
    for name, (M, N, K) in SHAPES.items():
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) / K ** 0.5
        for _ in range(ROUNDS):
            for cfg in CFGS:
                gemm_force_config(cfg)
                for mode in MODES:
                    for _ in range(PER):
                        op_linear(A, W, None, compute="bf16")
        torch.cuda.synchronize()
        print(f"done {name}", flush=True)
    gemm_force_config(-1)


def report(path):
    """The gemm dispatches in issue order are SHAPES x ROUNDS x CFGS x MODES x PER (run() order)."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
          if "gemm_" in r["Kernel_Name"]]
    assert len(ts) == len(SHAPES) * ROUNDS * len(CFGS) * len(MODES) * PER, len(ts)
    k = 0
    for name, (M, N, K) in SHAPES.items():
        got = {}
        for _ in range(ROUNDS):
            for cfg in CFGS:
                for mode in MODES:
                    got.setdefault((cfg, mode), []).extend(ts[k:k + PER])
                    k += PER
        line = []
        for (cfg, mode), t in got.items():
            t = sorted(t)[: len(t) * 3 // 4]  # drop the slowest quarter (cold caches)
            avg = sum(t) / len(t)
            tag = f"cfg{cfg}" + (f"/x{mode}" if len(MODES) > 1 else "")
            line.append(f"{tag:9s} {avg:8.2f}us {2 * M * N * K / avg / 1e6:5.0f}TF")
        print(f"{name:8s}")
        for i in range(0, len(line), 6):
            print("   " + " | ".join(line[i:i + 6]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--report")
    a = ap.parse_args()
    report(a.report) if a.report else run()
