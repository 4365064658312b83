"""Interleaved A/B of the bf16 attention variants in ONE process (cdna_hip_programming.md rule 24).
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aab -o run -- python tools/attn_ab.py 1 2 3
  python tools/attn_ab.py --report gpurun_out/aab/run_kernel_trace.csv"""
import csv
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
S, H, N, ROUNDS, REPS = 2, 16, 1876, int(os.environ.get("AB_ROUNDS", "12")), 10


def run(variants):
    import torch
    from f5_tts_amd.engine import attn_force_variant, op_attention
    g = torch.Generator(device="cpu").manual_seed(0)
    Q, K, V = (torch.randn(S, H, N, 64, generator=g).cuda() for _ in range(3))
    Q = Q * (0.125 * 1.4426950408889634)  # q_prescaled: the engine's layout (scores in log2 units)
    for _ in range(ROUNDS):
        for v in variants:
            attn_force_variant(v)
            for _ in range(REPS):
                op_attention(Q, K, V, None, compute="bf16", q_prescaled=True)
    torch.cuda.synchronize()
    attn_force_variant(-1)


def report(path):
    by = {}
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "attn_bf16" not in n:
            continue
        key = n.split("(")[0].replace("void ", "")
        by.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    fl = 4.0 * S * H * N * N * 64
    for k, ts in sorted(by.items()):
        med = statistics.median(ts)
        print(f"{k:50s} n={len(ts):4d} median {med:8.2f} us  min {min(ts):8.2f}  {fl / med / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    if sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run([int(v) for v in sys.argv[1:]])
