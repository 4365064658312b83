"""Summarise a rocprofv3 kernel_stats.csv: share of GPU time per kernel."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:6.2f}% calls={r['Calls']:>6} avg={float(r['AverageNs']) / 1e3:9.2f}us"
          f"  {r['Name'][:100]}")
print(f"total GPU ms {tot / 1e6:.2f}")
