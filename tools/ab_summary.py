"""Summarise a one-box interleaved A/B (tools/gpu_ab.sh output dir) as text: per config and arm, every round's
ms per call and the per-class average launch (bench.py roofline_classes, in-kernel stamps), then the arm means.

  python tools/ab_summary.py gpurun_out/<dir> [title] > profiles/<name>.txt
"""
import glob
import json
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
runs = defaultdict(list)  # (config, arm) -> [(round, line)]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    m = re.match(r"(c\d)_(.+)_(\d+)\.log$", os.path.basename(f))
    if not m:
        continue
    try:
        line = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    runs[(m.group(1), m.group(2))].append((int(m.group(3)), line))
print(f"# {title}")
heads = {(c, a): v[0][1].get("config", {}).get("head") for (c, a), v in runs.items()}
classes = ["qkv", "attention", "out", "norm", "ffn1", "ffn2", "conv"]
for cfg in sorted({c for c, _ in runs}):
    print(f"\n## {cfg}: ms per call (per-class avg launch us, probe pre-pass)")
    print("arm round ms " + " ".join(classes))
    means = {}
    for (c, arm), v in sorted(runs.items()):
        if c != cfg:
            continue
        ms = []
        for rnd, line in sorted(v, key=lambda t: t[0]):
            rc = line.get("roofline_classes") or {}
            cl = " ".join(f"{rc[k]['avg_launch_us']:.2f}" if k in rc else "-" for k in classes)
            print(f"{arm} {rnd} {line['ms_per_step']:.2f} {cl}")
            ms.append(line["ms_per_step"])
        means[arm] = sum(ms) / len(ms)
    print("mean: " + ", ".join(f"{a} {m:.2f}" for a, m in means.items()))
