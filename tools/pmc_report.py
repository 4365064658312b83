"""Mean per-dispatch value of every PMC counter per kernel, from rocprofv3 --pmc CSV output(s).
  python tools/pmc_report.py gpurun_out/p1/run_counter_collection.csv [more.csv ...] [--filter attn]"""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
filt = ""
if "--filter" in args:
    i = args.index("--filter")
    filt = args[i + 1]
    del args[i:i + 2]
paths = args
acc = defaultdict(lambda: defaultdict(list))
for p in paths:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if filt and filt not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
