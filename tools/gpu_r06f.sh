#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06f}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_fold.py 2>&1 | grep -v amdgpu.ids | tee $O/diag_fold.log || exit 1
for f in 0 1; do
  F5H_LNFOLD=$f timeout -k 10 300 python bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-vocos > $O/bench_fold$f.log 2>&1 || exit 1
  tail -1 $O/bench_fold$f.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("fold='$f'", d["ms_per_step"], {k: v["avg_launch_us"] for k, v in d["roofline_classes"].items()})'
done
cd /tmp && F5H_LNFOLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fold1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 4 --warmup 2 --no-cpu-baseline --no-vocos --probe none > $O/prof_fold1.log 2>&1 || exit 1
f=$(find $O/prof_fold1 -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["Percentage"])
for r in rows:
    if "lnfold" in r["Name"]: print("LNFOLD", r["Calls"], r["AverageNs"])
PY
