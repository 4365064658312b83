#!/bin/bash
# Round 3 GPU pass Y: the CFG-chain split at C3 and C4 (default split for B >= 4) vs F5H_SPLIT_CFG=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03y; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for c in c4 c3; do
    timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/${c}_split_$i.log 2>&1 || exit 1
    F5H_SPLIT_CFG=0 timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/${c}_packed_$i.log 2>&1 || exit 1
  done
done
for f in $O/c4_*.log $O/c3_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/call")')"; done | tee $O/ab.txt
