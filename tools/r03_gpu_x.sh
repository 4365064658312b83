#!/bin/bash
# Round 3 GPU pass X: re-measure the CFG-chain split with the round-3 kernels: C2 (default one packed
# chain) vs F5H_SPLIT_CFG=1 (cond/uncond as two concurrent chains), C5 (default split) vs F5H_SPLIT_CFG=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03x; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/c2_packed_$i.log 2>&1 || exit 1
  F5H_SPLIT_CFG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/c2_split_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c5_split_$i.log 2>&1 || exit 1
  F5H_SPLIT_CFG=0 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c5_packed_$i.log 2>&1 || exit 1
done
for f in $O/c2_*.log $O/c5_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/call")')"; done | tee $O/ab.txt
