#!/bin/bash
# Bench lines of C2 fp16 and C3/C4/C5 on one box (the configs other than the default C2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/cfgs; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compute fp16 --no-cpu-baseline --no-vocos > $O/bench_c2_fp16.log 2>&1 && echo "c2 fp16 ok" \
&& timeout -k 10 400 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c3.log 2>&1 && echo "c3 ok" \
&& timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c4.log 2>&1 && echo "c4 ok" \
&& timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c5.log 2>&1 && echo "c5 ok"
rc=$?
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
exit $rc
