#!/bin/bash
# GPU suite with the prologue graph (default), then an interleaved C2 A/B against F5H_PROLOGUE_GRAPH=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/pg; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pg/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"
tail -8 gpurun_out/pg/gputest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/pg/bench_on_$i.log 2>&1 || exit 1
  F5H_PROLOGUE_GRAPH=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/pg/bench_off_$i.log 2>&1 || exit 1
done
for f in gpurun_out/pg/bench_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pg -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/pg/bench_tr.log 2>&1 || exit 1
python tools/call_gaps.py gpurun_out/pg/run_results.db > gpurun_out/pg/call_gaps.txt && tail -5 gpurun_out/pg/call_gaps.txt
