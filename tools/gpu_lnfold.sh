#!/bin/bash
# GPU tests with the LayerNorm fold on (F5H_LNFOLD=1), then an interleaved A/B of the C2 bench, fold off/on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/lnf; export TMPDIR=/tmp
F5H_LNFOLD=1 timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/lnf/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"
tail -15 gpurun_out/lnf/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf/bench_off_$i.log 2>&1 || exit 1
  F5H_LNFOLD=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf/bench_on_$i.log 2>&1 || exit 1
done
for f in gpurun_out/lnf/bench_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
exit $rc
