#!/bin/bash
# GPU tests, then an interleaved A/B of the C2 bench with the 16-bit residual (default) and F5H_RES32=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r16; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/r16/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"
tail -4 gpurun_out/r16/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r16/bench_r16_$i.log 2>&1 || exit 1
  F5H_RES32=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r16/bench_r32_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r16/bench_r*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
exit $rc
