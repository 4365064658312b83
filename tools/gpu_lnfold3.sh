#!/bin/bash
# LayerNorm-fold parity tests, interleaved C2 A/B (fold off/on), then a kernel-time profile with it on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/lnf3; export TMPDIR=/tmp
F5H_LNFOLD=1 timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/lnf3/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"
tail -4 gpurun_out/lnf3/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf3/bench_off_$i.log 2>&1 || exit 1
  F5H_LNFOLD=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf3/bench_on_$i.log 2>&1 || exit 1
done
for f in gpurun_out/lnf3/bench_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
F5H_LNFOLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lnf3 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf3/bench.log 2>&1 || exit 1
python tools/rocpd_top.py gpurun_out/lnf3/run_results.db 8
