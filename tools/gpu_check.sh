#!/bin/bash
# One GPU verification pass: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
timeout -k 10 420 python -m pytest tests -m gpu -q -rf -x > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" \
&& timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 && echo "bench ok" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
     python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 && echo "prof ok"
rc=$?
tail -3 gpurun_out/gpu_tests.log
tail -1 gpurun_out/bench.log
exit $rc
