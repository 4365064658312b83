#!/bin/bash
# LayerNorm-fold parity tests, then a kernel-time profile of the C2 bench with the fold on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/lnf2; export TMPDIR=/tmp
F5H_LNFOLD=1 timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/lnf2/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"
tail -6 gpurun_out/lnf2/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
F5H_LNFOLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lnf2 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnf2/bench.log 2>&1 || exit 1
python tools/rocpd_top.py gpurun_out/lnf2/run_results.db 10
