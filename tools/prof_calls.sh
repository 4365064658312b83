#!/bin/bash
# Kernel trace of the default C2 bench (probe off), summarised per call by tools/call_gaps.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/cg; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/cg -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/cg/bench.log 2>&1 || exit 1
python tools/call_gaps.py gpurun_out/cg/run_results.db > gpurun_out/cg/call_gaps.txt && cat gpurun_out/cg/call_gaps.txt
