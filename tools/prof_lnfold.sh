#!/bin/bash
# Kernel-time summary of the C2 bench with the LayerNorm fold on (F5H_LNFOLD=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/lnfp; export TMPDIR=/tmp
export F5H_LNFOLD=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lnfp -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vocos --probe none > gpurun_out/lnfp/bench.log 2>&1 || exit 1
f=$(ls gpurun_out/lnfp/*/run_kernel_stats.csv gpurun_out/lnfp/run_kernel_stats.csv 2>/dev/null | head -1); cp "$f" gpurun_out/lnfp/stats.csv
head -14 gpurun_out/lnfp/stats.csv | cut -c1-200
