#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE) over C2 calls in the shipped graph mode -> per-class HBM bytes
# (tools/pmc_classes.py). rocprofv3 of this ROCm build dies with SIGSEGV after ~12-16k
# graph-launched dispatches whatever the program (tools/probes/launch_cost count reproduces it
# with empty kernels), so each pass makes 3 calls (~8k dispatches): 1 warm + 2 marked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
O=$PWD/gpurun_out/pmc_c2; mkdir -p $O
OUT=${1:-$O/r03_pmc_classes.json}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python tools/trace_c2.py run > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python tools/pmc_classes.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv \
  $OUT && echo "pmc ok"
