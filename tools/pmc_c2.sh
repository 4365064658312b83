#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE) over C2 calls (or C3/C4/C5: second argument) in the shipped graph mode -> per-class HBM bytes
# (tools/pmc_classes.py). rocprofv3 of this ROCm build dies with SIGSEGV after ~12-16k
# graph-launched dispatches whatever the program (tools/probes/launch_cost count reproduces it
# with empty kernels), so each pass makes 3 calls (~8k dispatches): 1 warm + 2 marked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
O=$PWD/gpurun_out/pmc_${2:-c2}; mkdir -p $O
OUT=${1:-$O/r03_pmc_classes.json}
CFG=${2:-c2}
# C3/C4/C5: graph-mode passes at the batch shapes never finish under the profiler (tools/r04_gpu_a.sh,
# r04_gpu_b.sh, r04_gpu_x.sh): ONE eager call (F5H_GRAPH=0) -- the same kernels, launched one by one
[ "$CFG" != c2 ] && export F5H_GRAPH=0 F5H_TRACE_WARM=0 F5H_TRACE_CALLS=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/${CFG}_$c -o run -- \
    python tools/trace_c2.py run $CFG > $O/pmc_${CFG}_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python tools/pmc_classes.py $O/${CFG}_FETCH_SIZE/run_counter_collection.csv \
  $O/${CFG}_WRITE_SIZE/run_counter_collection.csv $OUT $CFG || exit 1
echo "pmc ok"
[ -n "$KEEP_CSV" ] || find $O -name "*_counter_collection.csv" -delete
