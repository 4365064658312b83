#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE) over 3 C2 calls -> per-class HBM bytes (tools/pmc_classes.py).
# Step graphs off (F5H_GRAPH=0): the PMC pass over graph-replayed dispatches crashed rocprofv3 on
# this pool (SIGSEGV in the tool after HSA init); eager and graph launches are the same kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp F5H_GRAPH=0
O=$PWD/gpurun_out/pmc_c2; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python tools/trace_c2.py run > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python tools/pmc_classes.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv \
  $O/r02_pmc_classes.json && echo "pmc ok"
