#!/bin/bash
# Round-2 profile artifacts (run on the GPU box; copy gpurun_out/prof_<R>/ summaries into profiles/):
#   1. rocprofv3 --kernel-trace --stats of 3 C2 CFM.sample calls (tools/trace_c2.py) -> per-kernel table
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE; one counter block each, MI355X_MICROARCH.md PMC slots)
#      over the same calls -> per-class HBM bytes per launch (tools/pmc_classes.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r02}
O=$PWD/gpurun_out/prof_$R
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python tools/trace_c2.py run > $O/trace.log 2>&1 || exit 1
python tools/trace_c2.py report $O/trace/run_kernel_trace.csv > $O/${R}_c2_kernels.txt || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python tools/trace_c2.py run > $O/pmc_$c.log 2>&1 || exit 1
done
python tools/pmc_classes.py $O/FETCH_SIZE/run_counter_collection.csv $O/WRITE_SIZE/run_counter_collection.csv \
  $O/${R}_pmc_classes.json > /dev/null || exit 1
cat $O/${R}_c2_kernels.txt
