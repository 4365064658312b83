#!/bin/bash
# Round 6 second GPU pass: plugin/sample diagnostic (new vs r05 library), the C2 bench under rocprofv3 --kernel-trace
# (chain on, --probe none) reconciled with its own clock, then the vendor counter side-by-side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06b}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=r06b/diag bash tools/gpu_diag_plugin.sh > $O/diag.log 2>&1 || { echo "diag failed"; tail -20 $O/diag.log; exit 1; }
cat $O/diag.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python bench.py --steps 8 --warmup 1 --probe none --no-cpu-baseline --no-vocos > $O/bench_traced.log 2>&1 \
  || { echo "traced bench failed"; tail -5 $O/bench_traced.log; exit 1; }
tail -1 $O/bench_traced.log > $O/bench_traced_line.json
python tools/trace_overlap.py $O/tr/run_kernel_trace.csv $O/bench_traced_line.json $O/trace_overlap_c2.json | head -40
find $O/tr -name "*_kernel_trace.csv" -delete
OUT=r06b/vpmc bash tools/gpu_vendor_pmc.sh || exit 1
