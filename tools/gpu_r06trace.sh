#!/bin/bash
# The C2 bench command under rocprofv3 --kernel-trace, reconciled with its own clock (tools/trace_overlap.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06trace}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python bench.py --steps 8 --warmup 1 --probe none --no-cpu-baseline --no-vocos > $O/bench_traced.log 2>&1 \
  || { echo "traced bench failed"; tail -5 $O/bench_traced.log; exit 1; }
grep "^{\"metric\"" $O/bench_traced.log | tail -1 > $O/bench_traced_line.json
python tools/trace_overlap.py $O/tr/run_kernel_trace.csv $O/bench_traced_line.json $O/trace_overlap_c2.json | head -40
find $O/tr -name "*_kernel_trace.csv" -delete
