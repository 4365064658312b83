#!/bin/bash
# Round 6 after the chain fix (chain off by default): whole GPU suite, smoke, C2 bench line, the C2 bench under
# rocprofv3 --kernel-trace reconciled with its own clock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06d}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
OUT=${OUT:-r06d} MAXFAIL=3 KEEP_GOING=1 CONFIGS=c2 bash tools/gpu_suite.sh || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python bench.py --steps 8 --warmup 1 --probe none --no-cpu-baseline --no-vocos > $O/bench_traced.log 2>&1 \
  || { echo "traced bench failed"; tail -5 $O/bench_traced.log; exit 1; }
grep "^{\"metric\"" $O/bench_traced.log | tail -1 > $O/bench_traced_line.json
python tools/trace_overlap.py $O/tr/run_kernel_trace.csv $O/bench_traced_line.json $O/trace_overlap_c2.json | head -30
find $O/tr -name "*_kernel_trace.csv" -delete
