#!/bin/bash
# Round 3 GPU pass J (HEAD: step bookkeeping folded into the Euler launch, residual prefetch behind
# the first stages): the GPU suite (envelopes logged), C2 timelines, the default bench line, a kernel
# trace of C2 calls, the graph-mode PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03j; mkdir -p $O; export TMPDIR=/tmp
export F5H_ENVELOPE_LOG=$PWD/$O/envelopes.jsonl; rm -f $F5H_ENVELOPE_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
unset F5H_ENVELOPE_LOG
timeout -k 10 300 python tools/timeline_c2.py > $O/timeline_c2.log 2>&1; echo "timeline rc=$?"; tail -7 $O/timeline_c2.log
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
tail -1 $O/bench_c2.log | cut -c1-700
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/trace -o run -- \
  python tools/trace_c2.py run > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python tools/trace_c2.py report $O/trace/run_kernel_trace.csv > $O/r03_c2_kernels.txt; head -24 $O/r03_c2_kernels.txt
unset F5H_TRACE_WARM F5H_TRACE_CALLS
timeout -k 10 600 ./tools/pmc_c2.sh $PWD/$O/r03_pmc_classes.json > $O/pmc.log 2>&1; echo "pmc rc=$?"; tail -3 $O/pmc.log
