#!/bin/bash
# Round 3 GPU pass G (baseline at HEAD after the container restore): the GPU suite with envelopes
# logged, the default bench line, a kernel trace of C2 calls (graph mode), the graph-mode PMC passes,
# and the LayerNorm-launch bound (F5H_DIAG_SKIP_LN=1, timing only) interleaved with the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/intake 8 > $O/intake_8mb.log 2>&1 && timeout -k 10 60 ./tools/probes/intake 64 > $O/intake_64mb.log 2>&1 || exit 1
cat $O/intake_8mb.log $O/intake_64mb.log
export F5H_ENVELOPE_LOG=$PWD/$O/envelopes.jsonl; rm -f $F5H_ENVELOPE_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
unset F5H_ENVELOPE_LOG
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 1
tail -1 $O/bench_c2.log | cut -c1-400
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/trace -o run -- \
  python tools/trace_c2.py run > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python tools/trace_c2.py report $O/trace/run_kernel_trace.csv > $O/r03_c2_kernels.txt; head -20 $O/r03_c2_kernels.txt
unset F5H_TRACE_WARM F5H_TRACE_CALLS
timeout -k 10 600 ./tools/pmc_c2.sh $PWD/$O/r03_pmc_classes.json > $O/pmc.log 2>&1; echo "pmc rc=$?"; tail -3 $O/pmc.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/base_$i.log 2>&1 || exit 1
  F5H_DIAG_SKIP_LN=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/noln_$i.log 2>&1 || exit 1
done
for f in $O/base_*.log $O/noln_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
