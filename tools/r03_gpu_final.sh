#!/bin/bash
# Round 3 final artifacts at HEAD on one box (VALU row sums, 4-slot attention ring, Q between the first K/V tiles, one packed CFG chain): smoke, default bench line (CPU baseline, +Vocos), C2 fp16, C3 / C4
# (per rank) / C5 bench lines, kernel trace of C2 calls, graph-mode PMC classes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03f3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed" $O/gputest.log | tail -3
timeout -k 10 240 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 && echo "c2 ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compute fp16 --no-cpu-baseline --no-vocos > $O/bench_c2_fp16.log 2>&1 && echo "c2 fp16 ok" \
&& timeout -k 10 400 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c3.log 2>&1 && echo "c3 ok" \
&& timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c4.log 2>&1 && echo "c4 ok" \
&& timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c5.log 2>&1 && echo "c5 ok" || exit 1
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/trace -o run -- \
  python tools/trace_c2.py run > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
python tools/trace_c2.py report $O/trace/run_kernel_trace.csv > $O/r03_c2_kernels.txt; head -20 $O/r03_c2_kernels.txt
unset F5H_TRACE_WARM F5H_TRACE_CALLS
timeout -k 10 600 ./tools/pmc_c2.sh $PWD/$O/r03_pmc_classes.json > $O/pmc.log 2>&1; echo "pmc rc=$?"
for f in $O/bench_*.log; do echo "$(basename $f) $(tail -1 $f | cut -c1-150)"; done
