#!/bin/bash
# Round 3 GPU pass B: implicit-sync probe, the call a profiler crash happens in, the changed tests,
# and the LayerNorm-launch bound (F5H_DIAG_SKIP_LN=1, timing only) against the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03b; export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/launch_cost sync > gpurun_out/r03b/sync_probe.log 2>&1 || exit 1
cat gpurun_out/r03b/sync_probe.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b/lc -o lc -- ./tools/probes/launch_cost trace > gpurun_out/r03b/launch_cost_trace_prof.log 2>&1
echo "rocprof trace rc=$?"; grep -n "\[call\]" gpurun_out/r03b/launch_cost_trace_prof.log | tail -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_contract.py tests/test_gpu_parity.py -m gpu -q -rf -s --timeout 300 --timeout-method thread -k "graph or plugin or eviction" > gpurun_out/r03b/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "C2 bf16|passed|failed" gpurun_out/r03b/gputest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r03b/base_$i.log 2>&1 || exit 1
  F5H_DIAG_SKIP_LN=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r03b/noln_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r03b/base_*.log gpurun_out/r03b/noln_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
