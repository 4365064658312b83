#!/bin/bash
# Round 3 GPU pass C: host-stall diagnostic, profiler dispatch-count threshold, full GPU suite with the
# UNetT 16-bit residual / typed views / plugin cache changes (envelopes logged).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03c; export TMPDIR=/tmp
timeout -k 10 120 python tools/host_stall_probe.py > gpurun_out/r03c/host_stall.log 2>&1; echo "stall probe rc=$?"; cat gpurun_out/r03c/host_stall.log | tail -12
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03c/cnt150 -o c -- ./tools/probes/launch_cost count 150 400 > gpurun_out/r03c/count150.log 2>&1; echo "count150 rc=$?"; grep "\[count\]" gpurun_out/r03c/count150.log | tail -1
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03c/cnt10 -o c -- ./tools/probes/launch_cost count 10 4000 > gpurun_out/r03c/count10.log 2>&1; echo "count10 rc=$?"; grep "\[count\]" gpurun_out/r03c/count10.log | tail -1
export F5H_ENVELOPE_LOG=$PWD/gpurun_out/r03c/envelopes.jsonl; rm -f $F5H_ENVELOPE_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread > gpurun_out/r03c/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "C2 bf16|passed|failed|FAILED" gpurun_out/r03c/gputest.log | tail -12
cat $F5H_ENVELOPE_LOG
exit $rc
