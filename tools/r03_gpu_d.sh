#!/bin/bash
# Round 3 GPU pass D: eviction-stall trace, C2 kernel timelines, graph-mode PMC passes, re-run of
# the changed tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03d; export TMPDIR=/tmp
F5H_HOST_TRACE=1 timeout -k 10 120 python tools/host_stall_probe.py evict > gpurun_out/r03d/evict.log 2>&1; echo "evict rc=$?"
grep -v "^\[f5h host\] graph_get kind 0: lock 0.0" gpurun_out/r03d/evict.log | tail -25
timeout -k 10 300 python tools/timeline_c2.py > gpurun_out/r03d/timeline_c2.log 2>&1; echo "timeline rc=$?"; cat gpurun_out/r03d/timeline_c2.log | tail -8
timeout -k 10 600 ./tools/pmc_c2.sh gpurun_out/r03d/r03_pmc_classes.json > gpurun_out/r03d/pmc.log 2>&1; echo "pmc rc=$?"; tail -3 gpurun_out/r03d/pmc.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_contract.py tests/test_gpu_envelope.py -m gpu -q -rf -s --timeout 300 --timeout-method thread -k "plugin or envelope or eviction" > gpurun_out/r03d/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "C2 bf16|passed|failed|FAILED" gpurun_out/r03d/gputest.log | tail -8
exit $rc
