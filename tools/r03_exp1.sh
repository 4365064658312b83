#!/bin/bash
# Round 3, experiment 1: launch cost inside a replayed graph, and the C2 bound for removing the
# LayerNorm launches (F5H_DIAG_SKIP_LN=1, timing only), interleaved with the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03e1; export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/launch_cost > gpurun_out/r03e1/launch_cost.log 2>&1 || exit 1
cat gpurun_out/r03e1/launch_cost.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03e1/lc -o lc -- ./tools/probes/launch_cost > gpurun_out/r03e1/launch_cost_prof.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r03e1/base_$i.log 2>&1 || exit 1
  F5H_DIAG_SKIP_LN=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > gpurun_out/r03e1/noln_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r03e1/base_*.log gpurun_out/r03e1/noln_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done
