#!/bin/bash
# Round artifacts: C2 bench (with CPU baseline and +Vocos), C3/C5 bench lines, rocprof kernel stats
# and the attention PMC traffic (tools/profile_round.sh). Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${R}_bench.log 2>&1 && echo "c2 ok" \
&& timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > gpurun_out/${R}_bench_c3.log 2>&1 && echo "c3 ok" \
&& timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos > gpurun_out/${R}_bench_c5.log 2>&1 && echo "c5 ok" \
&& ROUND=$R bash tools/profile_round.sh > gpurun_out/${R}_profile.log 2>&1 && echo "prof ok"
rc=$?
for f in gpurun_out/${R}_bench.log gpurun_out/${R}_bench_c3.log gpurun_out/${R}_bench_c5.log; do tail -1 $f | cut -c1-400; done
exit $rc
