#!/bin/bash
# Round 4, box e: GPU suite after the conv XCD map, then the graph-mode FETCH/WRITE passes at C2
# (per-class HBM traffic: conv panel re-fetch) and a C2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04e; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" $O/gputest.log | tail -3
timeout -k 10 600 ./tools/pmc_c2.sh $O/r04_pmc_classes.json > $O/pmc.log 2>&1; echo "pmc rc=$?"
python -c "
import json; d=json.load(open('$O/r04_pmc_classes.json'))
for k,v in d['classes'].items(): print(k, v['hbm_over_algorithmic'], round(v['hbm_bytes']/1e6,1))"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-vocos > $O/bench_c2.log 2>&1 && tail -1 $O/bench_c2.log | cut -c1-200
