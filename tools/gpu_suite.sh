#!/bin/bash
# GPU parity suite + smoke + quick C2 / C3 bench lines (no CPU baseline, no Vocos) into gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-suite}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=${MAXFAIL:-1} --timeout 300 --timeout-method thread \
  > $O/gputest.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/gputest.log
# go on past plain test failures (rc 1) only: a timeout, a crash or a GPU fault ends the call here
if [ $rc -ne 0 ]; then
  [ $rc -eq 1 ] && [ -n "$KEEP_GOING" ] && ! grep -qE "Timeout|Fatal Python|Memory access fault|hipError|core dumped" $O/gputest.log \
    || exit $rc
fi
timeout -k 10 240 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
for c in ${CONFIGS:-c2 c3}; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline --no-vocos ${BENCH_ARGS} > $O/bench_$c.log 2>&1 \
    && echo "$c $(tail -1 $O/bench_$c.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], d["value"], r["kernel"], r["frac"])')" || exit 1
done
