#!/bin/bash
# Round 3 GPU pass Z: persistent ping-pong GEMM blocks (next tile's operands prefetched under the epilogue)
# for the large-batch GEMMs: GEMM tests, interleaved C4/C3/C5 benches against F5H_GEMM_PERSIST=0 (one block
# per tile, same library), then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03z; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -x -k "linear" --timeout 200 --timeout-method thread > $O/gemm_tests.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gemm_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in c4 c3 c5; do
    st=2; [ $c = c5 ] && st=3
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/${c}_persist_$i.log 2>&1 || exit 1
    F5H_GEMM_PERSIST=0 timeout -k 10 300 python bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/${c}_grid_$i.log 2>&1 || exit 1
  done
done
for f in $O/c4_*.log $O/c3_*.log $O/c5_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/call")')"; done | tee $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8
