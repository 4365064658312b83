#!/bin/bash
# Round 3 GPU pass S: the input projection (EPI_INPROJ) on the fast epilogue, proj_out over all 128 padded
# columns (fast epilogue too): the GPU suite, then interleaved C2 benches against the previous build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03s; mkdir -p $O; export TMPDIR=/tmp
BASE=$PWD/f5-tts_amd/f5_tts_amd/lib/libf5h_base.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -5
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  F5H_LIB=$BASE timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/new_$i.log 2>&1 || exit 1
done
for f in $O/base_*.log $O/new_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/call")')"; done | tee $O/ab.txt
