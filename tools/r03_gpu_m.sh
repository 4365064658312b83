#!/bin/bash
# Round 3 GPU pass M: the branch-free fast epilogue (buffer-descriptor stores, raw-bit row fetch, also on
# the 256x256 ping-pong kernel): GPU suite, C3 timelines and GEMM shapes, then C2/C3/C5 benches A/B
# against the previous build (libf5h_base.so), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03m; mkdir -p $O; export TMPDIR=/tmp
BASE=$PWD/f5-tts_amd/f5_tts_amd/lib/libf5h_base.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/timeline_c2.py --config c3 > $O/timeline_c3.log 2>&1; echo "timeline rc=$?"; tail -7 $O/timeline_c3.log
for i in 1 2; do
  F5H_LIB=$BASE timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/c2_base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/c2_new_$i.log 2>&1 || exit 1
done
F5H_LIB=$BASE timeout -k 10 400 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c3_base.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c3_new.log 2>&1 || exit 1
F5H_LIB=$BASE timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c5_base.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c5_new.log 2>&1 || exit 1
for f in $O/c2_*.log $O/c3_*.log $O/c5_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"; done | tee $O/ab.txt
