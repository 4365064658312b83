#!/bin/bash
# Round-2 closing artifacts on one box: GPU tests, smoke, C2 bench (CPU baseline, +Vocos), C2 fp16,
# C3/C4/C5 bench lines, then the kernel-trace + PMC profile (tools/profile_r02.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 && echo "tests ok" \
&& timeout -k 10 240 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_c2.log 2>&1 && echo "c2 ok" \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 3 --compute fp16 --no-cpu-baseline --no-vocos > $O/bench_c2_fp16.log 2>&1 && echo "c2 fp16 ok" \
&& timeout -k 10 400 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c3.log 2>&1 && echo "c3 ok" \
&& timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c4.log 2>&1 && echo "c4 ok" \
&& timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos > $O/bench_c5.log 2>&1 && echo "c5 ok" \
&& ROUND=r02 timeout -k 10 900 bash tools/profile_r02.sh > $O/profile.log 2>&1 && echo "profile ok"
rc=$?
tail -2 $O/gputest.log; for f in $O/bench_*.log; do tail -1 $f | cut -c1-200; done
exit $rc
