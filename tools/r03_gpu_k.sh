#!/bin/bash
# Round 3 GPU pass K: the two-tile pipelined attention with tiles staged three ahead in a 4-slot ring
# (F5H_ATTN_PIPE=1) against attn16_kernel: attention/sample tests with it, interleaved C2 benches with
# attention probed live.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03k; mkdir -p $O; export TMPDIR=/tmp
F5H_ATTN_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -x --timeout 120 --timeout-method thread -k "attention or c2 or sample_fp32 or masked" > $O/pipe_tests.log 2>&1; rc=$?
echo "pipe tests rc=$rc"; tail -3 $O/pipe_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/base_$i.log 2>&1 || exit 1
  F5H_ATTN_PIPE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/pipe_$i.log 2>&1 || exit 1
done
for f in $O/base_*.log $O/pipe_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms/call; attention", r.get("avg_launch_us"), "us, frac", r.get("frac"))')"; done | tee $O/ab.txt
