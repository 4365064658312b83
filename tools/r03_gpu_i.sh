#!/bin/bash
# Round 3 GPU pass I: attention as two 4-wave workgroups per CU (F5H_ATTN_NW=4) against one 8-wave
# workgroup: attention tests with the variant, interleaved C2 benches with attention probed live,
# then the per-workgroup timelines of the C2 kernel classes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03i; mkdir -p $O; export TMPDIR=/tmp
F5H_ATTN_NW=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -x --timeout 120 --timeout-method thread -k "attention or c2 or sample_fp32 or masked" > $O/nw4_tests.log 2>&1; rc=$?
echo "nw4 tests rc=$rc"; tail -3 $O/nw4_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/nw8_$i.log 2>&1 || exit 1
  F5H_ATTN_NW=4 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/nw4_$i.log 2>&1 || exit 1
done
for f in $O/nw8_*.log $O/nw4_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r.get("avg_launch_us"), r.get("frac"))')"; done
timeout -k 10 300 python tools/timeline_c2.py > $O/timeline_c2.log 2>&1; echo "timeline rc=$?"; tail -12 $O/timeline_c2.log
