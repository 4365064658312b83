#!/bin/bash
# Round 3 GPU pass N: attention with both V^T halves read before the row max (their LDS latency under the
# max instead of in front of the first PV MFMA): attention tests, interleaved C2 benches with attention
# probed live against the previous build (libf5h_base.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03n; mkdir -p $O; export TMPDIR=/tmp
BASE=$PWD/f5-tts_amd/f5_tts_amd/lib/libf5h_base.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -x --timeout 120 --timeout-method thread -k "attention or c2 or sample_fp32 or masked" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  F5H_LIB=$BASE timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/new_$i.log 2>&1 || exit 1
done
for f in $O/base_*.log $O/new_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms/call; attention", r.get("avg_launch_us"), "us, frac", r.get("frac"))')"; done | tee $O/ab.txt
