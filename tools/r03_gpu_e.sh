#!/bin/bash
# Round 3 GPU pass E: register-staged attention (T14) + widened epilogue (T21) against the LDS-DMA
# kernel (F5H_ATTN_STAGE=dma): attention tests, then interleaved C2 benches with the attention class
# probed live.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03e; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "attention or c2 or spike or sample_fp32" > gpurun_out/r03e/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r03e/gputest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > gpurun_out/r03e/rs_$i.log 2>&1 || exit 1
  F5H_ATTN_STAGE=dma timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > gpurun_out/r03e/dma_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r03e/rs_*.log gpurun_out/r03e/dma_*.log; do echo "$f $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r.get("avg_launch_us"), r.get("frac"))')"; done
