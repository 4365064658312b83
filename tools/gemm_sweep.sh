#!/bin/bash
# A/B the GEMM tile/stage variants: op-level + forward parity, then a short C2 bench each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2 3 4}; do
  F5H_GEMM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x \
      -k "linear or forward or sample_fp32" > gpurun_out/sweep_t$v.log 2>&1 || { echo "variant $v tests FAILED"; tail -5 gpurun_out/sweep_t$v.log; exit 1; }
  F5H_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --probe-all ${BENCH_ARGS} \
      > gpurun_out/sweep_b$v.log 2> gpurun_out/sweep_p$v.log || { echo "variant $v bench FAILED"; tail -5 gpurun_out/sweep_b$v.log; exit 1; }
  grep probe gpurun_out/sweep_p$v.log || tail -5 gpurun_out/sweep_p$v.log; echo "variant $v: $(tail -1 gpurun_out/sweep_b$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
