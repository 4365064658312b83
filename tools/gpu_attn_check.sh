#!/bin/bash
# Attention A/B on one box: parity tests of the default kernel, then kernel-trace timing of both
# variants (F5H_ATTN=0: 8-wave attn16_kernel, 1: one-wave-per-SIMD attn_pw_kernel) at the C2 shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/attn_time.py > gpurun_out/at1.log 2>&1 && echo "at1 ok" \
&& timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1 && echo "attn tests ok" \
&& F5H_ATTN=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/at0 -o run -- python tools/attn_time.py > gpurun_out/at0p.log 2>&1 && echo "prof0 ok" \
&& F5H_ATTN=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/at1 -o run -- python tools/attn_time.py > gpurun_out/at1p.log 2>&1 && echo "prof1 ok" \
&& ( [ -z "$FULL" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 ) && echo "done"
rc=$?
cat gpurun_out/at1.log; tail -3 gpurun_out/t_attn.log; [ -z "$FULL" ] || tail -3 gpurun_out/gpu_tests.log
exit $rc
