#!/bin/bash
# Round 3 GPU pass O: K32-stage deep-ring tiles (cfg 6: 192x128 x4 stages, 7: 128x128 x5, 8: 128x128 x4)
# against the K64 forms: every-tile-config bitwise tests, op-level timing at the C2 and C3 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -x --timeout 200 --timeout-method thread -k "tile_config" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
GT_CFGS=0,1,5,6,7,8 GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2,c3_qkv,c3_ffn2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/gt -o run -- python tools/gemm_tune.py > $O/gt.log 2>&1 || { echo "tune failed"; exit 1; }
GT_CFGS=0,1,5,6,7,8 GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2,c3_qkv,c3_ffn2 python tools/gemm_tune.py --report $O/gt/run_kernel_trace.csv | tee $O/gemm_tune_k32.txt
