#!/bin/bash
# Round 4, box n: GEMM tile configurations re-timed after the scalar-addressed DMA (tools/gemm_tune.py under a
# kernel trace), C2 / C3 / C5 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04n; mkdir -p $O; export TMPDIR=/tmp
export GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2,c3_qkv,c3_ffn1,c3_ffn2,c3_out,c5_qkv
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/gt -o run -- python tools/gemm_tune.py > $O/gt.log 2>&1 || exit 1
python tools/gemm_tune.py --report $O/gt/run_kernel_trace.csv > $O/report.txt 2>&1
cat $O/report.txt
