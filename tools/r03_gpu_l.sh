#!/bin/bash
# Round 3 GPU pass L: large-batch GEMMs (C3/C4/C5 run thousands of tiles per launch): per-workgroup
# timelines of the C3 classes, op-level timing of the C3 GEMM shapes per tile configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/timeline_c2.py --config c3 > $O/timeline_c3.log 2>&1; echo "timeline rc=$?"; tail -8 $O/timeline_c3.log
GT_CFGS=0,1,5,11 GT_SHAPES=c3_qkv,c3_ffn2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/gt -o run -- python tools/gemm_tune.py > $O/gt.log 2>&1 || { echo "tune failed"; exit 1; }
GT_CFGS=0,1,5,11 GT_SHAPES=c3_qkv,c3_ffn2 python tools/gemm_tune.py --report $O/gt/run_kernel_trace.csv | tee $O/gemm_tune_c3.txt
