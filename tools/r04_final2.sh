#!/bin/bash
# Round 4 final artifacts at the scalar-DMA HEAD, one box: GPU suite, then tools/r04_final.sh (smoke, C2 bf16 with
# CPU baseline and Vocos, C2 fp16, C1/C3/C4/C5, kernel trace of the default bench command).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${R04_FINAL:-r04final2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests rc=$?"; tail -2 $O/gputest.log
R04_OUT=${R04_FINAL:-r04final2} bash tools/r04_final.sh
