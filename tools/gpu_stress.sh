#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-stress}; mkdir -p $O; export TMPDIR=/tmp
echo "== new lib"; timeout -k 10 240 python tools/stress_chain.py 2>&1 | grep -v amdgpu.ids | tee $O/new.log || exit 1
echo "== new lib, fp32 params"; STRESS_BF16_PARAMS=0 timeout -k 10 240 python tools/stress_chain.py 2>&1 | grep -v amdgpu.ids | tee $O/new_f32p.log || exit 1
