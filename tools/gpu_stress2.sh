#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-stress2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python tools/stress_chain2.py 2>&1 | grep -v amdgpu.ids | tee $O/out.log
