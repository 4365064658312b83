#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-stress4}; mkdir -p $O; export TMPDIR=/tmp
run() { env "$@" STRESS_SHORT=1 timeout -k 10 200 python tools/stress_chain2.py 2>&1 | grep -v amdgpu.ids | tee -a $O/out.log; }
run STRESS_TAG=zero-kernel
run STRESS_TAG=zero-memset F5H_CHAIN_ZERO=memset
