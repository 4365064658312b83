#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-stress3}; mkdir -p $O; export TMPDIR=/tmp
run() { env "$@" STRESS_SHORT=1 timeout -k 10 200 python tools/stress_chain2.py 2>&1 | grep -v amdgpu.ids | tee -a $O/out.log; }
run STRESS_TAG=default
run STRESS_TAG=no-prologue-graph F5H_PROLOGUE_GRAPH=0
run STRESS_TAG=split-cfg-never F5H_SPLIT_CFG=0
