#!/bin/bash
# Round-6 final checks on one box: the whole GPU suite + smoke, then the C2 per-class profiles at this build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06final}; mkdir -p $O; export TMPDIR=/tmp
OUT=${OUT:-r06final} MAXFAIL=5 KEEP_GOING=1 CONFIGS=c2 bash tools/gpu_suite.sh || exit 1
F5H_HEAD=${F5H_HEAD:-unknown} PREFIX=r06 OUT=${OUT:-r06final}_prof CONFIGS=c2 CHAIN_TRACE=0 bash tools/gpu_profiles.sh || exit 1
