#!/bin/bash
# Round 3 GPU pass Q: do a wave's MFMAs and its SIMD partner's VALU work overlap on gfx950? (coexec probe)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 120 ./tools/probes/coexec > $O/coexec.log 2>&1; rc=$?; cat $O/coexec.log; exit $rc
