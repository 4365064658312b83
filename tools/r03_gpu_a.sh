#!/bin/bash
# Round 3 GPU pass A: the GPU suite (new envelope / C4 / graph-cache tests included, envelope values
# logged), then experiment 1 (launch cost, LayerNorm-launch bound).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03a; export TMPDIR=/tmp
export F5H_ENVELOPE_LOG=$PWD/gpurun_out/r03a/envelopes.jsonl
rm -f $F5H_ENVELOPE_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r03a/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/r03a/gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/r03_exp1.sh
