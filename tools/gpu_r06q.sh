#!/bin/bash
# UNetT RMSNorm fold: fold tests, envelopes, the whole GPU suite, then a one-box A/B at C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06q}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fold" -q -rf --timeout 300 --timeout-method thread \
  > $O/fold_tests.log 2>&1; rc=$?
tail -4 $O/fold_tests.log
[ $rc -eq 0 ] || exit $rc
F5H_ENVELOPE_LOG=$O/envelopes.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_envelope.py -q -rf -s --timeout 200 \
  --timeout-method thread > $O/envelope.log 2>&1; rc=$?
grep -E "envelope|passed|failed|Error" $O/envelope.log | head -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_c2.py --config c5 --rounds 3 --calls 2 --arms fold0,fold1 > $O/ab_fold_c5.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_c5.log
