#!/bin/bash
# equal-length batches as unmasked rows (the fold applies): DP / batch / parity tests, then one-box A/B at C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06p}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_envelope.py tests/test_gpu_parity.py -q -rf --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_c2.py --config c4 --rounds 3 --calls 2 --arms fold0,fold1 > $O/ab_fold_c4.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_c4.log
