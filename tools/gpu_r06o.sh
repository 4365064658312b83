#!/bin/bash
# fold statistics pinned (LNF 2 == LNF 3 bitwise): fold tile-config test, envelopes, contract tests, one-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06o}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "ln_fold or tile_config" tests/test_gpu_envelope.py -q -rf --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --rounds 4 --calls 4 --arms fold0,fold1 > $O/ab_fold_bf16.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_bf16.log
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --compute fp16 --rounds 3 --calls 4 --arms fold0,fold1 > $O/ab_fold_fp16.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_fp16.log
