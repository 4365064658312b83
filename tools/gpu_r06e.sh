#!/bin/bash
# LayerNorm fold: envelope tests (C2/C1 bf16 and fp16 fold on by default), the chain/plugin tests, then a one-box
# interleaved A/B of the fold at C2 (bf16, fp16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06e}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
F5H_ENVELOPE_LOG=$O/envelopes.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_envelope.py -q -rf -s --timeout 200 \
  --timeout-method thread > $O/envelope.log 2>&1; rc=$?
grep -E "envelope|passed|failed|Error" $O/envelope.log | head -30
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --rounds 4 --calls 4 --arms fold0,fold1 > $O/ab_fold_bf16.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_bf16.log
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --compute fp16 --rounds 3 --calls 4 --arms fold0,fold1 > $O/ab_fold_fp16.log 2>&1 || exit 1
grep -v amdgpu $O/ab_fold_fp16.log
exit $rc
