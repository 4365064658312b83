#!/bin/bash
# chain fix check: the chain tests (graph replays included) and the plugin C2 test, then a one-box interleaved
# A/B of the chain at C2 (bf16 and fp16), outputs compared on replayed calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06c}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_contract.py -q -rf -s -x --timeout 200 --timeout-method thread \
  -k "phase_chain or plugin_euler_loop_c2" > $O/chain_tests.log 2>&1; rc=$?
grep -E "concurrent chains|C2 bf16|passed|failed|Error" $O/chain_tests.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --rounds 5 --calls 4 --arms chain0,chain1 > $O/ab_chain_bf16.log 2>&1 || exit 1
cat $O/ab_chain_bf16.log
timeout -k 10 400 python -u tools/ab_c2.py --config c2 --compute fp16 --rounds 3 --calls 4 --arms chain0,chain1 > $O/ab_chain_fp16.log 2>&1 || exit 1
cat $O/ab_chain_fp16.log
