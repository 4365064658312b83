#!/bin/bash
# Round 6 first GPU pass: the new chain tests first, then the whole GPU suite, smoke, the C2 bench line (chain class
# probed) and the same-node PyTorch yardstick, into gpurun_out/${OUT:-r06a}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-r06a}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_contract.py -q -rf -s -x --timeout 120 --timeout-method thread \
  -k "phase_chain or eviction" > $O/chain_tests.log 2>&1 || { echo "chain tests failed"; tail -30 $O/chain_tests.log; exit 1; }
grep -E "concurrent chains|passed|failed" $O/chain_tests.log
OUT=${OUT:-r06a} MAXFAIL=3 KEEP_GOING=1 CONFIGS=c2 bash tools/gpu_suite.sh || exit 1
timeout -k 10 300 python -u tools/torch_path.py --out $O/torch_path_c2.json > $O/torch_path.log 2>&1 || { tail -20 $O/torch_path.log; exit 1; }
head -3 $O/torch_path.log
