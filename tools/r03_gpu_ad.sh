#!/bin/bash
# Round 3 GPU pass AD: attention prologue issues Q between the first and the next two K/V tiles (one counted wait):
# bitwise check, attention tests, interleaved C2 benches against the previous build (attention probed
# attention probed live), then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03ad; mkdir -p $O; export TMPDIR=/tmp
BASE=$PWD/f5-tts_amd/f5_tts_amd/lib/libf5h_base.so
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -x -k "attention or attn" --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1; rc=$?
echo "attn tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/attn_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
F5H_LIB=$BASE timeout -k 10 120 python tools/diag_lib_bitwise.py $O/bit_base.npy > $O/bit.log 2>&1 && timeout -k 10 120 python tools/diag_lib_bitwise.py $O/bit_new.npy >> $O/bit.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('$O/bit_base.npy'); b=np.load('$O/bit_new.npy'); print('bitwise identical to the previous build:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()), 'max abs diff', float(np.abs(a-b).max()))" | tee $O/bitwise.txt
for i in 1 2; do
  F5H_LIB=$BASE timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos > $O/base_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos > $O/new_$i.log 2>&1 || exit 1
done
for f in $O/base_*.log $O/new_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms/call; attention", r.get("avg_launch_us"), "us, frac", r.get("frac"))')"; done | tee $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8
