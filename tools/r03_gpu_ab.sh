#!/bin/bash
# Round 3 GPU pass AB: attention K/V ring depth 4 (committed build, and the same depth after the
# generalisation), 5 and 6 slots (DMA NS-1 tiles ahead): bitwise checks, interleaved C2 benches
# (attention probed live), attention tests on the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03ab; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -x -k "attention or attn" --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1; rc=$?
echo "attn tests rc=$rc"; grep -E "passed|failed" $O/attn_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for v in base new r5 r6; do
  lib=$L/libf5h.so; [ $v != new ] && lib=$L/libf5h_$v.so
  F5H_LIB=$lib timeout -k 10 120 python tools/diag_lib_bitwise.py $O/bit_$v.npy >> $O/bit.log 2>&1 || exit 1
done
python -c "
import numpy as np
a=np.load('$O/bit_base.npy')
for v in ('new','r5','r6'):
    b=np.load('$O/bit_'+v+'.npy'); print(v, 'bitwise identical to the committed build:', bool((a.view(np.uint32)==b.view(np.uint32)).all()))
" | tee $O/bitwise.txt
for i in 1 2; do
  for v in base new r5 r6; do
    lib=$L/libf5h.so; [ $v != new ] && lib=$L/libf5h_$v.so
    F5H_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe attention > $O/${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/base_*.log $O/new_*.log $O/r5_*.log $O/r6_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms/call; attention", r.get("avg_launch_us"), "us, frac", r.get("frac"))')"; done | tee $O/ab.txt
