#!/bin/bash
# Round 4, box g: fp16 epilogue rounding pinned (rounded()): bf16/E2 bit for bit against the previous build,
# fp16 per segment; then the full GPU suite and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04g; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_base.npy base > $O/bw_prev.log 2>&1 || exit 1
timeout -k 10 300 python tools/diag_lib_bitwise.py $O/new_base.npy base > $O/bw_new.log 2>&1 || exit 1
python -c "
import numpy as np
a=np.load('$O/prev_base.npy').view(np.uint32); b=np.load('$O/new_base.npy').view(np.uint32)
for name,s,e in (('F5 bf16',0,120000),('F5 fp16',120000,240000),('E2 bf16',240000,288000)):
    print(name, 'differing:', int((a[s:e]!=b[s:e]).sum()))
"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests rc=$?"; tail -3 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 $O/smoke.log
