#!/bin/bash
# Round 4, box f: packed-fp32 epilogue math (RoPE + q scale, GELU-tanh): bit-for-bit against the previous build
# (libf5h_prev.so) at Base size, interleaved C2 A/B; C3 full-batch pinning through the reference pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04f; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
for m in tiny base; do
  F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_$m.npy $m > $O/bw_prev_$m.log 2>&1 || exit 1
  timeout -k 10 300 python tools/diag_lib_bitwise.py $O/new_$m.npy $m > $O/bw_new_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/prev_$m.npy'); b=np.load('$O/new_$m.npy'); print('$m bitwise equal:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c3_full_batch or tile_config" -q -rf --timeout 300 --timeout-method thread > $O/c3pin.log 2>&1
echo "c3 pin + tiles rc=$?"; tail -3 $O/c3pin.log
for i in 1 2; do
  for k in prev new; do
    if [ $k = prev ]; then export F5H_LIB=$LIB/libf5h_prev.so; else unset F5H_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vocos --probe none > $O/c2_${k}_$i.log 2>&1 || exit 1
    timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c4_${k}_$i.log 2>&1 || exit 1
  done
done
unset F5H_LIB
for f in $O/c2_*.log $O/c4_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; done
