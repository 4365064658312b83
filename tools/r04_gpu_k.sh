#!/bin/bash
# Round 4, box k: attention with scalar-addressed LDS-DMA (buffer_load ... lds: tile offset in soffset, LDS base in
# M0) and the tile loop unrolled by the ring depth (LDS read offsets as immediates) against the previous build
# (libf5h_prev.so): attention tests, bit-for-bit library outputs, interleaved C2 and C4 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${R04_OUT:-r04k}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1
echo "attention tests rc=$?"; tail -2 $O/attn_tests.log
for m in tiny base; do
  F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_$m.npy $m > $O/bw_prev_$m.log 2>&1 || exit 1
  timeout -k 10 300 python tools/diag_lib_bitwise.py $O/new_$m.npy $m > $O/bw_new_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/prev_$m.npy'); b=np.load('$O/new_$m.npy'); print('$m bitwise equal:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
for i in 1 2; do
  for k in prev new; do
    if [ $k = prev ]; then export F5H_LIB=$LIB/libf5h_prev.so; else unset F5H_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vocos > $O/c2_${k}_$i.log 2>&1 || exit 1
  done
done
for k in prev new; do
  if [ $k = prev ]; then export F5H_LIB=$LIB/libf5h_prev.so; else unset F5H_LIB; fi
  timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/c4_${k}.log 2>&1 || exit 1
done
unset F5H_LIB
for f in $O/c2_*.log $O/c4_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel"], r["avg_launch_us"])')"; done
