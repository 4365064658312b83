#!/bin/bash
# Round 4, box m: gemm_kernel K loop unrolled by the ring depth (fragment reads at immediate offsets: no vector
# instructions in the K loop) = libf5h_g.so; plus attention row sums as two independent packed chains = libf5h.so;
# against the previous build (libf5h_prev.so). Full GPU suite on the new build, bitwise check of the GEMM-only
# build, interleaved C2 (three builds) and C4 (prev/new) benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${R04_OUT:-r04m}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests rc=$?"; tail -2 $O/gputest.log
for m in tiny base; do
  F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_$m.npy $m > $O/bw_prev_$m.log 2>&1 || exit 1
  F5H_LIB=$LIB/libf5h_g.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/g_$m.npy $m > $O/bw_g_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/prev_$m.npy'); b=np.load('$O/g_$m.npy'); print('$m gemm-only bitwise equal:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
for i in 1 2; do
  for k in prev g new; do
    if [ $k = new ]; then unset F5H_LIB; else export F5H_LIB=$LIB/libf5h_$k.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vocos > $O/c2_${k}_$i.log 2>&1 || exit 1
  done
done
for k in prev new; do
  if [ $k = new ]; then unset F5H_LIB; else export F5H_LIB=$LIB/libf5h_$k.so; fi
  timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-vocos > $O/c4_${k}.log 2>&1 || exit 1
done
unset F5H_LIB
for f in $O/c2_*.log $O/c4_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; c=d["roofline_classes"]; print(d["ms_per_step"], r["kernel"], r["avg_launch_us"], {k: v["avg_launch_us"] for k, v in c.items()})')"; done
