#!/bin/bash
# Round 4, box u: attention with the younger half of each workgroup at s_setprio 1 (static form).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${R04_OUT:-r04u}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k attention -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
echo "parity tests rc=$?"; tail -2 $O/parity.log
for m in tiny base; do
  F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_$m.npy $m > $O/bw_prev_$m.log 2>&1 || exit 1
  timeout -k 10 300 python tools/diag_lib_bitwise.py $O/new_$m.npy $m > $O/bw_new_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/prev_$m.npy'); b=np.load('$O/new_$m.npy'); print('$m bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
for i in 1 2; do
  for k in prev new; do
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
