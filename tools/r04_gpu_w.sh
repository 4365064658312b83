#!/bin/bash
# Round 4, box w: gemm_kernel tiles ordered by column group (an XCD's run is a rows x half-the-columns rectangle when
# there are >= 16 column tiles): bitwise check, GEMM tile-config tests, per-class HBM traffic, interleaved C2 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04w; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tile_config or pad_row or linear" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"; tail -2 $O/tests.log
for m in tiny base; do
  F5H_LIB=$LIB/libf5h_prev.so timeout -k 10 300 python tools/diag_lib_bitwise.py $O/prev_$m.npy $m > $O/bw_prev_$m.log 2>&1 || exit 1
  timeout -k 10 300 python tools/diag_lib_bitwise.py $O/new_$m.npy $m > $O/bw_new_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/prev_$m.npy'); b=np.load('$O/new_$m.npy'); print('$m bitwise equal:', bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
timeout -k 10 600 ./tools/pmc_c2.sh $O/r04_pmc_classes_xcdrect.json > $O/pmc.log 2>&1; echo "pmc rc=$?"
python -c "
import json; d=json.load(open('$O/r04_pmc_classes_xcdrect.json'))
for k,v in d['classes'].items(): print(k, v['hbm_over_algorithmic'], round(v['hbm_bytes']/1e6,1))"
for i in 1 2; do
  for k in prev new; do
    if [ $k = new ]; then unset F5H_LIB; else export F5H_LIB=$LIB/libf5h_prev.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vocos > $O/c2_${k}_$i.log 2>&1 || exit 1
  done
done
unset F5H_LIB
for f in $O/c2_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["roofline_classes"]; print(d["ms_per_step"], {k: v["avg_launch_us"] for k, v in c.items()})')"; done
