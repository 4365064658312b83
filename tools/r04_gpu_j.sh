#!/bin/bash
# Round 4, box j: two-tile software-pipelined attention (attn16p_kernel, F5H_ATTN_PIPE=1) against the shipped
# kernel: attention tests, bit-for-bit library outputs, interleaved C2 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04j; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
F5H_ATTN_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1
echo "kp attention tests rc=$?"; tail -2 $O/attn_tests.log
for m in tiny base; do
  timeout -k 10 300 python tools/diag_lib_bitwise.py $O/ref_$m.npy $m > $O/bw_ref_$m.log 2>&1 || exit 1
  F5H_ATTN_PIPE=1 timeout -k 10 300 python tools/diag_lib_bitwise.py $O/kp_$m.npy $m > $O/bw_kp_$m.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('$O/ref_$m.npy'); b=np.load('$O/kp_$m.npy'); print('$m bitwise equal:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()))"
done
for i in 1 2; do
  for k in ref kp; do
    if [ $k = kp ]; then export F5H_ATTN_PIPE=1; else unset F5H_ATTN_PIPE; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-vocos > $O/c2_${k}_$i.log 2>&1 || exit 1
  done
done
unset F5H_ATTN_PIPE
for f in $O/c2_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel"], r["avg_launch_us"])')"; done
