#!/bin/bash
# Round 4, box r: 16-byte-vector RMSNorm (UNetT, 16-bit residual, d = 1024): full GPU suite, interleaved C5 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04r; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
LIB=$PWD/f5-tts_amd/f5_tts_amd/lib
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests rc=$?"; tail -2 $O/gputest.log
for i in 1 2; do
  for k in prev new; do
    if [ $k = new ]; then unset F5H_LIB; else export F5H_LIB=$LIB/libf5h_prev.so; fi
    timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --no-vocos > $O/c5_${k}_$i.log 2>&1 || exit 1
  done
done
unset F5H_LIB
for f in $O/c5_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d["roofline_classes"]; print(d["ms_per_step"], {k: v["avg_launch_us"] for k, v in c.items()})')"; done
