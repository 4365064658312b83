#!/bin/bash
# Round 3 GPU pass W: AdaLN LayerNorm with the modulation rows staged once per workgroup in LDS (16 or 8
# rows per workgroup) against the previous build: bitwise comparison, interleaved C2 benches (norm class
# probed live), then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r03w; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/f5-tts_amd/f5_tts_amd/lib
F5H_LIB=$L/libf5h_base.so timeout -k 10 120 python tools/diag_lib_bitwise.py $O/bit_base.npy > $O/bit.log 2>&1 && timeout -k 10 120 python tools/diag_lib_bitwise.py $O/bit_new.npy >> $O/bit.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('$O/bit_base.npy'); b=np.load('$O/bit_new.npy'); print('bitwise identical to the previous build:', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()), 'max abs diff', float(np.abs(a-b).max()))" | tee $O/bitwise.txt
for i in 1 2; do
  for v in base r8 new; do
    lib=$L/libf5h.so; [ $v = base ] && lib=$L/libf5h_base.so; [ $v = r8 ] && lib=$L/libf5h_r8.so
    F5H_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vocos --probe norm > $O/${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/base_*.log $O/r8_*.log $O/new_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms/call; norm", r.get("avg_launch_us"), "us, frac", r.get("frac"))')"; done | tee $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/gputest.log | tail -8
