#!/bin/bash
# Round 4, box d: pad skip with the sequence-spreading XCD maps (bitwise tests, C3 interleaved A/B with the
# attention class probed live), fp16 vs bf16 SQ/GRBM pass at C2 (clock vs cycles), C4 counters in eager mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04d; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "pad_row_skip or permutation" -q -rf --timeout 300 --timeout-method thread > $O/padskip.log 2>&1
echo "padskip rc=$?"; tail -2 $O/padskip.log
for i in 1 2; do
  for k in off on; do
    if [ $k = off ]; then export F5H_NO_PAD_SKIP=1; else unset F5H_NO_PAD_SKIP; fi
    timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe attention > $O/c3_${k}_$i.log 2>&1 || exit 1
  done
done
unset F5H_NO_PAD_SKIP
for f in $O/c3_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_us"])')"; done
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for cm in bf16 fp16; do
  COMPUTE=$cm timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmc_c2_$cm -o run -- \
    python tools/trace_c2.py run c2 > $O/pmc_c2_$cm.log 2>&1 || { echo "pmc $cm failed"; exit 1; }
  (cd tools && python class_profile.py pmc c2 $O/pmc_c2_$cm.json $O/pmc_c2_$cm/run_counter_collection.csv > /dev/null) && echo "pmc $cm ok"
done
F5H_GRAPH=0 F5H_TRACE_WARM=0 F5H_TRACE_CALLS=1 timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmc_c4_1 -o run -- \
  python tools/trace_c2.py run c4 > $O/pmc_c4_1.log 2>&1 && echo "pmc c4 eager ok" || echo "pmc c4 eager failed"
