#!/bin/bash
# Round 4, box b: engine-drop diagnostic, pad-row-skip bitwise tests, interleaved C3 A/B (pad skip off/on),
# then the SQ/GRBM counter passes at C4 per rank (a heartbeat file keeps the long silent passes alive).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04b; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 python tools/diag_drop.py > $O/diag_drop.log 2>&1; echo "diag rc=$?"; tail -2 $O/diag_drop.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "pad_row_skip" -q -rf --timeout 300 --timeout-method thread > $O/padskip.log 2>&1
echo "padskip rc=$?"; tail -3 $O/padskip.log
for i in 1 2; do
  F5H_NO_PAD_SKIP=1 timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c3_off_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-vocos --probe none > $O/c3_on_$i.log 2>&1 || exit 1
done
for f in $O/c3_*.log; do echo "$(basename $f) $(tail -1 $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 500 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmc_c4_$i -o run -- \
    python tools/trace_c2.py run c4 > $O/pmc_c4_$i.log 2>&1 || { echo "pmc c4 pass $i failed"; exit 1; }
  echo "pmc c4 pass $i ok"
done
(cd tools && python class_profile.py pmc c4 $O/r04_pmc_mfma_c4.json $O/pmc_c4_1/run_counter_collection.csv \
  $O/pmc_c4_2/run_counter_collection.csv > /dev/null) && echo "pmc c4 ok"
