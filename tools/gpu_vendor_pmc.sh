#!/bin/bash
# Counter-level side-by-side of hipBLASLt and this build's GEMM classes at C2 and C4: the same
# four rocprofv3 --pmc passes (each within the gfx950 per-pass slots, --kernel-trace beside) over
# tools/vendor_ref.py (GEMMs only) and tools/trace_c2.py run c2 / c4, summarised by tools/vendor_pmc.py into
# $O/vendor_pmc_c2_c4.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-vpmc}; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT_sum"
P4="WRITE_SIZE TCC_MISS_sum"
REPS=5
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  VENDOR_GEMM_ONLY=1 VENDOR_REPS=$REPS timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv \
    -d $O/v$i -o run -- python tools/vendor_ref.py > $O/v$i.log 2>&1 || { echo "vendor pass $i failed"; tail -5 $O/v$i.log; exit 1; }
  F5H_CHAIN=0 F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2 timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv \
    -d $O/c2_$i -o run -- python tools/trace_c2.py run c2 > $O/c2_$i.log 2>&1 || { echo "c2 pass $i failed"; tail -5 $O/c2_$i.log; exit 1; }
  F5H_GRAPH=0 F5H_TRACE_WARM=0 F5H_TRACE_CALLS=1 timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv \
    -d $O/c4_$i -o run -- python tools/trace_c2.py run c4 > $O/c4_$i.log 2>&1 || { echo "c4 pass $i failed"; tail -5 $O/c4_$i.log; exit 1; }
  echo "pass $i ok"
done
python tools/vendor_pmc.py $O/vendor_pmc_c2_c4.json $REPS $O/v1 $O/v2 $O/v3 $O/v4 -- c2 $O/c2_1 $O/c2_2 $O/c2_3 $O/c2_4 \
  -- c4 $O/c4_1 $O/c4_2 $O/c4_3 $O/c4_4 > $O/summary.txt 2>&1; rc=$?
cat $O/summary.txt
find $O -name "*.csv" -size +2M -delete
exit $rc
