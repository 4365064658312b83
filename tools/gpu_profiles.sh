#!/bin/bash
# Per-class profile summaries for profiles/ (each stamped with F5H_HEAD and the engine source hash):
#   rocprof_classes_<c>.json  kernel-trace averages per class (graph mode, 1 warm + 2 marked calls)
#   pmc_mfma_<c>.json         SQ/GRBM counters per class (two passes within the gfx950 slot limits; eager, 1 call)
#   pmc_classes_<c>.json      HBM traffic per class (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_c2.sh)
# for each config in CONFIGS (default c2), with the phase chain off (F5H_CHAIN=0: every class its own launch, as the
# bench's per-class probes time them); at C2 also rocprof_chain_c2.json, the kernel trace with the chain on (its
# default). Output: gpurun_out/$OUT/<prefix>_*.json (PREFIX, default r05).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/${OUT:-profiles}; mkdir -p $O; export TMPDIR=/tmp
P=${PREFIX:-r05}
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
export F5H_CHAIN=0
for c in ${CONFIGS:-c2}; do
  F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2 timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- \
    python tools/trace_c2.py run $c > $O/tr_$c.log 2>&1 || { echo "trace $c failed"; exit 1; }
  (cd tools && python class_profile.py trace $O/tr_$c/run_kernel_trace.csv $c $O/${P}_rocprof_classes_$c.json > /dev/null) \
    && echo "trace $c ok" || exit 1
  if [ "${SQ:-1}" = 1 ]; then
    i=0
    for PP in "$P1" "$P2"; do
      i=$((i+1))
      # C2 in the shipped graph mode (1 warm + 2 marked calls, within the profiler's dispatch limit); the batch
      # configs eager, one call (their graph-mode counter passes never finish under this profiler)
      if [ $c = c2 ]; then EV="F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2"; else EV="F5H_GRAPH=0 F5H_TRACE_WARM=0 F5H_TRACE_CALLS=1"; fi
      env $EV timeout -s KILL 300 rocprofv3 --pmc $PP --kernel-trace --output-format csv -d $O/sq_${c}_$i -o run -- \
        python tools/trace_c2.py run $c > $O/sq_${c}_$i.log 2>&1 || { echo "sq $c pass $i failed"; exit 1; }
    done
    (cd tools && python class_profile.py pmc $c $O/${P}_pmc_mfma_$c.json $O/sq_${c}_1/run_counter_collection.csv \
      $O/sq_${c}_2/run_counter_collection.csv > /dev/null) && echo "sq $c ok" || exit 1
  fi
  if [ "${TRAFFIC:-1}" = 1 ]; then
    timeout -k 10 900 ./tools/pmc_c2.sh $O/${P}_pmc_classes_$c.json $c > $O/pmc_$c.log 2>&1 && echo "traffic $c ok" || exit 1
  fi
done
if [ "${CHAIN_TRACE:-1}" = 1 ] && echo " ${CONFIGS:-c2} " | grep -q " c2 "; then
  F5H_CHAIN=1 F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2 timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr_chain -o run -- \
    python tools/trace_c2.py run c2 > $O/tr_chain.log 2>&1 || { echo "chain trace failed"; exit 1; }
  (cd tools && python class_profile.py trace $O/tr_chain/run_kernel_trace.csv c2 $O/${P}_rocprof_chain_c2.json > /dev/null) \
    && echo "chain trace ok" || exit 1
fi
# keep the summaries (and the rocprof stats); the per-dispatch CSVs would exceed what a call may bring back
find $O -name "*_kernel_trace.csv" -delete -o -name "*_counter_collection.csv" -delete
du -sh $PWD/gpurun_out
