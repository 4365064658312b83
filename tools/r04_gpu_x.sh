#!/bin/bash
# Round 4, box x: per-class HBM traffic (FETCH_SIZE / WRITE_SIZE passes) at C3, C4 and C5, and the C5 kernel trace
# + SQ/GRBM counter passes (C5 had no class summaries; part 2), so the large-config bench lines carry traffic and counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04x; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
PART=${1:-1}
if [ $PART = 1 ]; then
for c in c4 c5; do
  timeout -k 10 900 ./tools/pmc_c2.sh $O/r04_pmc_classes_$c.json $c > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  echo "pmc $c ok"
done
exit 0
fi
timeout -k 10 900 ./tools/pmc_c2.sh $O/r04_pmc_classes_c3.json c3 > $O/pmc_c3.log 2>&1 || { echo "pmc c3 failed"; exit 1; }
echo "pmc c3 ok"
# kernel trace in the shipped graph mode (1 warm + 2 marked calls, as at C4: tools/r04_gpu_o.sh)
F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2 timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c5 -o run -- \
  python tools/trace_c2.py run c5 > $O/tr_c5.log 2>&1 || { echo "trace c5 failed"; exit 1; }
(cd tools && python class_profile.py trace $O/tr_c5/run_kernel_trace.csv c5 $O/r04_rocprof_classes_c5.json > /dev/null) \
  && echo "trace c5 ok"
# counter passes eager (F5H_GRAPH=0), one call: graph-mode PMC passes at the batch shapes never finish
export F5H_GRAPH=0 F5H_TRACE_WARM=0 F5H_TRACE_CALLS=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmc_c5_$i -o run -- \
    python tools/trace_c2.py run c5 > $O/pmc_c5_$i.log 2>&1 || { echo "pmc c5 pass $i failed"; exit 1; }
  echo "pmc c5 pass $i ok"
done
(cd tools && python class_profile.py pmc c5 $O/r04_pmc_mfma_c5.json $O/pmc_c5_1/run_counter_collection.csv \
  $O/pmc_c5_2/run_counter_collection.csv > /dev/null) && echo "pmc c5 ok"
python - <<EOF
import json
for c in ("c3", "c4", "c5"):
    d = json.load(open("$O/r04_pmc_classes_%s.json" % c))
    print(c, {k: (v["hbm_over_algorithmic"], v["dispatches"]) for k, v in d["classes"].items()})
d = json.load(open("$O/r04_pmc_mfma_c5.json"))
print("c5", {k: (v.get("mfma_busy"), v.get("valu_per_mfma")) for k, v in d["classes"].items()})
EOF
