#!/bin/bash
# Round 4, first box: GPU suite (+ reduced-precision envelopes logged), smoke, default bench line, then
# the per-class rocprofv3 summaries bench.py attaches: kernel-trace averages and SQ/GRBM counter passes
# (MFMA busy, wait / issue-stall split) at C2 and at C4 per rank, in the shipped graph mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
export F5H_ENVELOPE_LOG=$O/envelopes.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" $O/gputest.log | tail -3
unset F5H_ENVELOPE_LOG
timeout -k 10 240 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 && echo "c2 ok" || exit 1
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for cfg in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$cfg -o run -- \
    python tools/trace_c2.py run $cfg > $O/trace_$cfg.log 2>&1 || { echo "trace $cfg failed"; exit 1; }
  python tools/class_profile.py trace $O/trace_$cfg/run_kernel_trace.csv $cfg $O/r04_rocprof_classes_$cfg.json > /dev/null \
    && echo "trace $cfg ok"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmc_${cfg}_$i -o run -- \
      python tools/trace_c2.py run $cfg > $O/pmc_${cfg}_$i.log 2>&1 || { echo "pmc $cfg pass $i failed"; exit 1; }
  done
  python tools/class_profile.py pmc $cfg $O/r04_pmc_mfma_$cfg.json $O/pmc_${cfg}_1/run_counter_collection.csv \
    $O/pmc_${cfg}_2/run_counter_collection.csv > /dev/null && echo "pmc $cfg ok"
done
python - <<'PY'
import json
for c in ("c2", "c4"):
    d = json.load(open(f"gpurun_out/r04a/r04_pmc_mfma_{c}.json"))
    for k, v in d["classes"].items():
        print(c, k, {x: v.get(x) for x in ("mfma_busy", "wait_frac", "issue_stall_frac", "coexec_over_mfma", "clock_ghz")})
PY
tail -1 $O/bench_c2.log | cut -c1-400
