#!/bin/bash
# Round 4, box t: the SQ/GRBM counter passes of tools/r04_gpu_a.sh at C2 on the final HEAD (scalar-addressed DMA),
# graph mode, 1 warm + 2 marked calls per pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=$PWD/gpurun_out/r04t; mkdir -p $O; export TMPDIR=/tmp
( while true; do date +%s >> $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
export F5H_TRACE_WARM=1 F5H_TRACE_CALLS=2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmc_c2_$i -o run -- \
    python tools/trace_c2.py run c2 > $O/pmc_c2_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/class_profile.py pmc c2 $O/r04_pmc_mfma_c2_final.json $O/pmc_c2_1/run_counter_collection.csv \
  $O/pmc_c2_2/run_counter_collection.csv > /dev/null && echo "pmc ok"
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04t/r04_pmc_mfma_c2_final.json"))
for k, v in d["classes"].items():
    print(k, {x: v.get(x) for x in ("mfma_busy", "wait_frac", "issue_stall_frac", "active_frac", "valu_per_mfma", "clock_ghz", "_duration_us")})
a = d["classes"]["attention"]
waves = 2048; tiles = 30
print("attention per wave-tile cycles: wave", a["SQ_WAVE_CYCLES"] * 4 / waves / tiles, "active", a["SQ_ACTIVE_INST_ANY"] * 4 / waves / tiles,
      "valu", a["SQ_ACTIVE_INST_VALU"] * 4 / waves / tiles, "lds", a["SQ_ACTIVE_INST_LDS"] * 4 / waves / tiles,
      "valu insts", a["SQ_INSTS_VALU"] / waves / tiles)
PY
