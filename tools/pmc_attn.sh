#!/bin/bash
# SQ counters of the bf16 attention kernel at the C2 shape (tools/attn_time.py workload), two
# passes per variant; variants = values of F5H_ATTN given as arguments (default: 0 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ATTN_REPS=20
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
for v in ${@:-0 1}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    F5H_ATTN=$v timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_attn_v${v}_$i -o run -- python tools/attn_time.py > gpurun_out/pmc_attn_v${v}_$i.log 2>&1 || exit 1
  done
done
python - "${@:-0 1}" <<'PY'
import csv, statistics, collections, sys, glob
for v in sys.argv[1:]:
    for vv in v.split():
        d = collections.defaultdict(list)
        for i in (1, 2):
            for r in csv.DictReader(open(glob.glob(f"gpurun_out/pmc_attn_v{vv}_{i}/run_counter_collection.csv")[0])):
                if "attn" not in r["Kernel_Name"]:
                    continue
                d[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"F5H_ATTN={vv}")
        for c, x in sorted(d.items()):
            print(f"   {c:28s} {statistics.median(x):16.0f}")
PY
