#!/bin/bash
# SQ counters of the attention variants given as arguments (tools/attn_ab.py workload), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_LDS_DATA_FIFO_FULL"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_attn$i -o run -- python tools/attn_ab.py "$@" > gpurun_out/pmc_attn$i.log 2>&1 || exit 1
done
python - <<'PY'
import csv, statistics, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in (1, 2):
    for r in csv.DictReader(open(f"gpurun_out/pmc_attn{i}/run_counter_collection.csv")):
        if "attn16" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {statistics.median(v):16.0f}")
PY
