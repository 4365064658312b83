#!/bin/bash
# Round artifacts for profiles/: kernel-trace stats of the C2 bench and the attention kernel's
# HBM traffic (two PMC passes: FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §rocprofv3 PMC slots).
#   ROUND=r01 bash tools/profile_round.sh      (on the GPU box; then copy gpurun_out/profiles_*)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out/prof_$R
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_trace.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit 1
done
python - "$O" "$R" <<'PY'
import csv, json, sys, statistics
O, R = sys.argv[1], sys.argv[2]
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{O}/{c}/run_counter_collection.csv"))
            if "attn_bf16" in r["Kernel_Name"] and r["Counter_Name"] == c]
    out[c] = (statistics.median(vals), len(vals))
j = {"kernel": "attention (attn_bf16_*)", "fetch_size_kb": out["FETCH_SIZE"][0], "write_size_kb": out["WRITE_SIZE"][0],
     "dispatches": out["FETCH_SIZE"][1], "note": "median per dispatch; rocprofv3 --pmc, one counter per pass; "
     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE reads half of wide streaming reads)"}
json.dump(j, open(f"{O}/{R}_pmc_attention.json", "w"), indent=1)
print(json.dumps(j))
PY
