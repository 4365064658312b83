#!/bin/bash
# PMC evidence for the C2 GEMMs (tools/gemm_tune.py workload, the configurations pick_cfg uses at
# C2: QKV cfg5 192x128, FFN1 cfg1 128x128, out/FFN2 cfg0 64x128): one SQ pass and one pass per HBM
# counter (MI355X_MICROARCH.md: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2 -> separate passes).
#   bash tools/pmc_gemm.sh   (on the GPU box) -> gpurun_out/pmc_gemm/r01_pmc_gemm.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GT_SHAPES=c2_qkv,c2_ffn1,c2_out,c2_ffn2 GT_CFGS=0,1,5
O=gpurun_out/pmc_gemm
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
i=0
for P in "$P1" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python tools/gemm_tune.py > $O/p$i.log 2>&1 || exit 1
done
python - "$O" <<'PY'
import csv, json, statistics, collections, sys
O = sys.argv[1]
# (shape, cfg) -> kernel grid, as tools/gemm_tune.py keys its dispatches
sys.path.insert(0, "tools")
import gemm_tune as gt
want = {("c2_qkv", 5), ("c2_ffn1", 1), ("c2_out", 0), ("c2_ffn2", 0)}
# gemm dispatches in issue order are SHAPES x CFGS x REPS (tools/gemm_tune.py run() order)
shapes, cfgs = list(gt.SHAPES), list(gt.CFGS)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in (1, 2, 3):
    per = collections.OrderedDict()
    rows = [r for r in csv.DictReader(open(f"{O}/p{i}/run_counter_collection.csv")) if "gemm" in r["Kernel_Name"]]
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        per.setdefault(int(r["Dispatch_Id"]), []).append(r)
    assert len(per) == len(shapes) * len(cfgs) * gt.REPS, len(per)
    for idx, rs in enumerate(per.values()):
        si, ci = divmod(idx // gt.REPS, len(cfgs))
        for r in rs:
            agg[(shapes[si], cfgs[ci])][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for name, cfg in sorted(want):
    M, N, K = gt.SHAPES[name]
    grid = gt.grid_threads(M, N, cfg)
    d = {c: statistics.median(v) for c, v in agg.get((name, cfg), {}).items()}
    if not d:
        continue
    hbm = 2.0 * d.get("FETCH_SIZE", 0) * 1024 + d.get("WRITE_SIZE", 0) * 1024
    algo = 2.0 * (M * K + N * K) + 4.0 * M * N  # bf16 A and W read once, fp32 C written (op_linear)
    out[f"{name} cfg{cfg}"] = {"grid_threads": grid, "counters_median": d, "hbm_bytes": hbm,
                               "algorithmic_bytes": algo, "hbm_over_algorithmic": hbm / algo if algo else None}
out["note"] = ("median per dispatch over tools/gemm_tune.py's repetitions; bytes = 2*FETCH_SIZE*1024 + "
               "WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of wide streaming reads); op_linear "
               "epilogue (fp32 store), not the fused engine epilogues")
json.dump(out, open(f"{O}/r01_pmc_gemm.json", "w"), indent=1)
print(json.dumps({k: (v["hbm_over_algorithmic"] if isinstance(v, dict) else v) for k, v in out.items()}, indent=1))
PY
