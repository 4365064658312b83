"""Counter-level side-by-side of this build's GEMM classes and hipBLASLt at the same shapes.

Inputs: the same rocprofv3 --pmc passes (each with --kernel-trace beside) over
  * tools/vendor_ref.py with VENDOR_GEMM_ONLY=1 VENDOR_REPS=R (hipBLASLt through torch.mm, bf16, C = A.W^T),
  * tools/trace_c2.py run c2 (graph mode, phase chain off: every class its own launch) and run c4 (one eager call).

    python tools/vendor_pmc.py OUT.json R VENDOR_DIR1 [VENDOR_DIR2 ...] -- c2 OURS_C2_DIR1 ... -- c4 OURS_C4_DIR1 ...

Each DIR holds run_counter_collection.csv and run_kernel_trace.csv of one pass. Per class and side (median per
dispatch): duration, kernel name and VGPR/AGPR counts, MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the
dispatch's own GRBM clock estimate GRBM_GUI_ACTIVE / 8 / duration: the same formula on both sides, reads low on
short dispatches), MFMA cycles per instruction (16: 16x16x32, 32: 32x32x16), VALU / LDS instructions per MFMA, LDS
bank-conflict cycles over LDS-array cycles, wave-cycle split (wait / issue-stall / active), HBM bytes (2 x
FETCH_SIZE per the gfx950 note + WRITE_SIZE) over the algorithmic bytes, L2 hit rate.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_classes import classify  # noqa: E402

N_FR, D, F_DIM = 1876, 1024, 2048
OPS = []
for cfg, S in (("c2", 2), ("c4", 64)):
    M = S * N_FR
    OPS += [(f"{cfg}_qkv", M, 3 * D, D), (f"{cfg}_out", M, D, D), (f"{cfg}_ffn1", M, F_DIM, D),
            (f"{cfg}_ffn2", M, D, F_DIM)]


def read_pass(d):
    per = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], int(r.get("VGPR_Count", 0) or 0), int(r.get("Accum_VGPR_Count", 0) or 0),
                     int(r.get("Grid_Size", 0) or 0))
    dur = {}
    kt = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(kt):
        for r in csv.DictReader(open(kt)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return [(did, meta[did], per[did], dur.get(did)) for did in sorted(per)]


def vendor_groups(dirs, reps):
    """op name -> list of per-dispatch counter dicts (the timed launches: 3 warm + reps per op, SH order)."""
    acc = defaultdict(list)
    for d in dirs:
        disp = [x for x in read_pass(d) if "Cijk" in x[1][0] or "gemm" in x[1][0].lower()]
        per_op = 3 + reps
        if len(disp) != per_op * len(OPS):
            print(f"warning: {d}: {len(disp)} GEMM dispatches, expected {per_op * len(OPS)}", file=sys.stderr)
        for i, (_, meta, cnt, us) in enumerate(disp[: per_op * len(OPS)]):
            op = OPS[i // per_op][0]
            if i % per_op >= 3:  # skip the warm launches
                acc[op].append((meta, cnt, us))
    return acc


def ours_groups(config, dirs):
    acc = defaultdict(list)
    for d in dirs:
        disp = read_pass(d)
        cls = classify([(did, meta[0], 0.0) for did, meta, _, _ in disp])
        for i, (_, meta, cnt, us) in enumerate(disp):
            c = cls.get(i)
            if c in ("qkv", "out", "ffn1", "ffn2"):
                acc[f"{config}_{c}"].append((meta, cnt, us))
    return acc


def summarise(rows, alg_bytes):
    if not rows:
        return None
    keys = set()
    for _, cnt, _ in rows:
        keys |= set(cnt)
    med = {k: statistics.median([cnt[k] for _, cnt, _ in rows if k in cnt]) for k in sorted(keys)}
    durs = [us for _, _, us in rows if us]
    meta = rows[0][0]
    e = {"kernel": meta[0][:160], "vgpr": meta[1], "agpr": meta[2], "grid": meta[3], "dispatches": len(rows)}
    if durs:
        e["duration_us"] = round(statistics.median(durs), 2)
    m = med
    if m.get("GRBM_GUI_ACTIVE") and durs:
        e["clock_est_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / (statistics.median(durs) * 1e3), 3)
    if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
        e["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 4)
    if m.get("SQ_INSTS_MFMA"):
        mf = m["SQ_INSTS_MFMA"]
        e["mfma_cycles_per_inst"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / mf, 2)
        for k, name in (("SQ_INSTS_VALU", "valu_per_mfma"), ("SQ_INSTS_LDS", "lds_per_mfma")):
            if k in m:
                e[name] = round(m[k] / mf, 3)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_conflict_over_active"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_WAIT_INST_LDS", "lds_issue_stall_frac"),
                        ("SQ_ACTIVE_INST_LDS", "lds_active_frac"), ("SQ_ACTIVE_INST_VALU", "valu_active_frac")):
            if k in m:
                e[name] = round(m[k] / wc, 4)
        e["wave_cycles"] = wc
    if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and "SQ_VALU_MFMA_COEXEC_CYCLES" in m:
        e["coexec_over_mfma"] = round(m["SQ_VALU_MFMA_COEXEC_CYCLES"] / m["SQ_VALU_MFMA_BUSY_CYCLES"], 4)
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        hbm = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024  # KB -> B; FETCH doubled (gfx950)
        e["hbm_bytes"] = hbm
        e["traffic_over_algorithmic"] = round(hbm / alg_bytes, 3)
    if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
        t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
        if t:
            e["l2_hit_rate"] = round(m["TCC_HIT_sum"] / t, 4)
    return e


def main():
    out, reps = sys.argv[1], int(sys.argv[2])
    groups, cur = [], []
    for a in sys.argv[3:]:
        if a == "--":
            groups.append(cur)
            cur = []
        else:
            cur.append(a)
    groups.append(cur)
    vend = vendor_groups(groups[0], reps)
    ours = {}
    for g in groups[1:]:
        ours.update(ours_groups(g[0], g[1:]))
    res = {}
    for op, M, N, K in OPS:
        alg = 2 * (M * K + N * K + M * N)  # bf16 A, W, C (the library writes C only)
        v = summarise(vend.get(op, []), alg)
        o = summarise(ours.get(op, []), alg)
        ent = {"M": M, "N": N, "K": K, "flops": 2.0 * M * N * K, "algorithmic_bytes_plain": alg, "vendor": v,
               "ours": o}
        if v and o and v.get("duration_us") and o.get("duration_us"):
            ent["ours_over_vendor_time"] = round(o["duration_us"] / v["duration_us"], 3)
            for side in (v, o):
                side["frac_of_2p5pf"] = round(ent["flops"] / (side["duration_us"] * 1e-6) / 2.5e15, 4)
        res[op] = ent
    j = {"note": "rocprofv3 --pmc passes (SQ / LDS / FETCH_SIZE+TCC_HIT / WRITE_SIZE+TCC_MISS, --kernel-trace beside) "
                 "over hipBLASLt (tools/vendor_ref.py, torch.mm bf16, plain C = A.W^T) and this build's GEMM classes "
                 "(tools/trace_c2.py: c2 graph mode with the phase chain off, c4 one eager call) on one box; medians "
                 "per dispatch; ours carry their fused epilogues (QKV RoPE + q/k/v scatter, out/FFN2 gate + residual "
                 "read/write, FFN1 GELU-tanh), traffic_over_algorithmic is against the plain A + W + C bytes on "
                 "both sides",
         "ops": res}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    j.update(bench.summary_stamp())
    json.dump(j, open(out, "w"), indent=1)
    for op, e in res.items():
        v, o = e["vendor"] or {}, e["ours"] or {}
        print(f"{op:9s} time {o.get('duration_us')} / {v.get('duration_us')} us  busy {o.get('mfma_busy')} / "
              f"{v.get('mfma_busy')}  cyc/mfma {o.get('mfma_cycles_per_inst')} / {v.get('mfma_cycles_per_inst')}  "
              f"lds/mfma {o.get('lds_per_mfma')} / {v.get('lds_per_mfma')}  valu/mfma {o.get('valu_per_mfma')} / "
              f"{v.get('valu_per_mfma')}  wait {o.get('wait_frac')} / {v.get('wait_frac')}  stall "
              f"{o.get('issue_stall_frac')} / {v.get('issue_stall_frac')}  traffic {o.get('traffic_over_algorithmic')}"
              f" / {v.get('traffic_over_algorithmic')}  vgpr {o.get('vgpr')}+{o.get('agpr')} / {v.get('vgpr')}+"
              f"{v.get('agpr')}")
        print(f"          vendor kernel: {v.get('kernel')}")


if __name__ == "__main__":
    main()
