"""Per-kernel-class summaries of a DiT CFM.sample run from rocprofv3 output, at one launch shape.

    # kernel trace (durations) of tools/trace_c2.py calls
    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python tools/trace_c2.py run c2
    python tools/class_profile.py trace D/run_kernel_trace.csv c2 OUT.json

    # SQ/GRBM counter passes (separate runs, each within the gfx950 slot limits) + the kernel trace of pass 1
    python tools/class_profile.py pmc c2 OUT.json D1/run_counter_collection.csv [D2/run_counter_collection.csv ...]

Dispatches are classified by position around each attention dispatch (a DiT block issues norm1, qkv,
attention, out, norm, ffn1, ffn2 in that order; conv by name), as tools/pmc_classes.py does. Output
files hold {"shape": {S, L, dim, depth}, "classes": {...}}; bench.py attaches a class's entry to its
line only at the shape it was measured on.

Derived per class (median per dispatch; chip totals):
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of the
                   launch's cycles the matrix pipes were busy (GRBM_GUI_ACTIVE sums the 8 XCDs' busy
                   cycles, MI355X_MICROARCH.md 'DVFS give-back'; MFMA_BUSY counts cycles per SIMD, 32 per
                   32x32x16 and 16 per 16x16x32 bf16 MFMA)
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked at s_waitcnt / barrier)
  issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: MFMA dependency / pipe busy)
  active_frac    = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  coexec_over_mfma = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (vector work under the MFMAs)
  valu_per_mfma  = SQ_INSTS_VALU / SQ_INSTS_MFMA
  clock_ghz      = GRBM_GUI_ACTIVE / 8 / kernel-trace duration (reads high under ~0.3 ms dispatches)
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

from pmc_classes import classify

SHAPES = {"c2": {"config": "c2", "S": 2, "L": 1876, "dim": 1024, "depth": 22},
          "c3": {"config": "c3", "S": 64, "L": 1876, "dim": 1024, "depth": 22},
          "c4": {"config": "c4", "S": 64, "L": 1876, "dim": 1024, "depth": 22}}
NSIMD = 1024  # 256 CUs x 4 SIMDs


def _trace_rows(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    return [(int(r["Dispatch_Id"]), r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            for r in rows]


def trace(path, config, out):
    disp = _trace_rows(path)
    cls = classify(disp)
    acc = defaultdict(list)
    for i, (_, _, us) in enumerate(disp):
        if i in cls:
            acc[cls[i]].append(us)
    res = {c: {"avg_launch_us": round(statistics.mean(v), 3), "median_launch_us": round(statistics.median(v), 3),
               "dispatches": len(v)} for c, v in acc.items()}
    j = {"note": f"rocprofv3 --kernel-trace of tools/trace_c2.py run {config} (warm + marked CFM.sample calls); "
                 f"per class mean/median dispatch duration (End - Start), classes by position around attention",
         "source": path, "shape": SHAPES[config], "classes": res}
    json.dump(j, open(out, "w"), indent=1)
    print(json.dumps(j, indent=1))


def _counters(path):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    return [(d, names[d], dict(per[d])) for d in sorted(per)]


def pmc(config, out, *paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        disp = _counters(p)
        cls = classify([(d, n, 0.0) for d, n, _ in disp])
        for i, (_, _, cnt) in enumerate(disp):
            if i in cls:
                for k, v in cnt.items():
                    acc[cls[i]][k].append(v)
        # durations from the kernel trace written beside the counters (--kernel-trace in the same pass)
        kt = p.replace("counter_collection", "kernel_trace")
        try:
            tr = _trace_rows(kt)
        except OSError:
            tr = []
        if tr:
            tcls = classify(tr)
            for i, (_, _, us) in enumerate(tr):
                if i in tcls:
                    acc[tcls[i]]["_duration_us"].append(us)
    res = {}
    for c, d in acc.items():
        m = {k: statistics.median(v) for k, v in d.items() if v}
        e = {k: m[k] for k in sorted(m)}
        grbm = m.get("GRBM_GUI_ACTIVE")
        if grbm and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            e["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * grbm / 8.0), 4)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for k, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                            ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if k in m:
                    e[name] = round(m[k] / wc, 4)
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and "SQ_VALU_MFMA_COEXEC_CYCLES" in m:
            e["coexec_over_mfma"] = round(m["SQ_VALU_MFMA_COEXEC_CYCLES"] / m["SQ_VALU_MFMA_BUSY_CYCLES"], 4)
        if m.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in m:
            e["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 3)
        if grbm and m.get("_duration_us"):
            e["clock_ghz"] = round(grbm / 8.0 / (m["_duration_us"] * 1e3), 3)
        res[c] = e
    j = {"note": f"rocprofv3 --pmc passes (each within the gfx950 per-pass slots, --kernel-trace beside) over "
                 f"tools/trace_c2.py run {config} in the shipped graph mode; median per dispatch of each class; "
                 f"SQ_WAVE_CYCLES/WAIT_*/ACTIVE_* in quad-cycles, MFMA_BUSY in cycles; derived metrics in "
                 f"tools/class_profile.py",
         "sources": list(paths), "shape": SHAPES[config], "classes": res}
    json.dump(j, open(out, "w"), indent=1)
    print(json.dumps(j, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(*sys.argv[2:5])
    else:
        pmc(sys.argv[2], sys.argv[3], *sys.argv[4:])
