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
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x kernel-trace duration): the fraction
                   of the launch's cycles the matrix pipes were busy (MFMA_BUSY sums per-SIMD busy cycles:
                   32 per 32x32x16, 16 per 16x16x32 bf16 MFMA). clock: the slope of GRBM_GUI_ACTIVE against
                   the duration over the classes / 8 XCDs (GRBM_GUI_ACTIVE carries a fixed per-dispatch part
                   under the profiler, so GRBM / 8 / duration "reads high on short dispatches",
                   MI355X_MICROARCH.md 'DVFS give-back'); mfma_busy_grbm = the raw MFMA_BUSY / (1024 x
                   GRBM / 8), a lower bound
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked at s_waitcnt / barrier)
  issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: MFMA dependency / pipe busy)
  active_frac    = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  coexec_over_mfma = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (vector work under the MFMAs)
  valu_per_mfma  = SQ_INSTS_VALU / SQ_INSTS_MFMA
  clock_ghz      = the fitted clock (above), one value for the run
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

from pmc_classes import SHAPES as _SHAPES, classify

SHAPES = {c: {k: s[k] for k in ("config", "S", "L", "dim", "depth")} for c, s in _SHAPES.items()}
NSIMD = 1024  # 256 CUs x 4 SIMDs



def _stamp():
    """Provenance of a summary (bench.summary_stamp): the git head (F5H_HEAD) and the engine source hash."""
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    import bench
    return bench.summary_stamp()

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
         "source": path, "shape": SHAPES[config], "classes": res, **_stamp()}
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
    med = {c: {k: statistics.median(v) for k, v in d.items() if v} for c, d in acc.items()}
    # GRBM_GUI_ACTIVE per dispatch = fixed profiler part + 8 XCDs x clock x duration (it "reads high on
    # short dispatches", MI355X_MICROARCH.md DVFS give-back): a least-squares line over the classes gives
    # the clock the chip held under this load and the fixed part
    pts = [(m["_duration_us"], m["GRBM_GUI_ACTIVE"]) for m in med.values()
           if m.get("_duration_us") and m.get("GRBM_GUI_ACTIVE")]
    fit = None
    if len(pts) >= 3:
        n = len(pts)
        mx, my = sum(p[0] for p in pts) / n, sum(p[1] for p in pts) / n
        sxx = sum((p[0] - mx) ** 2 for p in pts)
        if sxx > 0:
            slope = sum((p[0] - mx) * (p[1] - my) for p in pts) / sxx
            fit = {"clock_ghz": round(slope / 8.0 / 1e3, 4), "grbm_fixed": round(my - slope * mx, 1)}
    res = {}
    for c, m in med.items():
        e = {k: m[k] for k in sorted(m)}
        grbm = m.get("GRBM_GUI_ACTIVE")
        if fit and m.get("_duration_us") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            cyc = fit["clock_ghz"] * 1e3 * m["_duration_us"]  # kernel cycles at the fitted clock
            e["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * cyc), 4)
        if grbm and "SQ_VALU_MFMA_BUSY_CYCLES" in m:  # the raw form, low on short dispatches
            e["mfma_busy_grbm"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * grbm / 8.0), 4)
        if m.get("SQ_INSTS_MFMA"):
            e["mfma_cycles_per_inst"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / m["SQ_INSTS_MFMA"], 2)
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
        if fit:
            e["clock_ghz"] = fit["clock_ghz"]
        res[c] = e
    j = {"note": f"rocprofv3 --pmc passes (each within the gfx950 per-pass slots, --kernel-trace beside) over "
                 f"tools/trace_c2.py run {config} in the shipped graph mode; median per dispatch of each class; "
                 f"SQ_WAVE_CYCLES/WAIT_*/ACTIVE_* in quad-cycles, MFMA_BUSY in cycles; derived metrics in "
                 f"tools/class_profile.py",
         "sources": list(paths), "shape": SHAPES[config], "grbm_fit": fit, "classes": res, **_stamp()}
    json.dump(j, open(out, "w"), indent=1)
    print(json.dumps(j, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(*sys.argv[2:5])
    else:
        pmc(sys.argv[2], sys.argv[3], *sys.argv[4:])
