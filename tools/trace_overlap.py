"""Reconcile a rocprofv3 kernel trace of bench.py with the bench's own clock.

    python tools/trace_overlap.py RUN_kernel_trace.csv BENCH_LINE.json OUT.json

Per kernel class (chain, attention, conv, other): dispatches, mean duration (End - Start); over the timed calls'
window: the sum of all dispatch durations, the union of their [Start, End) intervals (device-busy time) and the
overlap between consecutive dispatches (a dispatch that starts before its predecessor ends: the profiler's
per-dispatch timestamps then count shared time twice). The bench line run under the profiler gives ms_per_step
(the profiled wall per call) for comparison with the per-call kernel sums.
"""
import csv
import json
import statistics
import sys


def klass(name):
    for k, pat in (("chain", "chain_kernel"), ("attention", "attn16"), ("conv", "conv16"), ("euler", "cfg_euler")):
        if pat in name:
            return k
    if "gemm" in name:
        return "gemm"
    return "other"


def main(trace, line_path, out):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    disp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    steps = line["steps"]
    # the timed calls are the last `steps` calls: each call has nfe x depth chain launches (C2: 16 x 22 = 352)
    # each call ends its NFE steps with one cfg_euler launch per step (C2: 16); the timed calls are the last `steps`
    # calls: the window starts right after the euler launch that ended the call before them
    eul = [i for i, d in enumerate(disp) if "cfg_euler" in d[2]]
    nfe = 16
    if len(eul) < (steps + 1) * nfe:
        raise SystemExit(f"{len(eul)} euler dispatches, fewer than {steps + 1} calls x {nfe}")
    j = eul[-steps * nfe - 1] + 1
    win = disp[j:]
    t0, t1 = win[0][0], max(e for _, e, _ in win)
    by = {}
    for s, e, n in win:
        by.setdefault(klass(n), []).append((e - s) / 1e3)
    busy, cur_s, cur_e = 0, None, None
    overlap, n_ov = 0, 0
    prev_e = None
    for s, e, _ in win:
        if prev_e is not None and s < prev_e:
            overlap += min(prev_e, e) - s
            n_ov += 1
        prev_e = e if prev_e is None else max(prev_e, e)
        if cur_s is None or s > cur_e:
            if cur_s is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ssum = sum(e - s for s, e, _ in win)
    res = {
        "note": "rocprofv3 --kernel-trace of bench.py (C2, --probe none) over the timed calls' window (from the end of the last untimed call's final Euler launch)",
        "calls": steps, "bench_ms_per_step_under_profiler": line["ms_per_step"],
        "window_ms_per_call": round((t1 - t0) / 1e6 / steps, 3),
        "sum_of_durations_ms_per_call": round(ssum / 1e6 / steps, 3),
        "union_busy_ms_per_call": round(busy / 1e6 / steps, 3),
        "overlapping_dispatches": n_ov, "overlap_ms_per_call": round(overlap / 1e6 / steps, 3),
        "classes": {k: {"dispatches": len(v), "mean_us": round(statistics.mean(v), 3),
                        "median_us": round(statistics.median(v), 3), "ms_per_call": round(sum(v) / 1e3 / steps, 3)}
                    for k, v in sorted(by.items())},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
