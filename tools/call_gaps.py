"""Per-call host-overhead view of a rocprofv3 kernel trace (rocpd database) of bench.py:
    rocprofv3 --kernel-trace -d gpurun_out/cg -o run -- python bench.py --probe none --no-vocos --no-cpu-baseline
    python tools/call_gaps.py gpurun_out/cg/run_results.db
A call ends at its final_where_out launch; its prologue is every launch before the first step_begin.
Prints, per call: device span, the prologue's launch count, span and busy time (their difference is
the launch gaps a prologue graph could remove), and the device idle time before the call starts.
"""
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "final_where" in r[0]]
    for ci, e in enumerate(ends):
        s = ends[ci - 1] + 1 if ci else 0
        seg = rows[s:e + 1]
        fb = next(i for i, r in enumerate(seg) if "step_begin" in r[0])
        busy = sum(r[2] - r[1] for r in seg[:fb])
        gap = (seg[0][1] - rows[s - 1][2]) if s else 0
        print(f"call {ci:2d}: span {(seg[-1][2] - seg[0][1]) / 1e6:8.3f} ms | prologue {fb:3d} launches, "
              f"span {(seg[fb][1] - seg[0][1]) / 1e6:6.3f} ms, busy {busy / 1e6:6.3f} ms | idle before call "
              f"{max(gap, 0) / 1e6:6.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
