"""Kernel-level anatomy of CFM.sample calls from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python tools/trace_c2.py run [--config c2]
    python tools/trace_c2.py report gpurun_out/tr/run_kernel_trace.csv

`run` does 3 warm calls and 3 marked calls (a torch.sort marker brackets them); `report` lists
per kernel name the dispatch count, mean duration and share of the marked window, and the GPU
idle time between consecutive kernels inside it (dispatch gaps).
"""
import csv
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd")]


def run(config="c2", calls=None):
    # F5H_TRACE_WARM / F5H_TRACE_CALLS (default 3 / 3): rocprofv3 of this ROCm build crashes after
    # ~12-16k graph-launched dispatches (tools/probes/launch_cost count), ~2.6k per C2 call, so a
    # graph-mode PMC pass uses 1 warm call + 2 marked calls
    warm = int(os.environ.get("F5H_TRACE_WARM", "3"))
    calls = int(os.environ.get("F5H_TRACE_CALLS", "3")) if calls is None else calls
    import torch

    import bench
    from f5_tts_amd import synthetic

    dev = torch.device("cuda", 0)
    case = {"c2": synthetic.c2_case, "c3": synthetic.c3_case, "c4": synthetic.c4_case, "c5": synthetic.c5_case}[config]()
    model, arch = bench.build_model(case["preset"], os.environ.get("COMPUTE", "bf16"), dev)
    B = case["B"]
    refs = case["ref"] if isinstance(case["ref"], list) else [case["ref"]] * B
    tots = case["total"] if isinstance(case["total"], list) else [case["total"]] * B
    inp = synthetic.make_case(B=B, ref_frames=refs, total_frames=tots, n_text=case["nt"])
    # lengths as host tensors (as the DP driver passes them): no device sync inside the calls
    kw = dict(cond=inp["cond"].to(dev), text=inp["text"].to(dev), duration=inp["duration"],
              lens=inp["lens"], steps=case["nfe"], cfg_strength=case["cfg"],
              sway_sampling_coef=case["sway"], seed=0, keep_trajectory=False)
    for _ in range(warm):
        model.sample(**kw)
    torch.cuda.synchronize()
    marker = torch.rand(64, device=dev)
    torch.sort(marker)  # start marker (a sort kernel: no sort runs inside CFM.sample)
    for _ in range(calls):
        model.sample(**kw)
    torch.sort(marker)  # end marker
    torch.cuda.synchronize()
    print("done", flush=True)


def report(path, calls=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "sort" in r["Kernel_Name"].lower()]
    i0, i1 = marks[0], marks[-1]  # the first and last sort kernels bracket the marked calls
    win = rows[i0 + 1:i1]
    t0 = int(win[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in win)
    span = (t1 - t0) / 1e3
    per = defaultdict(list)
    busy_end = t0
    idle = 0
    gaps = []
    prev = win[0]["Kernel_Name"]
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        per[r["Kernel_Name"].split("(")[0][:90]].append((e - s) / 1e3)
        if s > busy_end:
            idle += s - busy_end
            gaps.append(((s - busy_end) / 1e3, prev.split("(")[0][:50], r["Kernel_Name"].split("(")[0][:50]))
        busy_end = max(busy_end, e)
        prev = r["Kernel_Name"]
    print(f"window {span:.1f} us for {calls} calls = {span / calls:.1f} us/call; idle gaps {idle / 1e3:.1f} us "
          f"({idle / 1e3 / span * 100:.1f} %), {len(win)} dispatches")
    big = sorted(gaps, reverse=True)
    small = [g for g in gaps if g[0] < 5.0]
    print(f"gaps: {len(gaps)}; < 5 us: {len(small)} totalling {sum(g[0] for g in small):.1f} us; "
          f">= 5 us: {len(gaps) - len(small)} totalling {sum(g[0] for g in gaps) - sum(g[0] for g in small):.1f} us")
    for g in big[:12]:
        print(f"   gap {g[0]:8.1f} us  after {g[1]}  before {g[2]}")
    tot = sum(sum(v) for v in per.values())
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / tot * 100:5.1f}%  n={len(v) // calls:5d}/call  avg {sum(v) / len(v):8.2f} us  {name}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2] if len(sys.argv) > 2 else "c2")
    else:
        report(sys.argv[2])
