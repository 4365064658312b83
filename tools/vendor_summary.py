"""Summarise a tools/gpu_vendor.sh run into profiles/<name>.json: per op the hipBLASLt / SDPA kernel-trace average
(timed launches only: the first 3 of each op's dispatch run are its warm-up) and the HIP-event average,
plus this build's per-class kernel-trace averages from the same box ("ours", when the run traced them).

  python tools/vendor_summary.py gpurun_out/<dir> profiles/r05_vendor_c2_c4.json
"""
import csv
import json
import os
import sys

d, out = sys.argv[1], sys.argv[2]
rows = sorted(csv.DictReader(open(os.path.join(d, "vendor", "run_kernel_trace.csv"))),
              key=lambda r: int(r["Start_Timestamp"]))
ev = json.load(open(os.path.join(d, "vendor_ops.json")))
order = [k for k in ev["ops"] if not k.endswith("attention")]
runs = []  # consecutive dispatches of one GEMM kernel at one grid = one op's launches
for r in rows:
    n = r["Kernel_Name"]
    if "Cijk" not in n:
        continue
    key = (n, r["Grid_Size_X"])
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if runs and runs[-1][0] == key:
        runs[-1][1].append(dur)
    else:
        runs.append([key, [dur]])
res = {"source": f"tools/gpu_vendor.sh ({d}): tools/vendor_ref.py under rocprofv3 --kernel-trace on one MI355X; "
                 "kernel_us = kernel-trace average of the timed launches (each op's first 3 launches are warm-up), "
                 "event_us = HIP-event average of the same back-to-back launches (launch gaps included). hipBLASLt "
                 "GEMMs carry no epilogue (ours fuse bias, RoPE + q/k/v scatter, GELU or the gated residual); SDPA is "
                 "torch's attention (bf16, D = 64, non-causal).",
       "torch": ev.get("torch"), "ops": {}}
for name, (key, durs) in zip(order, runs):
    o = {k: v for k, v in ev["ops"][name].items() if k not in ("us", "frac", "tflops")}
    o["kernel"] = key[0].split("_UserArgs_")[-1][:40] if "_UserArgs_" in key[0] else key[0][:60]
    t = durs[3:] or durs
    o["kernel_us"] = round(sum(t) / len(t), 2)
    o["event_us"] = round(ev["ops"][name]["us"], 2)
    res["ops"][name] = o
for k in ("c2_attention", "c4_attention"):
    if k in ev["ops"]:
        o = {kk: v for kk, v in ev["ops"][k].items() if kk not in ("us", "frac", "tflops")}
        o["event_us"] = round(ev["ops"][k]["us"], 2)
        res["ops"][k] = o
# this build's per-class kernel-trace averages from the same box (gpu_vendor.sh traces them after the vendor run)
for cfg in ("c2", "c4"):
    f = os.path.join(d, f"classes_{cfg}.json")
    if os.path.exists(f):
        j = json.load(open(f))
        res.setdefault("ours", {})[cfg] = {"head": j.get("head"), "src_hash": j.get("src_hash"),
                                           "classes": {c: {"avg_launch_us": v["avg_launch_us"]}
                                                       for c, v in j["classes"].items()}}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["ops"], indent=1))
