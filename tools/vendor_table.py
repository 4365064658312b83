"""Markdown table of this build's per-class kernel-trace averages against the vendor libraries on the same box
(VERDICT r04 item 4): hipBLASLt GEMMs (torch.mm, no epilogue) and torch SDPA at the C2 and C4-per-rank shapes.

  python tools/vendor_table.py profiles/r05_vendor_c2_c4.json [profiles/r05_rocprof_classes_c2.json ...]
"""
import json
import sys

vj = json.load(open(sys.argv[1]))
vendor = vj["ops"]
ours = {cfg: o["classes"] for cfg, o in vj.get("ours", {}).items()}  # same box as the vendor run
for path in sys.argv[2:]:  # or per-class summaries given explicitly (these win)
    j = json.load(open(path))
    cfg = "c2" if j["shape"].get("S") == 2 else "c4"
    ours[cfg] = j["classes"]
print("| class | C2 ours µs | C2 vendor µs | C2 ours / vendor | C4 ours µs | C4 vendor µs | C4 ours / vendor |")
print("|---|---|---|---|---|---|---|")
for c in ("qkv", "out", "ffn1", "ffn2", "attention"):
    row = [c]
    for cfg in ("c2", "c4"):
        o = ours.get(cfg, {}).get(c, {}).get("avg_launch_us")
        v = vendor.get(f"{cfg}_{c}", {})
        vu = v.get("kernel_us", v.get("event_us"))
        tag = "" if "kernel_us" in v else " (event)"
        row += [f"{o:.1f}" if o else "—", f"{vu:.1f}{tag}" if vu else "—",
                f"{o / vu:.2f}" if o and vu else "—"]
    print("| " + " | ".join(row) + " |")
