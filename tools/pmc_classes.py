"""HBM traffic per launch of each kernel class of a CFM.sample call (C2 by default; C3/C4/C5 with the
trailing config argument and `trace_c2.py run --config cN`), from rocprofv3 PMC passes.

Per pass one counter (MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE uses 3 TCC slots,
WRITE_SIZE 2, so they cannot share a pass):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python tools/trace_c2.py run
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python tools/trace_c2.py run
    python tools/pmc_classes.py gpurun_out/pmc_f/run_counter_collection.csv \
        gpurun_out/pmc_w/run_counter_collection.csv profiles/r02_pmc_classes.json [c2|c3|c4|c5]

Dispatches are classified by their position around each attention dispatch (one DiT block issues
norm1, qkv, attention, out, norm, ffn1, ffn2 in that order; a UNetT block the same, after its skip
GEMM in the later half; a position whose kernel is not of the expected kind is dropped). hbm_bytes = 2 x FETCH_SIZE (gfx950
counts half of wide streaming reads) + WRITE_SIZE, in bytes (the counters report KB), median over
the dispatches of the class. algorithmic_bytes: operands + results at their widths, all S x L rows
(padded rows included: at C3 the batch is padded to the longest utterance).
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ORDER = {-2: "norm1", -1: "qkv", 1: "out", 2: "norm", 3: "ffn1", 4: "ffn2"}
# with the LayerNorm fold (round 6) the FFN-norm launch is gone and layers after the first have no
# attention-norm either: attention is followed by out, FFN1, FFN2 directly
ORDER_FOLD = {-2: "norm1", -1: "qkv", 1: "out", 2: "ffn1", 3: "ffn2"}
GEMMS = ("qkv", "out", "ffn1", "ffn2")
# launch shapes as bench.py names them (S = CFG-packed sequences, L = padded frames), FFN width
SHAPES = {"c2": dict(config="c2", S=2, L=1876, dim=1024, depth=22, ff=2048),
          "c3": dict(config="c3", S=64, L=1876, dim=1024, depth=22, ff=2048),
          "c4": dict(config="c4", S=64, L=1876, dim=1024, depth=22, ff=2048),
          "c5": dict(config="c5", S=16, L=1877, dim=1024, depth=24, ff=4096)}  # UNetT: + the time token



def _stamp():
    """Provenance of a summary (bench.summary_stamp): the git head (F5H_HEAD) and the engine source hash."""
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    import bench
    return bench.summary_stamp()

def load(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        did = int(r["Dispatch_Id"])
        rows[did] = (r["Kernel_Name"], rows.get(did, (None, 0.0))[1] + float(r["Counter_Value"]))
    return [(d, n, v) for d, (n, v) in sorted(rows.items())]


def classify(disp):
    cls = {}
    for i, (_, name, _) in enumerate(disp):
        if "chain_kernel" in name:  # the phase chain (chain.hip): out-proj .. next QKV as one launch
            cls[i] = "chain"
    for i, (_, name, _) in enumerate(disp):
        if "attn16" in name or "attn_f32" in name:
            cls[i] = "attention"
            folded = i + 2 < len(disp) and "gemm" in disp[i + 2][1] and "chain_kernel" not in disp[i + 2][1]
            for off, c in (ORDER_FOLD if folded else ORDER).items():
                if 0 <= i + off < len(disp) and "chain_kernel" not in disp[i + off][1] and \
                        ("gemm" in disp[i + off][1]) == (c in GEMMS):
                    cls.setdefault(i + off, c)
        elif "conv16_kernel" in name or "conv_kernel" in name:  # ConvPositionEmbedding layers (conv.hip)
            cls[i] = "conv"
    return cls


def algorithmic(c, S=2, L=1876, d=1024, ff=2048, H=16, es=2, rb=2):
    """rb: residual stream width (2 on the 16-bit DiT path since EPI_RESID16, 4 with F5H_RES32=1)."""
    rows = S * L
    gemm = {"qkv": (d, 3 * d, es), "out": (d, d, 2 * rb), "ffn1": (d, ff, es), "ffn2": (ff, d, 2 * rb)}
    if c in gemm:
        K, N, out_b = gemm[c]
        return es * (rows * K + N * K) + out_b * rows * N
    if c == "attention":
        return 4 * es * S * H * L * 64  # q, k, v read + o written
    if c in ("norm", "norm1"):
        return rows * d * (rb + es)
    if c == "conv":  # the two grouped conv layers (31 taps, 16 groups), mean: layer 1 fp32 input + operand output,
        # layer 2 operand input + fp32 residual (the input embedding) + residual-stream output; plus the weights
        return rows * d * ((4 + es) + (es + 4 + rb)) / 2 + d * (d // 16) * 31 * es
    return None


def main(fpath, wpath, out, config="c2"):
    shp = SHAPES[config]
    n = int(os.environ.get("F5H_TRACE_WARM", "3")) + int(os.environ.get("F5H_TRACE_CALLS", "3"))
    calls = (f"{n} CFM.sample call{'s' if n > 1 else ''}"
             + (" in eager mode (F5H_GRAPH=0: graph-mode passes at this shape never finish under the profiler)"
                if os.environ.get("F5H_GRAPH") == "0" else " in the shipped graph mode"))
    f = load(fpath, "FETCH_SIZE")
    w = load(wpath, "WRITE_SIZE")
    cf, cw = classify(f), classify(w)
    acc = defaultdict(lambda: {"f": [], "w": []})
    for i, (_, _, v) in enumerate(f):
        if i in cf:
            acc[cf[i]]["f"].append(v)
    for i, (_, _, v) in enumerate(w):
        if i in cw:
            acc[cw[i]]["w"].append(v)
    res = {}
    for c, a in acc.items():
        if not a["f"] or not a["w"]:
            continue
        fk, wk = statistics.median(a["f"]), statistics.median(a["w"])
        hbm = (2.0 * fk + wk) * 1024.0
        alg = algorithmic(c, S=shp["S"], L=shp["L"], d=shp["dim"], ff=shp["ff"])
        res[c] = {"fetch_size_kb": fk, "write_size_kb": wk, "dispatches": len(a["f"]), "hbm_bytes": hbm,
                  "algorithmic_bytes": alg, "hbm_over_algorithmic": round(hbm / alg, 3) if alg else None}
    j = {"note": f"{config.upper()} call (S={shp['S']}, L={shp['L']}, depth {shp['depth']}, bf16), rocprofv3 --pmc "
                 f"one counter per pass over {calls} (tools/trace_c2.py run {config}); median per dispatch; hbm_bytes = "
                 "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reads half of wide streaming reads, "
                 "MI355X_MICROARCH.md HBM section); FETCH counts Infinity-Cache hits too",
         # bench.py attaches traffic only at this shape (the config key only when not C2, as the C2 summaries
         # committed before it had none)
         "shape": {k: shp[k] for k in ("S", "L", "dim", "depth")} | ({"config": config} if config != "c2" else {}),
         "classes": res}
    j.update(_stamp())
    json.dump(j, open(out, "w"), indent=1)
    print(json.dumps(j, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
