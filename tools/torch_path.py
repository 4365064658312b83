"""Same-node PyTorch yardstick for a whole C2 call.

The reference's GPU path is composed PyTorch: aten GEMMs (hipBLASLt on ROCm), F.scaled_dot_product_attention,
MIOpen conv1d and elementwise kernels (modules.py:481-483,519,548; the pytorch backend of
runtime/triton_trtllm/benchmark.py:296-313). This script runs the oracle's restatement of that path
(oracle/ref_cpu.py: the same functions the parity tests pin to the reference's own outputs) once per call on the
MI355X through torch-ROCm, weights in bf16 and the ops under torch.autocast(bf16) (the restatement keeps a few
pieces in fp32, as the reference's x_transformers rotary and torch.layer_norm do internally), on the C2 inputs
bench.py uses, and records ms per call plus the kernel-time classes of one call (torch.profiler).

Never part of bench.py's timed region; tools only (the oracle is test infrastructure).

    python tools/torch_path.py [--calls 3] [--out gpurun_out/torch_path_c2.json]
"""

from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "f5-tts_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

CLASSES = (  # kernel name -> class (first match)
    ("attention (SDPA)", r"attn|fmha|flash|softmax|sdpa"),
    ("gemm (hipBLASLt / rocBLAS)", r"Cijk|gemm|Gemm|GEMM|matmul|hipblaslt"),
    ("conv (MIOpen)", r"conv|Conv|naive_conv|igemm|miopen"),
    ("layer_norm", r"layer_norm|LayerNorm|norm"),
    ("elementwise / copies", r"elementwise|vectorized|unrolled|copy|Copy|cat|fill|reduce|index|where|mish|gelu"),
)


def classify(name):
    for cls, pat in CLASSES:
        if re.search(pat, name):
            return cls
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "torch_path_c2.json"))
    args = ap.parse_args()
    from f5_tts_amd import configs, synthetic
    from oracle import ref_cpu

    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    case = synthetic.c2_case()
    arch = configs.get_arch(case["preset"])
    W = {k: v.to(dev, torch.bfloat16) for k, v in synthetic.make_weights_torch(arch).items()}
    inp = synthetic.make_case(B=1, ref_frames=[case["ref"]], total_frames=[case["total"]], n_text=[case["nt"]],
                              seed=1234)
    kw = dict(lens=inp["lens"].to(dev), steps=case["nfe"], cfg_strength=case["cfg"],
              sway_sampling_coef=case["sway"], seed=0)
    cond, text, dur = inp["cond"].to(dev), inp["text"].to(dev), inp["duration"].to(dev)
    gen = case["total"] - case["ref"]
    torch.set_default_device(dev)

    def call():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            out, _ = ref_cpu.cfm_sample(W, arch, cond, text, dur, **kw)
        return out

    call()  # warm (kernel selection, allocator)
    torch.cuda.synchronize()
    times = []
    for _ in range(args.calls):
        t0 = time.perf_counter()
        call()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ms = min(times) * 1e3
    print(f"torch path C2: {[round(t * 1e3, 1) for t in times]} ms per call", flush=True)

    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        call()
        torch.cuda.synchronize()
    kern = {}
    for ev in prof.key_averages():
        dt = getattr(ev, "device_time_total", None)
        if dt is None:
            dt = getattr(ev, "cuda_time_total", 0)
        if dt and ev.key and not ev.key.startswith(("aten::", "cuda", "hip", "Memcpy", "Memset")):
            kern[ev.key] = (kern.get(ev.key, (0.0, 0))[0] + dt, kern.get(ev.key, (0.0, 0))[1] + ev.count)
    total_us = sum(v[0] for v in kern.values())
    classes = {}
    for name, (us, n) in kern.items():
        c = classes.setdefault(classify(name), {"us": 0.0, "launches": 0})
        c["us"] += us
        c["launches"] += n
    for c in classes.values():
        c["ms"] = round(c.pop("us") / 1e3, 3)
        c["share"] = round(c["ms"] * 1e3 / total_us, 4) if total_us else None
    top = sorted(kern.items(), key=lambda kv: -kv[1][0])[:15]
    res = {
        "what": "oracle/ref_cpu.py restatement of CFM.sample at C2 on MI355X via torch-ROCm: bf16 weights, ops under "
                "torch.autocast(bf16): aten GEMM (hipBLASLt), SDPA, MIOpen conv1d, elementwise (eager, one stream)",
        "config": "C2: F5TTS_v1_Base, B=1, 938 + 938 frames, 300 tokens, NFE 16 EPSS + sway -1, CFG 2",
        "calls_ms": [round(t * 1e3, 2) for t in times],
        "ms_per_call": round(ms, 2),
        "mel_frames_per_s": round(gen / (ms / 1e3), 1),
        "rtf": round(ms / 1e3 / (gen * 256 / 24000), 5),
        "kernel_ms_per_call": round(total_us / 1e3, 2),
        "kernel_launches_per_call": sum(v[1] for v in kern.values()),
        "classes": classes,
        "top_kernels": [{"name": k[:120], "ms": round(v[0] / 1e3, 3), "launches": v[1]} for k, v in top],
        "torch": torch.__version__,
        "device": torch.cuda.get_device_name(0),
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("ms_per_call", "mel_frames_per_s", "kernel_ms_per_call",
                                          "kernel_launches_per_call")}), flush=True)
    print(json.dumps(res["classes"], indent=1), flush=True)


if __name__ == "__main__":
    main()
