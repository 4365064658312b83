"""Benchmark: F5-TTS CFM.sample on MI355X through the HIP engine.

Workload (BASELINE.json configs[1] = SURVEY C2): F5TTS_v1_Base, bf16 MFMA engine, NFE 16
(EPSS grid) + sway -1, CFG 2.0, B=1 per GPU, 10 s prompt (938 ref frames) + 938 generated
frames = 1876 frames, 300 text tokens. One "step" = one full `CFM.sample()` call (text
embedding, 16 packed cond/uncond DiT forwards, CFG + Euler, final cond overwrite) plus the
RCCL all-gather of the finished mels. Synthetic data and hash-PRNG weights of the real
architecture (checkpoints are network-only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

Prints ONE JSON line on rank 0 (contract in the task statement). The default (and the driver's)
workload is C2; --config c3 (B=32 mixed lengths, NFE 32, batch-mask path) and c5 (E2 UNetT,
B=8) measure the other BASELINE.json configs the same way (no CPU baseline for those).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "f5-tts_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HOP, SR = 256, 24000
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)


def attn_flops(S, H, L):
    return 4.0 * S * H * L * L * 64  # QK^T + PV per launch


def seq_flops(arch, N):
    """Algorithmic FLOPs of one sequence-forward at padded length N (linear part per
    token + attention part; DiT Base: 378.888e6 N + 90112 N^2; E2 UNetT attends over N+1)."""
    d, depth, ff = arch["dim"], arch["depth"], int(arch["dim"] * arch["ff_mult"])
    per_tok = depth * (8.0 * d * d + 4.0 * d * ff) + 2.0 * 2 * 31 * 64 * d + 2.0 * d * arch["mel_dim"]
    if arch["backbone"] == "DiT":
        L = N
        per_tok += 2.0 * (2 * arch["mel_dim"] + arch["text_dim"]) * d
    else:
        L = N + 1
        per_tok += (depth // 2) * 2.0 * 2 * d * d + 2.0 * (2 * arch["mel_dim"] + arch["text_dim"]) * d
    return per_tok * L + 4.0 * depth * d * L * L


def pmc_traffic(kernel_class):
    """HBM bytes per launch of the probed kernel from the committed rocprofv3 PMC summary
    (profiles/*_pmc_<class>.json, written by tools/profile_round.sh): FETCH_SIZE doubled (it
    reads 1/2 of wide streaming reads on gfx950, MI355X_MICROARCH.md §HBM) + WRITE_SIZE."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_pmc_{kernel_class}.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return (2.0 * d["fetch_size_kb"] + d["write_size_kb"]) * 1024.0, os.path.relpath(files[-1], REPO)


def build_model(preset, compute, device):
    from f5_tts_amd import configs, synthetic
    from f5_tts_amd.model import CFM, DiT, UNetT

    arch = configs.get_arch(preset)
    cls = DiT if arch["backbone"] == "DiT" else UNetT
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = cls(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute=compute).to(device), arch


def cpu_baseline(case, arch, threads):
    """Oracle (fp32 PyTorch-CPU restatement) on a bounded sample of the same workload:
    1 and 3 Euler steps of the C2 call; full-call time extrapolated as prologue + NFE x step."""
    from f5_tts_amd import synthetic
    from oracle import ref_cpu

    torch.set_num_threads(threads)
    W = synthetic.make_weights_torch(arch)
    inp = synthetic.make_case(B=1, ref_frames=case["ref"], total_frames=case["total"], n_text=case["nt"])
    t = {}
    for ms in (1, 3):
        t0 = time.perf_counter()
        ref_cpu.cfm_sample(W, arch, inp["cond"], inp["text"], inp["duration"], lens=inp["lens"], steps=case["nfe"],
                           cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=0, max_steps=ms)
        t[ms] = time.perf_counter() - t0
    step = (t[3] - t[1]) / 2
    full = (t[1] - step) + case["nfe"] * step
    gen = case["total"] - case["ref"]
    return {"value": gen / full, "unit": "mel-frames/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/ref_cpu.py fp32, C2 call truncated to 1 and 3 Euler steps "
                      f"({t[1]:.1f}s, {t[3]:.1f}s); full 16-step call extrapolated = {full:.1f}s",
            "rtf": full / (gen * HOP / SR)}


def class_flops(kc, arch, S, L):
    """Algorithmic FLOPs of one launch of a probed kernel class (SURVEY §8d per-op terms)."""
    d, ff = arch["dim"], int(arch["dim"] * arch["ff_mult"])
    return {"attention": attn_flops(S, arch["heads"], L), "ffn1": 2.0 * S * L * d * ff, "ffn2": 2.0 * S * L * d * ff,
            "qkv": 2.0 * S * L * d * 3 * d, "out": 2.0 * S * L * d * d,
            "conv": 2.0 * S * L * d * (d // 16) * 31}.get(kc, 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="F5TTS_v1_Base")
    ap.add_argument("--compute", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe", default="attention", help="kernel class timed live (in-kernel device wall-clock stamps) for the roofline")
    ap.add_argument("--config", default="c2", choices=("c2", "c3", "c4", "c5"),
                    help="workload (SURVEY §8d); c2 is the headline line")
    ap.add_argument("--no-vocos", action="store_true", help="skip the +Vocos decode timing (SURVEY §8f1)")
    ap.add_argument("--probe-all", action="store_true",
                    help="after the measurement, time every kernel class in its own loop (table on stderr)")
    args = ap.parse_args()

    from f5_tts_amd import synthetic

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    case = {"c2": synthetic.c2_case, "c3": synthetic.c3_case, "c4": synthetic.c4_case,
            "c5": synthetic.c5_case}[args.config]()
    if args.config == "c2":
        case["preset"] = args.preset
    model, arch = build_model(case["preset"], args.compute, device)
    B = case["B"]
    refs = case["ref"] if isinstance(case["ref"], list) else [case["ref"]] * B
    tots = case["total"] if isinstance(case["total"], list) else [case["total"]] * B
    inp = synthetic.make_case(B=B, ref_frames=refs, total_frames=tots, n_text=case["nt"], seed=1234 + rank)
    cond, text = inp["cond"].to(device), inp["text"].to(device)
    duration, lens = inp["duration"].to(device), inp["lens"].to(device)
    gen_frames = sum(t - r for t, r in zip(tots, refs))
    Nmax = max(tots)
    gathered = torch.empty(world, gen_frames * 100, device=device)

    def step():
        out, _ = model.sample(cond=cond, text=text, duration=duration, lens=lens, steps=case["nfe"],
                              cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=rank)
        mel = torch.cat([out[b, refs[b]:tots[b]].reshape(-1) for b in range(B)])
        if world > 1:
            dist.all_gather_into_tensor(gathered, mel)  # finished mels only
        return mel

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    eng = model.transformer.get_engine(model.engine_compute(), device)
    eng.probe(args.probe)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    n_launch, probe_ms = eng.probe_read()
    eng.probe(None)
    if world > 1:
        tt = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    frames = gen_frames * args.steps * world
    value = frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    rtf = elapsed / (frames * HOP / SR) * world  # wall / generated audio seconds, per GPU stream

    S = 2 * B if case["cfg"] >= 1e-5 else B
    H = arch["heads"]
    L = Nmax if arch["backbone"] == "DiT" else Nmax + 1
    roof = None
    if n_launch:
        avg_ms = probe_ms / n_launch
        fl = class_flops(args.probe, arch, S, L)
        ach = fl / (avg_ms * 1e-3) / 1e12 if fl else 0.0
        traffic, tsrc = pmc_traffic(args.probe) if args.config == "c2" else (None, None)
        roof = {"bound": "mfma", "kernel": args.probe, "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                "traffic_unit": "bytes/launch", "traffic_source": tsrc,
                "avg_launch_ms": round(avg_ms, 5), "launches": n_launch, "flops_per_launch": fl,
                "timing": "in-kernel s_memrealtime stamps: first workgroup start to last wave end of the probed "
                          "kernel's launches in every 4th ODE step inside the timed region (all layers)"}

    if args.probe_all and rank == 0:
        import sys
        for kc in ("qkv", "attention", "out", "norm", "ffn1", "ffn2", "conv"):
            eng.probe(kc)
            for _ in range(max(1, min(args.steps, 3))):
                step()
            torch.cuda.synchronize()
            n, ms = eng.probe_read()
            eng.probe(None)
            if n:
                avg = ms / n
                fl = class_flops(kc, arch, S, L)
                print(f"[probe] {kc:9s} sampled launches {n:5d}  avg {avg * 1e3:8.2f} us"
                      + (f"  {fl / (avg * 1e-3) / 1e12:7.1f} TF/s" if fl else ""), file=sys.stderr, flush=True)

    # +Vocos ("report an optional +Vocos RTF once f1 exists"): the reference decodes each
    # generated mel after sampling (utils_infer.py:506-511, benchmark.py:430-435); timed separately
    # on the same device, K rounds over this rank's utterances, bf16 backbone + fp32 iSTFT head.
    vocos = None
    if not args.no_vocos:
        from f5_tts_amd.vocos import Vocos, make_weights as vocos_weights

        voc = Vocos(compute="bf16")
        voc.load_state_dict(vocos_weights())
        voc.to(device)
        out, _ = model.sample(cond=cond, text=text, duration=duration, lens=lens, steps=case["nfe"],
                              cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=rank)
        gens = [out[b, refs[b]:tots[b]].t().unsqueeze(0).float().contiguous() for b in range(B)]
        for g in gens:
            voc.decode(g)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tv = time.perf_counter()
        for _ in range(args.steps):
            for g in gens:
                voc.decode(g)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        vel = time.perf_counter() - tv
        if world > 1:
            tt = torch.tensor([vel], device=device, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            vel = float(tt.item())
        v_ms = vel / args.steps * 1e3
        vocos = {"ms_per_step": round(v_ms, 3), "rtf_with_vocos": round((ms_per_step + v_ms) / 1e3 / (gen_frames * HOP / SR), 5),
                 "note": "Vocos mel-24khz decode of each generated mel (per utterance, as the reference), "
                         "synthetic weights; rtf_with_vocos = (CFM + Vocos wall) / generated audio seconds"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        cpu = cpu_baseline(case, arch, threads=min(16, os.cpu_count() or 1))

    # whole-path algorithmic FLOPs: NFE * S * F(N) at the padded length
    flops_call = case["nfe"] * S * seq_flops(arch, Nmax)
    # useful work of a mixed-length batch: each utterance at its own length
    useful_call = case["nfe"] * (S // B) * sum(seq_flops(arch, t) for t in tots)
    if rank == 0:
        workloads = {
            "c2": "C2: F5TTS_v1_Base CFM.sample, NFE 16 EPSS + sway -1, CFG 2.0, 1 utterance per GPU, "
                  "938 prompt + 938 generated frames (1876), 300 tokens",
            "c3": "C3: F5TTS_v1_Base CFM.sample, NFE 32 linspace + sway -1, CFG 2.0, 32 utterances per GPU, "
                  "564..1876 frames (half prompt), padded to 1876, batch-mask path",
            "c4": "C4 (per rank): F5TTS_v1_Base CFM.sample, NFE 16 EPSS + sway -1, CFG 2.0, 32 utterances per GPU "
                  "(256 over 8 GPUs), 938 prompt + 938 generated frames each, 300 tokens, batch path",
            "c5": "C5: E2TTS_Base (UNetT) CFM.sample, NFE 16 EPSS + sway -1, CFG 2.0, 8 utterances per GPU, "
                  "938 prompt + 938 generated frames, 300 tokens",
        }
        line = {
            "metric": f"mel-frames/s (RTF alongside), {case['preset']} NFE={case['nfe']} CFM.sample",
            "value": round(value, 2),
            "unit": "mel-frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.compute,
            "data": f"synthetic (hash-PRNG weights of {case['preset']}, N(-4,2) cond mel, uniform text ids)",
            "config": {"workload": workloads[args.config], "batch_per_gpu": B, "frames": Nmax,
                       "gen_frames": gen_frames, "nfe": case["nfe"], "parallelism": f"dp{world}"},
            "rtf": round(rtf, 5),
            "path_tflops": round(flops_call * args.steps * world / elapsed / 1e12, 2),
            "path_tflops_useful": round(useful_call * args.steps * world / elapsed / 1e12, 2),
            "roofline": roof,
            "vocos": vocos,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
