"""Benchmark: F5-TTS CFM.sample on MI355X through the HIP engine.

Workload (BASELINE.json configs[1] = SURVEY C2): F5TTS_v1_Base, bf16 MFMA engine, NFE 16
(EPSS grid) + sway -1, CFG 2.0, B=1 per GPU, 10 s prompt (938 ref frames) + 938 generated
frames = 1876 frames, 300 text tokens. One "step" = one pass of the data-parallel job driver
(f5_tts_amd.parallel.run_sharded: LPT shard -> length buckets -> CFM.sample per batch -> keep the
generated frames -> RCCL gather of the finished mels when N > 1), i.e. one full `CFM.sample()` per
GPU at C2. Synthetic data and hash-PRNG weights of the real architecture (checkpoints are
network-only); inputs are resident on the device before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5] [--compute bf16|fp16]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)

`--gpus N` alone starts the N rank processes itself (one per GPU, RCCL); under an outer launcher
(torchrun) WORLD_SIZE must equal N. Prints ONE JSON line on rank 0 (contract in the task statement).
`roofline` is the kernel class that takes the most time per step (in-kernel device wall-clock stamps,
probed live over the timed region, with the committed rocprofv3 average and MFMA-busy counters of the
class beside them); `roofline_classes` lists every class from a probe pre-pass. The default (and the
driver's) workload is C2; --config c1 (Small 4-layer, NFE 4), c3 (B=32 mixed lengths, NFE 32,
batch-mask path), c4 (32 utterances per GPU) and c5 (E2 UNetT, B=8) measure the other BASELINE.json
configs the same way. `cpu_baseline` (rank 0, N=1): the oracle timed in full for C1/C2, per NFE step on
a slice of the batch and extrapolated for C3/C4/C5.
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


def _same_shape(a, b, match_compute=True):
    """Launch shapes agree on S, L, dim, depth (and on the workload when both name one); timings also on
    the compute dtype (summaries without one were measured in bf16: fp16 runs at a lower clock)."""
    if not a or not b:
        return False
    keys = ("S", "L", "dim", "depth")
    if any(a.get(k) != b.get(k) for k in keys):
        return False
    if match_compute and a.get("compute", "bf16") != b.get("compute", "bf16"):
        return False
    return a.get("config") is None or b.get("config") is None or a["config"] == b["config"]


PROFILES = os.path.join(REPO, "profiles")  # committed summaries (older rounds' files live in profiles/archive/)
_SRC_HASH = None


def src_hash():
    """Content hash of the engine's sources (f5-tts_amd/csrc, include/f5h.h): what a profile summary was
    measured with (summaries record it as "src_hash", with the git "head" they were committed from), so a
    bench line can say whether an attached summary matches the library it ran."""
    global _SRC_HASH
    if _SRC_HASH is None:
        import glob
        import hashlib

        h = hashlib.sha256()
        files = sorted(glob.glob(os.path.join(REPO, "f5-tts_amd", "csrc", "*")))
        files.append(os.path.join(REPO, "include", "f5h.h"))
        for f in files:
            if os.path.isfile(f) and (f.endswith((".hip", ".h", ".cpp")) or os.path.basename(f) == "Makefile"):
                h.update(os.path.basename(f).encode())
                h.update(open(f, "rb").read())
        _SRC_HASH = h.hexdigest()[:16]
    return _SRC_HASH


def summary_stamp():
    """The provenance fields a profile summary carries (tools/class_profile.py, tools/pmc_classes.py):
    the git head it was measured at (F5H_HEAD, passed in by the launching script: the GPU box has no .git)
    and the source hash of the tree it ran."""
    return {"head": os.environ.get("F5H_HEAD", "unknown"), "src_hash": src_hash()}


def profile_class(pattern, kernel_class, shape, match_compute=True):
    """A kernel class's entry in the newest committed profile summary (profiles/<pattern>, written by
    tools/pmc_classes.py or tools/class_profile.py) measured at this launch shape, its source file, and its
    provenance {"head", "src_hash", "matches_build"}: the git head the summary was measured at and whether its
    source hash is this tree's. Summaries of other shapes are never attached (None, reason, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(PROFILES, pattern)))
    if not files:
        return None, None, None
    for f in reversed(files):
        d = json.load(open(f))
        if _same_shape(d.get("shape"), shape, match_compute):
            prov = {"head": d.get("head"), "src_hash": d.get("src_hash"),
                    "matches_build": d.get("src_hash") == src_hash()}
            return d.get("classes", {}).get(kernel_class), os.path.relpath(f, REPO), prov
    return None, f"no profiles/{pattern} summary at shape {shape} (newest: {os.path.relpath(files[-1], REPO)})", None


def pmc_traffic(kernel_class, shape):
    """HBM bytes per launch of a kernel class from the newest committed rocprofv3 PMC summary at this
    launch shape (profiles/*_pmc_classes.json, tools/pmc_classes.py: separate FETCH_SIZE and WRITE_SIZE
    passes, 2 x FETCH_SIZE (gfx950 counts half of wide streaming reads, MI355X_MICROARCH.md §HBM) +
    WRITE_SIZE), and its source file; other shapes get None. Bytes do not depend on the 16-bit type."""
    ent, src, prov = profile_class("*_pmc_classes*.json", kernel_class, shape, match_compute=False)
    return (ent["hbm_bytes"] if ent else None), src, prov


def build_model(preset, compute, device):
    from f5_tts_amd import configs, synthetic
    from f5_tts_amd.model import CFM, DiT, UNetT

    arch = configs.get_arch(preset)
    cls = DiT if arch["backbone"] == "DiT" else UNetT
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = cls(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute=compute).to(device), arch


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """Physical cores of the host, and the physical cores this process may run on: the CPUs of its
    affinity mask counted once per (package, core) from /proc/cpuinfo, capped by a cgroup v2 CPU
    quota when one is set. The CPU baseline runs one thread per usable physical core."""
    phys, cpu_core = set(), {}
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (x.strip() for x in line.split(":", 1))
                cur[k] = v
            elif cur:
                if "processor" in cur:
                    key = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                    phys.add(key)
                    cpu_core[int(cur["processor"])] = key
                cur = {}
        if cur and "processor" in cur:
            key = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
            phys.add(key)
            cpu_core[int(cur["processor"])] = key
    except OSError:
        pass
    aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else set(range(os.cpu_count() or 1))
    usable = len({cpu_core.get(c, ("?", c)) for c in aff}) if cpu_core else len(aff)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    if quota is not None:
        usable = min(usable, quota)
    return {"physical": len(phys) or (os.cpu_count() or 1), "usable": max(1, usable), "affinity_cpus": len(aff),
            "cgroup_cpus": quota}


def _as_list(v, n):
    return list(v) if isinstance(v, list) else [v] * n


# utterances of the batch the CPU baseline runs per config: C1/C2 whole calls; C3/C4/C5 a slice of the
# batch at the batch's padded length, one and two NFE steps, extrapolated
CPU_SLICE = {"c1": None, "c2": None, "c3": 2, "c4": 2, "c5": 2}


def cpu_baseline(config, case, arch, threads):
    """Oracle (fp32 PyTorch-CPU restatement of the reference path, `oracle/ref_cpu.py`) timed on the
    host cores.

    C1 and C2: one full CFM.sample call (text embedding, NFE packed CFG forwards, Euler, final overwrite).
    C3/C4/C5 ("timed per NFE step and extrapolated x NFE"): a slice of `b` utterances of
    the batch (the longest and the shortest, padded to the batch's length, batch-mask path as B > 1) is run
    for one and for two NFE steps; per step = t2 - t1, per call fixed part = t1 - per step, and the batch
    call is extrapolated as (fixed + NFE * per step) * B / b (the packed forward is linear in the batch at a
    fixed padded length)."""
    from f5_tts_amd import synthetic
    from oracle import ref_cpu

    torch.set_num_threads(threads)
    W = synthetic.make_weights_torch(arch)
    B = case["B"]
    refs, tots, nts = _as_list(case["ref"], B), _as_list(case["total"], B), _as_list(case["nt"], B)
    gen_batch = sum(t - r for t, r in zip(tots, refs))
    b = CPU_SLICE.get(config)
    kw = dict(cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=0)
    vocab = min(2545, arch["text_num_embeds"])
    if b is None:
        inp = synthetic.make_case(B=B, ref_frames=refs, total_frames=tots, n_text=nts, vocab=vocab)
        t0 = time.perf_counter()
        ref_cpu.cfm_sample(W, arch, inp["cond"], inp["text"], inp["duration"], lens=inp["lens"], steps=case["nfe"], **kw)
        full = time.perf_counter() - t0
        sample = (f"oracle/ref_cpu.py fp32, one full {case['nfe']}-step {config.upper()} call ({full:.1f}s, "
                  f"{gen_batch} generated frames)")
        extra = {"extrapolated": False, "seconds": round(full, 2)}
    else:
        order = sorted(range(B), key=lambda i: tots[i])
        pick = [order[-1], order[0]][:b]  # the longest sets the padded length; the shortest rides along
        n_pad = max(tots)
        inp = synthetic.make_case(B=b, ref_frames=[refs[i] for i in pick], total_frames=[n_pad] * b,
                                  n_text=[nts[i] for i in pick], vocab=vocab)
        times = []
        for ms in (1, 2):
            t0 = time.perf_counter()
            ref_cpu.cfm_sample(W, arch, inp["cond"], inp["text"], inp["duration"], lens=inp["lens"],
                               steps=case["nfe"], max_steps=ms, **kw)
            times.append(time.perf_counter() - t0)
        per_step = max(times[1] - times[0], 1e-9)
        fixed = max(times[0] - per_step, 0.0)
        full = (fixed + case["nfe"] * per_step) * B / b
        sample = (f"oracle/ref_cpu.py fp32, {b} of the {B} utterances padded to {n_pad} frames, 1 and 2 NFE steps "
                  f"({times[0]:.1f}s, {times[1]:.1f}s): per step {per_step:.2f}s, fixed {fixed:.2f}s, extrapolated to "
                  f"the {case['nfe']}-step call of all {B} ({full:.1f}s, {gen_batch} generated frames)")
        extra = {"extrapolated": True, "seconds_measured": round(sum(times), 2), "seconds": round(full, 2),
                 "per_step_s": round(per_step, 3), "slice_utterances": b}
    line = {"value": round(gen_batch / full, 3), "unit": "mel-frames/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": sample + f" on {cpu_model()}, {torch.get_num_threads()} threads (one per physical core "
                               f"usable by this process)",
            "rtf": round(full / (gen_batch * HOP / SR), 4)}
    line.update(extra)
    return line


def class_flops(kc, arch, S, L):
    """Algorithmic FLOPs of one launch of a probed kernel class (SURVEY §8d per-op terms). The phase chain (C2's
    shipped form: one launch per layer running out-proj, LayerNorm, FFN1, FFN2, the next layer's LayerNorm and its
    QKV) is priced on its GEMM phases, averaged over the depth launches of a step (the last layer's has no QKV)."""
    d, ff = arch["dim"], int(arch["dim"] * arch["ff_mult"])
    chain = 2.0 * S * L * d * (d + 2 * ff) + 2.0 * S * L * d * 3 * d * (arch["depth"] - 1) / arch["depth"]
    return {"attention": attn_flops(S, arch["heads"], L), "ffn1": 2.0 * S * L * d * ff, "ffn2": 2.0 * S * L * d * ff,
            "qkv": 2.0 * S * L * d * 3 * d, "out": 2.0 * S * L * d * d,
            "conv": 2.0 * S * L * d * (d // 16) * 31, "chain": chain}.get(kc, 0.0)


def resid_bytes(arch, esz=2):
    """Width of the residual stream: the operand dtype in the 16-bit modes, for DiT and UNetT alike
    (engine.cpp backbone_part `r16`; the UNetT stream is 16-bit since a041ce0), fp32 in the fp32 parity
    mode."""
    del arch  # the same width on both backbones
    return esz if esz == 2 else 4


def class_bytes(kc, arch, S, L, esz=2):
    """Algorithmic HBM bytes of one launch of an HBM-bound class: the pre-FFN norm reads the residual
    rows and writes the 16-bit GEMM operand."""
    if kc == "norm":
        return S * L * arch["dim"] * (resid_bytes(arch, esz) + esz)
    return 0.0


# "chain": the phase-chain launch (16-bit DiT calls without row masks, i.e. C2): while one of qkv/out/norm/ffn1/ffn2
# is probed the chain is off (those launches are timed one by one), so their rows describe the unchained form and
# the chain row the form C2 ships; the chain probe times nothing at the other configs (no launch: no row)
PROBE_CLASSES = ("qkv", "attention", "out", "norm", "ffn1", "ffn2", "conv", "chain")
PEAK_HBM_GBPS = 8000.0


def live_flops(kc, arch, L, qlens):
    """Algorithmic FLOPs of one launch when the pad-row skip is on (batch path, B > 1): pad query rows' attention
    output is zeroed after to_out (modules.py:551-553), so attention needs only the live query rows (against all
    L keys, or the sequence's own keys with attn_mask_enabled) and the out-projection only the live rows; the other
    classes need every row (pad rows' K/V and hidden states feed live rows of the next layer). None: no change."""
    d = arch["dim"]
    if kc == "attention":
        keys = qlens if arch.get("attn_mask_enabled") else [L] * len(qlens)
        return 4.0 * arch["heads"] * 64 * sum(q * k for q, k in zip(qlens, keys))
    if kc == "out":
        return 2.0 * sum(qlens) * d * d
    return None


def class_entry(kc, avg_ms, n, arch, S, L, launches_per_call, ms_call, chains=1, config=None, esz=2, compute="bf16",
                qlens=None):
    """One kernel class: algorithmic work per launch slot / average launch span. With the two CFG
    chains captured in parallel (chains = 2, F5H_SPLIT_CFG=1) each chain launches the class
    on half the sequences and the two chains' launches of a class overlap in time, so a slot (the span
    of one launch) covers both halves: flops are counted for all S sequences and the slot count is per
    chain. qlens (per-sequence lengths, CFG copies included) when the pad-row skip runs: attention and the
    out-projection are priced on their live rows (the padded count stays in padded_flops_per_launch)."""
    fl = class_flops(kc, arch, S, L)
    padded = None
    if fl and qlens is not None and len(set(qlens)) > 1:
        lf = live_flops(kc, arch, L, qlens)
        if lf is not None:
            padded, fl = fl, lf
    e = {"kernel": kc, "avg_launch_us": round(avg_ms * 1e3, 3), "sampled_launches": n,
         "launches_per_call": launches_per_call, "cfg_chains": chains,
         "share_of_call": round(avg_ms * launches_per_call / ms_call, 4) if ms_call else None}
    if fl:
        ach = fl / (avg_ms * 1e-3) / 1e12
        e.update(bound="mfma", achieved=round(ach, 2), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                 frac=round(ach / PEAK_BF16_TFLOPS, 4), flops_per_launch=fl)
        if padded is not None:
            e["padded_flops_per_launch"] = padded
            e["flops_basis"] = "live rows (pad-row skip): attention queries / out-proj rows of each sequence's length"
    else:
        by = class_bytes(kc, arch, S, L, esz)
        ach = by / (avg_ms * 1e-3) / 1e9 if by else 0.0
        e.update(bound="hbm", achieved=round(ach, 1), peak=PEAK_HBM_GBPS, unit="GB/s",
                 frac=round(ach / PEAK_HBM_GBPS, 4), bytes_per_launch=by)
    shape = {"S": S, "L": L, "dim": arch["dim"], "depth": arch["depth"], "config": config, "compute": compute}
    traffic, src, tprov = pmc_traffic(kc, shape)
    e["traffic"] = traffic
    e["traffic_source"] = src
    if tprov:
        e["traffic_provenance"] = tprov
    # the same class in the committed rocprofv3 kernel trace (profiler timestamps, dispatch ramp included)
    rp, rsrc, rprov = profile_class("*_rocprof_classes*.json", kc, shape)
    if rp:
        e["rocprof_avg_launch_us"] = rp["avg_launch_us"]
        e["rocprof_source"] = rsrc
        e["rocprof_provenance"] = rprov
        if fl:
            e["rocprof_frac"] = round(fl / (rp["avg_launch_us"] * 1e-6) / 1e12 / PEAK_BF16_TFLOPS, 4)
        elif e.get("bytes_per_launch"):
            e["rocprof_frac"] = round(e["bytes_per_launch"] / (rp["avg_launch_us"] * 1e-6) / 1e9 / PEAK_HBM_GBPS, 4)
    # MFMA utilisation and stall split from the committed SQ counter passes (tools/class_profile.py pmc)
    mf, msrc, mprov = profile_class("*_pmc_mfma*.json", kc, shape)
    if mf:
        e["pmc"] = {k: mf[k] for k in ("mfma_busy", "wait_frac", "issue_stall_frac", "active_frac",
                                       "coexec_over_mfma", "valu_per_mfma", "clock_ghz") if k in mf}
        e["pmc_source"] = msrc
        e["pmc_provenance"] = mprov
    if traffic and kc in ("qkv", "out", "ffn1", "ffn2", "attention", "conv"):
        d, ff = arch["dim"], int(arch["dim"] * arch["ff_mult"])
        kn = {"qkv": (d, 3 * d), "out": (d, d), "ffn1": (d, ff), "ffn2": (ff, d)}.get(kc)
        # rows the launch must touch: with the pad-row skip (live pricing) the out-projection's live rows only
        rows = sum(qlens) if (padded is not None and kc == "out") else S * L
        if kn:  # operands + result at the operand width (residual read+write for RESID)
            K, Nn = kn
            alg = esz * (rows * K + Nn * K) + (2 * resid_bytes(arch, esz) if kc in ("out", "ffn2") else esz) * rows * Nn
        elif kc == "conv":  # the mean of the two grouped conv layers (tools/pmc_classes.py): layer 1 reads the
            # fp32 input embedding and writes the operand dtype, layer 2 reads that, the fp32 input embedding
            # (its residual) and writes the residual stream; plus the 16 groups' 31-tap weights
            per_elem = ((4 + esz) + (esz + 4 + resid_bytes(arch, esz))) / 2
            alg = S * L * d * per_elem + d * (d // 16) * 31 * esz
        elif padded is not None:  # K and V of every row, Q read and O written for the live query rows only
            alg = 2 * esz * arch["heads"] * 64 * (S * L + sum(qlens))
        else:
            alg = 4 * esz * S * arch["heads"] * L * 64
        e["algorithmic_bytes"] = alg
        e["traffic_over_algorithmic"] = round(traffic / alg, 3)
    elif traffic and e.get("bytes_per_launch"):  # an HBM-bound class: against the bytes it is priced on
        e["traffic_over_algorithmic"] = round(traffic / e["bytes_per_launch"], 3)
    return e


def build_job(case, world):
    """The whole job of this run: per-GPU utterances of the config x world (weak scaling), identical on
    every rank (one seeded generator), as parallel.run_sharded utterance dicts."""
    from f5_tts_amd import synthetic

    B = case["B"]
    refs = case["ref"] if isinstance(case["ref"], list) else [case["ref"]] * B
    tots = case["total"] if isinstance(case["total"], list) else [case["total"]] * B
    nts = case["nt"] if isinstance(case["nt"], list) else [case["nt"]] * B
    refs, tots, nts = refs * world, tots * world, nts * world
    inp = synthetic.make_case(B=B * world, ref_frames=refs, total_frames=tots, n_text=nts, seed=1234)
    utts = []
    for i in range(B * world):
        utts.append(dict(cond=inp["cond"][i, : refs[i]], text=inp["text"][i, : nts[i]], ref=refs[i], total=tots[i]))
    return utts


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Without an outer launcher (WORLD_SIZE unset) and N > 1, bench.py "
                         "starts the N rank processes itself; under torchrun WORLD_SIZE must equal N")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="F5TTS_v1_Base")
    ap.add_argument("--compute", default="bf16", choices=("bf16", "fp16", "fp32"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe", default="auto",
                    help="kernel class probed live over the timed region (in-kernel device wall-clock stamps); "
                         "'auto' = the class with the largest share of the call in the probe pre-pass, 'none' = off")
    ap.add_argument("--config", default="c2", choices=("c1", "c2", "c3", "c4", "c5"),
                    help="workload (SURVEY §8d); c2 is the headline line")
    ap.add_argument("--no-vocos", action="store_true", help="skip the +Vocos decode timing (SURVEY §8f1)")
    # launcher test hook: the rank processes run the job driver on CPU over gloo with a stand-in sampler
    ap.add_argument("--standin", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def kfd_gpu_nodes(root="/sys/class/kfd/kfd/topology/nodes"):
    """Physical GPUs from the KFD topology in sysfs (nodes whose properties list `simd_count > 0`; CPU nodes
    have 0). Pure file reads, no HIP call. None when the topology is unreadable."""
    try:
        names = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in names:
        try:
            with open(os.path.join(root, d, "properties")) as f:
                props = dict(ln.split(None, 1) for ln in f if len(ln.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    return n


def visible_gpus(root="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs a rank process would see, counted without any HIP call in the launcher's process
    (torch.cuda.device_count() can fall back to hipGetDeviceCount when amdsmi cannot initialise, which starts
    the HIP runtime in the parent of the ranks): the KFD topology in sysfs, narrowed by ROCR_VISIBLE_DEVICES
    and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES the way the runtime applies them. Only if sysfs is
    unreadable is the count taken from a child process."""
    n = kfd_gpu_nodes(root)
    if n is None:
        import subprocess

        code = "import torch; print(torch.cuda.device_count())"
        try:
            out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                                 env=dict(os.environ))
            return int(out.stdout.strip().splitlines()[-1])
        except (subprocess.SubprocessError, ValueError, IndexError):
            return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args, argv):
    """`--gpus N` with no outer launcher: start N fresh rank processes of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what torchrun would set; the reference's
    benchmark is launched per rank and initialises NCCL itself, benchmark.py:199-212,470-471). The parent
    never touches the GPU (no HIP call before the children exist); rank 0 prints the line. If a rank fails,
    the others are stopped (by PID) and the exit code is non-zero."""
    import subprocess

    n = args.gpus
    if not args.standin:
        have = visible_gpus()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:  # a rank died: the others would wait at a collective forever
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: WORLD_SIZE={env_world} (outer launcher) but --gpus {args.gpus}", file=sys.stderr)
            return 2
    elif args.gpus > 1:
        return launch_ranks(args, argv)
    return run_standin(args) if args.standin else run_rank(args)


def _rank_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _time_region(step, steps, world, device):
    """EXACTLY `steps` calls of `step`, bracketed by a barrier + device synchronisation on both sides;
    the max over ranks. Returns (elapsed seconds, ranks that joined)."""
    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    joined = 1
    if world > 1:
        tt = torch.tensor([elapsed, 1.0], device=device, dtype=torch.float64)
        mx = tt[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        cnt = tt[1:].clone()
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        elapsed, joined = float(mx.item()), int(cnt.item())
    return elapsed, joined


def run_standin(args):
    """Launcher test (CPU): every rank runs parallel.run_sharded over gloo with a deterministic stand-in
    sampler on a small job, through the same timed region and line as the real bench."""
    from f5_tts_amd import parallel

    world, rank, _ = _rank_env()
    if world > 1:
        dist.init_process_group("gloo")
    device = torch.device("cpu")
    utts = []
    for i in range(4 * world):
        total = 64 + 8 * i
        utts.append(dict(cond=torch.full((total // 2, 100), float(i)), text=torch.arange(10) + i, ref=total // 2,
                         total=total))

    def sample(cond, text, dur, lens):
        n = int(dur.max())
        return cond.new_zeros(len(dur), n, 100) + dur.float()[:, None, None]

    plan_all = parallel.plan([u["total"] for u in utts], world, max_batch=4)

    def step():
        return parallel.run_sharded(utts, sample, rank=rank, world=world, device=device, plan_all=plan_all)

    for _ in range(args.warmup):
        got = step()
    elapsed, joined = _time_region(step, args.steps, world, device)
    frames = sum(u["total"] - u["ref"] for u in utts) * args.steps
    got = step()  # a collective: every rank takes part
    if rank == 0:
        print(json.dumps({"metric": "mel-frames/s (launcher stand-in)", "value": round(frames / elapsed, 2),
                          "unit": "mel-frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "ranks_joined": joined, "utterances_gathered": len(got),
                          "config": {"workload": "stand-in", "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def run_rank(args):
    from f5_tts_amd import parallel, synthetic

    world, rank, local = _rank_env()
    if world > 1:
        if torch.cuda.device_count() <= local:
            print(f"bench.py: rank {rank} has LOCAL_RANK {local} but {torch.cuda.device_count()} GPU(s)",
                  file=sys.stderr)
            return 2
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    case = {"c1": synthetic.c1_case, "c2": synthetic.c2_case, "c3": synthetic.c3_case, "c4": synthetic.c4_case,
            "c5": synthetic.c5_case}[args.config]()
    if args.config == "c2":
        case["preset"] = args.preset
    model, arch = build_model(case["preset"], args.compute, device)
    B = case["B"]
    utts = build_job(case, world)
    for u in utts:  # inputs resident in HBM before anything is timed
        u["cond"], u["text"] = u["cond"].to(device), u["text"].to(device)
    plan_all = parallel.plan([u["total"] for u in utts], world, max_batch=B)
    batches = plan_all[rank]
    my = [i for b in batches for i in b]
    gen_frames = sum(utts[i]["total"] - utts[i]["ref"] for i in my)
    job_frames = sum(u["total"] - u["ref"] for u in utts)
    Nmax = max(utts[i]["total"] for i in my)

    def sample(cond, text, dur, lens):
        out, _ = model.sample(cond=cond, text=text, duration=dur, lens=lens, steps=case["nfe"],
                              cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=rank,
                              keep_trajectory=False)
        return out

    def step():
        return parallel.run_sharded(utts, sample, rank=rank, world=world, device=device, plan_all=plan_all)

    eng = model.transformer.get_engine(model.engine_compute(), device)
    esz = 4 if args.compute == "fp32" else 2
    S = 2 * B if case["cfg"] >= 1e-5 else B
    # the engine's CFG launch chains: one packed chain unless F5H_SPLIT_CFG=1 forces the split
    chains = 2 if (case["cfg"] >= 1e-5 and os.environ.get("F5H_SPLIT_CFG") == "1") else 1
    L = Nmax if arch["backbone"] == "DiT" else Nmax + 1
    launches = {"norm": arch["depth"]}
    for kc in ("qkv", "attention", "out", "ffn1", "ffn2"):
        launches[kc] = arch["depth"]
    launches["conv"] = 1
    launches["chain"] = arch["depth"]
    # the pad-row skip runs on the batch path (B > 1, one bucket): attention and out-proj work on live rows
    qlens = None
    if B > 1 and len(batches) == 1 and os.environ.get("F5H_NO_PAD_SKIP") != "1":
        qlens = [utts[i]["total"] for i in batches[0]] * (S // B)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- probe pre-pass: every kernel class timed by its in-kernel stamps, one call each (skipped with
    # --probe none: plain timing runs, e.g. interleaved A/B)
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    ms_pre = (time.perf_counter() - t0) * 1e3
    classes = {}
    for kc in (PROBE_CLASSES if args.probe != "none" else ()):
        eng.probe(kc)
        step()  # captures the probed step graph (the probe is part of the graph key)
        step()
        torch.cuda.synchronize()
        n, ms = eng.probe_read()
        eng.probe(None)
        if n:
            classes[kc] = class_entry(kc, ms / n, n, arch, S, L, launches[kc] * case["nfe"], ms_pre, chains,
                                      config=args.config, esz=esz, compute=args.compute, qlens=qlens)
    probe = args.probe
    if probe == "auto":
        probe = max(classes, key=lambda k: classes[k]["share_of_call"] or 0.0) if classes else "none"

    # ---- timed region (the probed class stamped live; its graph captured before the region)
    if probe != "none":
        eng.probe(probe)
        step()
    elapsed, joined = _time_region(step, args.steps, world, device)
    roof = None
    if probe != "none":
        n_launch, probe_ms = eng.probe_read()
        eng.probe(None)
        if n_launch:
            roof = class_entry(probe, probe_ms / n_launch, n_launch, arch, S, L, launches[probe] * case["nfe"],
                               elapsed / args.steps * 1e3, chains, config=args.config, esz=esz,
                               compute=args.compute, qlens=qlens)
            roof["timing"] = ("in-kernel s_memrealtime stamps: first workgroup start to last wave end of every "
                              "launch of the class in every 4th ODE step inside the timed region (rank 0); "
                              "rocprof_* = the committed rocprofv3 kernel-trace average of the class at this shape")

    frames = job_frames * args.steps
    value = frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    rtf = elapsed / (frames * HOP / SR) * world  # wall / generated audio seconds, per GPU stream

    # +Vocos ("report an optional +Vocos RTF once f1 exists"): the reference decodes each
    # generated mel after sampling (utils_infer.py:506-511, benchmark.py:430-435); timed separately
    # on the same device, K rounds over this rank's utterances, bf16 backbone + fp32 iSTFT head.
    vocos = None
    if not args.no_vocos:
        from f5_tts_amd.vocos import Vocos, make_weights as vocos_weights

        voc = Vocos(compute="bf16")
        voc.load_state_dict(vocos_weights())
        voc.to(device)
        mels = parallel.run_sharded(utts, sample, rank=0, world=1, device=device, plan_all=[batches])
        gens = [mels[i].t().unsqueeze(0).float().contiguous() for i in my]
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
        vocos = {"ms_per_step": round(v_ms, 3),
                 "rtf_with_vocos": round((ms_per_step + v_ms) / 1e3 / (gen_frames * HOP / SR), 5),
                 "note": "Vocos mel-24khz decode of each generated mel (per utterance, as the reference), "
                         "synthetic weights; rtf_with_vocos = (CFM + Vocos wall) / generated audio seconds"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cores()
        cpu = cpu_baseline(args.config, case, arch, threads=hc["usable"])
        cpu["host_cores"] = hc

    # whole-path algorithmic FLOPs: NFE * S * F(N) at the padded length, per rank
    flops_call = case["nfe"] * S * seq_flops(arch, Nmax) * len(batches)
    # useful work of a mixed-length batch: each utterance at its own length
    useful_call = case["nfe"] * (S // B) * sum(seq_flops(arch, utts[i]["total"]) for i in my)
    if rank == 0:
        workloads = {
            "c1": "C1: F5TTS_v1_Small_4L CFM.sample, NFE 4 EPSS + sway -1, CFG 2.0, 1 utterance per GPU, "
                  "282 prompt + 282 generated frames (564), 90 tokens",
            "c2": "C2: F5TTS_v1_Base CFM.sample, NFE 16 EPSS + sway -1, CFG 2.0, 1 utterance per GPU, "
                  "938 prompt + 938 generated frames (1876), 300 tokens",
            "c3": "C3: F5TTS_v1_Base CFM.sample, NFE 32 linspace + sway -1, CFG 2.0, 32 utterances per GPU, "
                  "564..1876 frames (half prompt), padded to 1876, batch-mask path",
            "c4": "C4 (32 per GPU): F5TTS_v1_Base CFM.sample, NFE 16 EPSS + sway -1, CFG 2.0, 32 x world utterances "
                  "(256 over 8 GPUs) LPT-sharded, 938 prompt + 938 generated frames each, 300 tokens, batch path",
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
                       "gen_frames_per_gpu": gen_frames, "nfe": case["nfe"], "parallelism": f"dp{world}"},
            "ranks_joined": joined,
            "rtf": round(rtf, 5),
            "path_tflops": round(flops_call * args.steps * world / elapsed / 1e12, 2),
            "path_tflops_useful": round(useful_call * args.steps * world / elapsed / 1e12, 2),
            "roofline": roof,
            "roofline_classes": classes,
            "vocos": vocos,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
