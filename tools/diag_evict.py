"""Diagnostic for test_graph_eviction_never_waits_for_other_streams: per new-shape call while a spin
kernel occupies another stream, time the input copies and the sample call separately and count the
caching allocator's device allocations / frees around each call."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import torch
import golden_cases as gc
from f5_tts_amd import synthetic
from f5_tts_amd.model import CFM, DiT

DEV = "cuda:0"


def model():
    arch = gc.arch_of("tiny")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute="bf16").to(DEV)


def case(n, i):
    inp = synthetic.make_case(B=1, ref_frames=n // 3, total_frames=n, n_text=8, vocab=64, seed=300 + i)
    return inp, synthetic.reference_noise(inp["duration"], i)


def run(m, inp, y0):
    t0 = time.perf_counter()
    c, tx, y = inp["cond"].to(DEV), inp["text"].to(DEV), y0.to(DEV)
    t1 = time.perf_counter()
    out, _ = m.sample(cond=c, text=tx, duration=inp["duration"], lens=inp["lens"], steps=2, cfg_strength=2.0,
                      sway_sampling_coef=-1.0, y0=y, keep_trajectory=False)
    t2 = time.perf_counter()
    return t1 - t0, t2 - t1


def stats():
    s = torch.cuda.memory_stats()
    return s.get("num_device_alloc", 0), s.get("num_device_free", 0), s.get("num_sync_all_streams", 0)


for rep in range(2):
    m = model()
    cases = [case(40 + 5 * i, i) for i in range(24)]
    for inp, y0 in cases[:17]:
        run(m, inp, y0)
    torch.cuda.synchronize()
    other = torch.cuda.Stream()
    with torch.cuda.stream(other):
        torch.cuda._sleep(int(2.0e9))
    rows = []
    for inp, y0 in cases[17:]:
        a0 = stats()
        cp, sm = run(m, inp, y0)
        a1 = stats()
        rows.append((round(cp, 4), round(sm, 4), tuple(b - a for a, b in zip(a0, a1))))
    busy = not other.query()
    torch.cuda.synchronize()
    print(f"rep {rep}: spin still busy {busy}; (copy s, sample s, (device allocs, frees, sync_all)) per call:", flush=True)
    for r in rows:
        print("  ", r, flush=True)
    del m
