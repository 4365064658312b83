"""Diagnostic: what an engine drop costs other threads/streams while unrelated work runs.

A ~1 s spin kernel occupies stream A. The test drops a model (engine + Vocos + log-mel) and times:
  drop      the dropping thread (del + gc.collect)
  launch_c  a small torch op launched and synchronised on a third stream C right after the drop
  query_a   hipStreamQuery on stream A (does not wait for A's work itself)
while the reaper thread releases the objects (their own events, then their device memory).
Prints one line per phase with host seconds since the spin was launched.
"""
import gc
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import golden_cases as gcases  # noqa: E402
from f5_tts_amd import _lib, synthetic  # noqa: E402
from f5_tts_amd.model import CFM, DiT  # noqa: E402

DEV = "cuda:0"


def model():
    arch = gcases.arch_of("tiny")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute="bf16").to(DEV)


def run(m):
    inp = synthetic.make_case(B=1, ref_frames=20, total_frames=60, n_text=8, vocab=64, seed=3)
    y0 = synthetic.reference_noise(inp["duration"], 1)
    out, _ = m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"],
                      lens=inp["lens"], steps=2, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV),
                      keep_trajectory=False)
    return out


def main():
    m = model()
    run(m)
    torch.cuda.synchronize()
    a, c = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.randn(1024, device=DEV)
    with torch.cuda.stream(a):
        torch.cuda._sleep(int(2.0e9))
    t0 = time.perf_counter()
    run(m)
    t_run = time.perf_counter() - t0
    t1 = time.perf_counter()
    del m
    gc.collect()
    t_drop = time.perf_counter() - t1
    t2 = time.perf_counter()
    with torch.cuda.stream(c):
        y = x * 2
    c.synchronize()
    t_c = time.perf_counter() - t2
    t3 = time.perf_counter()
    busy = not a.query()
    t_q = time.perf_counter() - t3
    pend = _lib.lib().f5h_release_pending(0)
    t4 = time.perf_counter()
    _lib.lib().f5h_release_pending(1)
    t_rel = time.perf_counter() - t4
    a.synchronize()
    t_spin = time.perf_counter() - t0
    print(f"run {t_run:.4f}s drop {t_drop:.4f}s third-stream op {t_c:.4f}s query_a {t_q:.4f}s (busy={busy}) "
          f"pending after drop {pend}, release wait {t_rel:.4f}s, spin done at {t_spin:.3f}s; y ok {bool(y.sum() != 0)}",
          flush=True)


if __name__ == "__main__":
    main()
