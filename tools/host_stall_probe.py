"""Which host-side steps of a CFM.sample call wait for unrelated device work: a ~1 s spin kernel runs
on another stream while each step is timed on the host (round-3 diagnostic for the graph-cache
eviction test). Prints one line per step: host ms and whether the spin was still running after."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import golden_cases as gc  # noqa: E402
from f5_tts_amd import synthetic  # noqa: E402
from f5_tts_amd.model import CFM, DiT  # noqa: E402

DEV = "cuda:0"


def model():
    arch = gc.arch_of("tiny")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    return CFM(transformer=net, num_channels=100, compute="bf16").to(DEV)


def main():
    m = model()
    other = torch.cuda.Stream()

    def timed(what, fn):
        with torch.cuda.stream(other):
            torch.cuda._sleep(int(2.0e9))
        time.sleep(0.02)
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        busy = not other.query()
        print(f"{what:<52s} host {dt * 1e3:9.3f} ms   spin still running after: {'yes' if busy else 'NO (waited)'}",
              flush=True)
        torch.cuda.synchronize()

    host = torch.arange(1000, dtype=torch.float32)
    timed("torch.tensor(list, device=cuda)", lambda: torch.tensor([1, 2, 3], device=DEV))
    timed("pageable CPU tensor .to(cuda)", lambda: host.to(DEV))
    timed("pinned CPU tensor .to(cuda, non_blocking)", lambda: host.pin_memory().to(DEV, non_blocking=True))
    timed("torch.empty 64 MB (new size)", lambda: torch.empty(16 << 20, device=DEV))
    timed("torch.empty 3 MB", lambda: torch.empty(777777, device=DEV))
    for i, n in enumerate((61, 67, 73)):
        inp = synthetic.make_case(B=1, ref_frames=n // 3, total_frames=n, n_text=8, vocab=64, seed=500 + i)
        y0 = synthetic.reference_noise(inp["duration"], i)
        cond, text = inp["cond"].to(DEV), inp["text"].to(DEV)
        y0d = y0.to(DEV)
        torch.cuda.synchronize()
        timed(f"CFM.sample new shape N={n} (capture)", lambda: m.sample(
            cond=cond, text=text, duration=inp["duration"], lens=inp["lens"], steps=2, cfg_strength=2.0,
            sway_sampling_coef=-1.0, y0=y0d, keep_trajectory=False))
        timed(f"CFM.sample same shape N={n} (replay)", lambda: m.sample(
            cond=cond, text=text, duration=inp["duration"], lens=inp["lens"], steps=2, cfg_strength=2.0,
            sway_sampling_coef=-1.0, y0=y0d, keep_trajectory=False))


def eviction():
    """The graph-cache eviction scenario of test_graph_eviction_never_waits_for_other_streams, with
    F5H_HOST_TRACE=1 phase timings on stderr."""
    m = model()
    other = torch.cuda.Stream()
    cases = []
    for i in range(24):
        n = 40 + 5 * i
        inp = synthetic.make_case(B=1, ref_frames=n // 3, total_frames=n, n_text=8, vocab=64, seed=300 + i)
        cases.append((inp, synthetic.reference_noise(inp["duration"], i)))

    def run(inp, y0):
        m.sample(cond=inp["cond"].to(DEV), text=inp["text"].to(DEV), duration=inp["duration"], lens=inp["lens"],
                 steps=2, cfg_strength=2.0, sway_sampling_coef=-1.0, y0=y0.to(DEV), keep_trajectory=False)

    for c in cases[:17]:
        run(*c)
    torch.cuda.synchronize()
    with torch.cuda.stream(other):
        torch.cuda._sleep(int(2.0e9))
    for i, c in enumerate(cases[17:]):
        print(f"--- evicting call {i}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        run(*c)
        print(f"evicting call {i}: host {(time.perf_counter() - t0) * 1e3:.3f} ms, spin running: {not other.query()}",
              flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "evict":
        eviction()
    else:
        main()
