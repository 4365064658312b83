"""Does CFM.sample return before the GPU finishes (no host sync in the preamble)?
Prints the host time each call takes to return, for back-to-back C2 calls without synchronizing."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd")]


def main():
    import torch

    import bench
    from f5_tts_amd import synthetic

    dev = torch.device("cuda", 0)
    case = synthetic.c2_case()
    model, arch = bench.build_model(case["preset"], "bf16", dev)
    inp = synthetic.make_case(B=1, ref_frames=[case["ref"]], total_frames=[case["total"]], n_text=case["nt"])
    kw = dict(cond=inp["cond"].to(dev), text=inp["text"].to(dev), duration=inp["duration"], lens=inp["lens"],
              steps=case["nfe"], cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], seed=0,
              keep_trajectory=False)
    print("duration", type(inp["duration"]), "lens", type(inp["lens"]))
    for _ in range(3):
        model.sample(**kw)
    torch.cuda.synchronize()
    if len(sys.argv) > 1 and sys.argv[1] == "profile":
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
    t0 = time.perf_counter()
    rets = []
    for _ in range(6):
        model.sample(**kw)
        rets.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    if len(sys.argv) > 1 and sys.argv[1] == "profile":
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    print("host return times (ms):", [round(r * 1e3, 2) for r in rets], "all done", round(t1 * 1e3, 2))


if __name__ == "__main__":
    main()
