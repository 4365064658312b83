"""A/B of engine execution options on a BASELINE config, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24). Prints ms per CFM.sample call per arm and checks that every
arm's output is bitwise identical to the first arm's.

    python tools/ab_c2.py [--config c2] [--rounds 5] [--calls 5] [--arms streams1,streams2]
Arms: streams1 / streams2 (f5h_set_cfg_streams), gemmN (f5h_gemm_force_config N, -1 = auto),
eager (step graph off), chain0 / chain1 (f5h_set_chain), fold0 / fold1 (f5h_set_ln_fold). Outputs are compared for the warm call (a graph capture)
AND the last timed call of every arm (graph replays only: round 6 found a bug that only replays showed).
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from f5_tts_amd import synthetic  # noqa: E402
from f5_tts_amd.engine import gemm_force_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--compute", default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--arms", default="streams1,streams2")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    case = {"c2": synthetic.c2_case, "c3": synthetic.c3_case, "c4": synthetic.c4_case, "c5": synthetic.c5_case}[a.config]()
    model, arch = bench.build_model(case["preset"], a.compute, dev)
    B = case["B"]
    refs = case["ref"] if isinstance(case["ref"], list) else [case["ref"]] * B
    tots = case["total"] if isinstance(case["total"], list) else [case["total"]] * B
    inp = synthetic.make_case(B=B, ref_frames=refs, total_frames=tots, n_text=case["nt"])
    kw = dict(cond=inp["cond"].to(dev), text=inp["text"].to(dev), duration=inp["duration"].to(dev),
              lens=inp["lens"].to(dev), steps=case["nfe"], cfg_strength=case["cfg"],
              sway_sampling_coef=case["sway"], seed=0, keep_trajectory=False)
    eng = model.transformer.get_engine(model.engine_compute(), dev)
    arms = a.arms.split(",")

    def setup(arm):
        eng.set_graph_mode(arm != "eager")
        eng.set_cfg_streams(1 if arm == "streams1" else (2 if arm == "streams2" else 0))
        gemm_force_config(int(arm[4:]) if arm.startswith("gemm") else -1)
        if arm.startswith("chain"):
            eng.set_chain(arm == "chain1")
        if arm.startswith("fold"):
            eng.set_ln_fold(arm == "fold1")

    outs, lasts, times = {}, {}, {arm: [] for arm in arms}
    for arm in arms:  # warm every arm (graph capture) before timing
        setup(arm)
        outs[arm] = model.sample(**kw)[0].clone()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for arm in arms:
            setup(arm)
            model.sample(**kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.calls):
                last = model.sample(**kw)[0]
            torch.cuda.synchronize()
            lasts[arm] = last.clone()
            times[arm].append((time.perf_counter() - t0) / a.calls * 1e3)
    setup(arms[0])
    for arm in arms:
        t = sorted(times[arm])
        same = torch.equal(outs[arm], outs[arms[0]]) and torch.equal(lasts[arm], outs[arms[0]])
        ref = outs[arms[0]].float()
        rel = float((lasts[arm].float() - ref).norm() / ref.norm())
        print(f"{arm:10s} median {t[len(t) // 2]:8.3f} ms  min {t[0]:8.3f} ms  bitwise-equal-to-{arms[0]} {same} "
              f"(warm and last timed call; rel-L2 of the last {rel:.3e})", flush=True)


if __name__ == "__main__":
    main()
