"""Where one launch of each hot kernel class spends its time at C2 (round-3 diagnostic): the per-
workgroup timeline stamps (entry, main loop entered = first operand stage landed, main loop done,
exit) of the class's first launch in a probed step, summarised as
  spread   last workgroup entry - first entry (dispatch of the grid)
  ramp     loop entered - entry (first stage latency), median / max
  loop     loop done - loop entered, median / max
  epi      exit - loop done (epilogue: accumulators -> LDS -> fused epilogue -> stores), median / max
  span     last exit - first entry
    python tools/timeline_c2.py [--config c2|c5] [--compute bf16]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from f5_tts_amd import parallel, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--compute", default="bf16")
    args = ap.parse_args()
    device = torch.device("cuda", 0)
    case = {"c2": synthetic.c2_case, "c5": synthetic.c5_case, "c3": synthetic.c3_case}[args.config]()
    model, arch = bench.build_model(case["preset"], args.compute, device)
    utts = bench.build_job(case, 1)
    for u in utts:
        u["cond"], u["text"] = u["cond"].to(device), u["text"].to(device)
    plan_all = parallel.plan([u["total"] for u in utts], 1, max_batch=case["B"])

    def sample(cond, text, dur, lens):
        return model.sample(cond=cond, text=text, duration=dur, lens=lens, steps=case["nfe"], cfg_strength=case["cfg"],
                            sway_sampling_coef=case["sway"], seed=0, keep_trajectory=False)[0]

    def step():
        return parallel.run_sharded(utts, sample, rank=0, world=1, device=device, plan_all=plan_all)

    eng = model.transformer.get_engine(model.engine_compute(), device)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    print(f"{args.config} {args.compute}: per-workgroup timeline of each class's first launch (us)")
    print(f"{'class':10s} {'WGs':>5s} {'spread':>7s} {'ramp med/max':>14s} {'loop med/max':>14s} "
          f"{'epi med/max':>14s} {'span':>7s}")
    for kc in ("qkv", "attention", "out", "ffn1", "ffn2"):
        eng.probe(kc)
        step()
        torch.cuda.synchronize()
        t = eng.probe_timeline()
        eng.probe(None)
        if len(t) == 0:
            print(f"{kc:10s} no timeline")
            continue
        ok = ~np.isnan(t).any(axis=1)
        t = t[ok]
        ramp, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
        print(f"{kc:10s} {len(t):5d} {t[:, 0].max():7.2f} {np.median(ramp):6.2f}/{ramp.max():6.2f} "
              f"{np.median(loop):6.2f}/{loop.max():6.2f} {np.median(epi):6.2f}/{epi.max():6.2f} {t[:, 3].max():7.2f}",
              flush=True)
        np.save(os.path.join(REPO, "gpurun_out", f"timeline_{args.config}_{kc}.npy"), t)


if __name__ == "__main__":
    main()
