"""Where the phase-chain launch (chain.hip) spends its time at C2: the per-workgroup timeline of one chain launch
(entry, rows acquired, results stored, exit), per phase: blocks, first / median / last entry, median wait from
entry to acquired rows, median compute (acquired -> stored), last exit; times in us from the launch's first entry.
Phase block ranges follow chain_launch (chain.hip) for the C2 shape (M = 2 x 1876, d 1024, ff 2048, QKV 3072).

    python tools/chain_timeline.py [--config c2]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from f5_tts_amd import parallel, synthetic  # noqa: E402


def phase_starts(M, d=1024, ff=2048, nq=3072, qkv=True, ln_rows=32):
    cd = lambda a, b: (a + b - 1) // b
    r8 = lambda n: (n + 7) // 8 * 8
    cnt = [cd(M, 64) * (d // 128), cd(M, ln_rows), cd(M, 128) * (ff // 128), cd(M, 64) * (d // 128), cd(M, ln_rows),
           cd(M, 192) * (nq // 128) if qkv else 0]
    st = [0]
    for c in cnt:
        st.append(st[-1] + r8(c))
    return st, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    device = torch.device("cuda", 0)
    case = {"c2": synthetic.c2_case}[args.config]()
    model, arch = bench.build_model(case["preset"], "bf16", device)
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
    eng.probe("chain")
    step()
    torch.cuda.synchronize()
    t = eng.probe_timeline()
    eng.probe(None)
    M = 2 * case["total"] if isinstance(case.get("total"), int) else 2 * 1876
    st, cnt = phase_starts(M)
    print(f"{args.config}: chain launch timeline, {len(t)} workgroups, M = {M} (us from the first entry)")
    names = ["out", "ln1", "ffn1", "ffn2", "ln2", "qkv"]
    t0 = np.nanmin(t[:, 0])
    print(f"{'phase':6s} {'WGs':>5s} {'entry first/med/last':>22s} {'wait med/max':>14s} {'compute med/max':>16s} "
          f"{'exit last':>9s}")
    for p, nm in enumerate(names):
        rows = t[st[p]:st[p] + cnt[p]]
        rows = rows[~np.isnan(rows[:, 0]) & (rows[:, 3] > 0)]
        if len(rows) == 0:
            continue
        e = rows[:, 0] - t0
        acq = np.where(rows[:, 1] > 0, rows[:, 1], rows[:, 0])
        sto = np.where(rows[:, 2] > 0, rows[:, 2], rows[:, 3])
        wait, comp = acq - rows[:, 0], sto - acq
        print(f"{nm:6s} {len(rows):5d} {e.min():6.1f}/{np.median(e):6.1f}/{e.max():6.1f}   {np.median(wait):6.2f}/"
              f"{wait.max():6.2f} {np.median(comp):7.2f}/{comp.max():7.2f} {(rows[:, 3] - t0).max():9.1f}", flush=True)
    np.save(os.path.join(REPO, "gpurun_out", f"chain_timeline_{args.config}.npy"), t)


if __name__ == "__main__":
    main()
