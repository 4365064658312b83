"""Does the host run ahead of the device across back-to-back C2 calls? Times each call's return on the host
(no synchronisation) and the device span of the whole loop: if the host returns every ~call-length, something
in the call waits for the device.  python tools/diag_host_sync.py [calls]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from f5_tts_amd import parallel, synthetic  # noqa: E402


def main(n=8):
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    case = synthetic.c2_case()
    model, arch = bench.build_model(case["preset"], "bf16", device)
    utts = bench.build_job(case, 1)
    for u in utts:
        u["cond"], u["text"] = u["cond"].to(device), u["text"].to(device)
    plan_all = parallel.plan([u["total"] for u in utts], 1, max_batch=case["B"])

    def sample(cond, text, dur, lens):
        out, _ = model.sample(cond=cond, text=text, duration=dur, lens=lens, steps=case["nfe"], cfg_strength=case["cfg"],
                              sway_sampling_coef=case["sway"], seed=0, keep_trajectory=False)
        return out

    def step():
        return parallel.run_sharded(utts, sample, rank=0, world=1, device=device, plan_all=plan_all)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for label in ("plain", "no-seed"):
        if label == "no-seed":
            def sample(cond, text, dur, lens):  # noqa: F811
                out, _ = model.sample(cond=cond, text=text, duration=dur, lens=lens, steps=case["nfe"],
                                      cfg_strength=case["cfg"], sway_sampling_coef=case["sway"], keep_trajectory=False)
                return out
            step()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        rets = []
        for _ in range(n):
            step()
            rets.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) * 1e3
        print(label, "host returns (ms):", [round(r, 2) for r in rets], "all done:", round(tot, 2),
              "per call:", round(tot / n, 3), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
