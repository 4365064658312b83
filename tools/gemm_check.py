"""Check GEMM tile configurations on the GPU: every config against fp64 and bit for bit against cfg 0.

python tools/gemm_check.py 50,51,52   (configs; default: the ones gemm_tune.py times)
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "f5-tts_amd"))


def main():
    import torch
    from f5_tts_amd.engine import gemm_force_config, op_linear

    cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 5]
    shapes = [(3752, 1024, 1024), (3752, 2048, 1024), (3752, 3072, 1024), (3752, 1024, 2048), (517, 1024, 1024),
              (130, 512, 64)]
    bad = 0
    for M, N, K in shapes:
        g = torch.Generator(device="cpu").manual_seed(M + N + K)
        A = torch.randn(M, K, generator=g).cuda()
        W = (torch.randn(N, K, generator=g) / K ** 0.5).cuda()
        b = torch.randn(N, generator=g).cuda()
        ref = A.double() @ W.double().t() + b.double()
        gemm_force_config(0)
        base = op_linear(A, W, b)
        for c in cfgs:
            gemm_force_config(c)
            C = op_linear(A, W, b)
            torch.cuda.synchronize()
            err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
            same = torch.equal(C, base)
            ok = err < 2e-2 and same
            bad += not ok
            print(f"M={M} N={N} K={K} cfg={c}: err={err:.2e} bitwise={'yes' if same else 'NO'} {'ok' if ok else 'FAIL'}",
                  flush=True)
    gemm_force_config(-1)
    print("ALL OK" if not bad else f"{bad} FAILED")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
