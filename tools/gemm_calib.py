#!/usr/bin/env python3
"""hipBLASLt (torch.matmul, bf16) vs our MFMA GEMM (1x1-conv path, best config) on the ViT-B/16
GEMM shapes at batch 32 (M = 32 x 197 tokens).  Calibrates how far the conv/GEMM kernel is from the
vendor library on large GEMMs."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(torch, fn, reps=10, trials=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(trials):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0 / reps)
    return statistics.median(ts)


def main():
    import torch

    import die_amd  # noqa: F401
    from die_amd.ops import kernels as K

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    M = B * 197
    for name, Kd, N in [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768),
                        ("big4096", 4096, 4096)]:
        Mx = 4096 if name == "big4096" else M
        a = torch.randn(Mx, Kd, device="cuda").to(torch.bfloat16)
        b = torch.randn(Kd, N, device="cuda").to(torch.bfloat16)
        t_lib = timed(torch, lambda: torch.matmul(a, b))
        x = a.view(Mx, 1, 1, Kd)
        w = torch.randn(N, Kd, 1, 1, device="cuda") * 0.02
        pr = K.ConvProblem(x, w, max_splits=4)
        best = (1e9, None)
        for cfg in range(20):
            for sp in (1, 2, 4):
                if pr.launch(cfg, sp, True) != 0:
                    continue
                t = timed(torch, lambda: pr.launch(cfg, sp, True))
                best = min(best, (t, (cfg, sp)))
        fl = 2.0 * Mx * N * Kd
        print("%-8s M=%d N=%d K=%d  hipBLASLt %.1f us (%.0f TF)  ours %.1f us (%.0f TF) cfg %s" % (
            name, Mx, N, Kd, t_lib, fl / t_lib / 1e6, best[0], fl / best[0] / 1e6, best[1]), flush=True)


if __name__ == "__main__":
    main()
