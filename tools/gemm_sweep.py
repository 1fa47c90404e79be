#!/usr/bin/env python3
"""Time given launch configs of the implicit-GEMM kernel on ViT-B/16-shaped GEMMs (fp32 split mode
by default), each as a captured hipGraph of back-to-back launches; hipBLASLt bf16 / fp32 on the same
GEMM view for reference (profiles/r4_gemm_sweep_vit_*.md).

  python tools/gemm_sweep.py --batch 32 --cfgs 0,4,20,21,22 [--md out.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # name, K (Cin), N (Cout), epilogue
    ("qkv", 768, 2304, "plain"),
    ("attn_out", 768, 768, "res"),
    ("mlp1", 768, 3072, "gelu"),
    ("mlp2", 3072, 768, "res"),
    ("fc", 2048, 1000, "plain"),  # a classifier head (ResNet50: --tokens 1 --batch <serving batch>)
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--tokens", type=int, default=197)
    ap.add_argument("--cfgs", default="0,4,20,21,22")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--bf16", action="store_true", help="bf16 operands instead of split fp32")
    ap.add_argument("--md", default="")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
    ap.add_argument("--order", type=int, default=0, help="ConvArgs::order (XCD tile order)")
    ap.add_argument("--no-blas", action="store_true", help="skip the hipBLASLt reference columns")
    ap.add_argument("--probe", type=int, default=0,
                    help="ConvArgs::probe: 1 = MFMAs without operand DMA, 2 = DMA without MFMAs (LDS-DMA kernels)")
    a = ap.parse_args()
    import torch

    import die_amd  # noqa: F401
    from die_amd.ops import kernels as K

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.trials):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0 / a.reps)
        return statistics.median(ts)

    # "cfg" or "cfg:splits" (fused split-K)
    cfgs = [tuple(int(v) for v in (c.split(":") + ["1"])[:2]) for c in a.cfgs.split(",")]
    split = not a.bf16
    M = a.batch * a.tokens
    lines = ["# GEMM config sweep, ViT-B/16 shapes, M = %d rows (%s)" % (M, "fp32 split" if split else "bf16"), "",
             "| shape | K | N | " + " | ".join("cfg %d" % c if s == 1 else "cfg %d/%d" % (c, s) for c, s in cfgs) +
             " | hipBLASLt bf16 | hipBLASLt fp32 |",
             "|---|---:|---:|" + "---:|" * (len(cfgs) + 2)]
    for name, Kd, N, epi in SHAPES:
        if a.shapes and name not in a.shapes.split(","):
            continue
        x = torch.randn(a.batch, a.tokens, 1, Kd, device="cuda")
        if not split:
            x = x.to(torch.bfloat16)
        w = torch.randn(N, Kd, 1, 1, device="cuda") / Kd ** 0.5
        kw = dict(bias=torch.randn(N, device="cuda") * 0.1)
        if epi == "res":
            kw["res"] = torch.randn(a.batch, a.tokens, 1, N, device="cuda")
            if not split:
                kw["res"] = kw["res"].to(torch.bfloat16)
        pr = K.ConvProblem(x, w, relu=(epi == "gelu"), split=split, max_splits=max(s for _, s in cfgs), **kw)
        row = []
        for c, sp in cfgs:
            ex = {"probe": a.probe} if a.probe else None
            rc = pr.launch(c, sp, order=a.order, extra=ex)
            row.append("n/a" if rc == 1 else "%.1f" % timed(lambda: pr.launch(c, sp, order=a.order, extra=ex)))
        tb = tf = float("nan")
        if not a.no_blas:
            A_ = torch.randn(M, Kd, device="cuda")
            W_ = torch.randn(Kd, N, device="cuda")
            ab, wb = A_.to(torch.bfloat16), W_.to(torch.bfloat16)
            tb = timed(lambda: torch.matmul(ab, wb))
            torch.backends.cuda.matmul.allow_tf32 = False
            tf = timed(lambda: torch.matmul(A_, W_))
        lines.append("| %s | %d | %d | %s | %.1f | %.1f |" % (name, Kd, N, " | ".join(row), tb, tf))
        print(lines[-1], flush=True)
    if a.md:
        open(a.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
