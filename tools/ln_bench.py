#!/usr/bin/env python3
"""LayerNorm kernel variants (kernels/transformer.hip layernorm_rows `variant`) on ViT-B/16 rows:
[B * 197, 768], split (fp32 mode) and bf16, each a captured hipGraph of 20 launches, median of 5;
checked against torch (float64) first.

  python tools/ln_bench.py [--batch 32] [--md out.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    import torch

    import die_amd  # noqa: F401
    from die_amd.ops import kernels as K

    rows = a.batch * 197
    x = torch.randn(rows, a.C, device="cuda") * 2 + 0.5
    g = torch.rand(a.C, device="cuda") + 0.5
    b = torch.randn(a.C, device="cuda") * 0.1
    ref = torch.nn.functional.layer_norm(x.double(), (a.C,), g.double(), b.double(), 1e-5)
    lines = ["# LayerNorm variants, %d rows x %d (MI355X)" % (rows, a.C), "",
             "| mode | variant | us | GB/s | rel err |", "|---|---:|---:|---:|---:|"]
    for split in (True, False):
        xin = x if split else x.to(torch.bfloat16)
        for v in (0, 1, 2):
            out = K.layernorm(xin, g, b, split=split, variant=v)
            err = float((out.double() - ref).norm() / ref.norm())
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(20):
                    K.layernorm(xin, g, b, split=split, variant=v)
            gr.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gr.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000 / 20)
            us = statistics.median(ts)
            nbytes = rows * a.C * 2 * (2 if split else 1) * 2
            lines.append("| %s | %d | %.2f | %.0f | %.1e |" % ("fp32 split" if split else "bf16", v, us, nbytes / us / 1e3, err))
            print(lines[-1], flush=True)
    if a.md:
        open(a.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
