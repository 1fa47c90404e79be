#!/usr/bin/env python3
"""Streaming-attention variants (kernels.h set_attention_variant: 0 default, 1 K/V two tiles ahead,
2 without the XCD-aware pair mapping) on ViT-B/16's attention: packed
QKV rows [B * 197, 3 * 768] as the fused QKV GEMM writes them, 12 heads of 64, fp32 split mode and
bf16; each a captured hipGraph of 20 launches, median of 5 trials; outputs checked against the
default variant (bitwise) and against torch float64.

  python tools/attn_bench.py [--batch 32] [--seq 197] [--md out.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=197)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    import die_amd  # noqa: F401
    from die_amd import native
    from die_amd.ops import kernels as K

    B, S, H, D = a.batch, a.seq, a.heads, 64
    C = H * D
    qkv = torch.randn(B, S, 3 * C, device="cuda")
    q, k, v = (qkv[..., i * C:(i + 1) * C].double().reshape(B, S, H, D).transpose(1, 2) for i in range(3))
    ref = torch.softmax(q @ k.transpose(-1, -2) / np.sqrt(D), -1) @ v
    ref = ref.transpose(1, 2).reshape(B, S, C)
    L = native.kernels()
    lines = ["# Streaming attention variants, B=%d S=%d H=%d D=64 (MI355X)" % (B, S, H), "",
             "| mode | variant | us | rel err vs fp64 | bitwise = variant 0 |", "|---|---:|---:|---:|---|"]
    for split in (True, False):
        if split:
            src = K.split_planes(qkv)  # [2, B, S, 3C] bf16
            out = torch.empty((2, B, S, C), dtype=torch.bfloat16, device="cuda")
        else:
            src = qkv.to(torch.bfloat16).contiguous()
            out = torch.empty((B, S, C), dtype=torch.bfloat16, device="cuda")
        base = src.data_ptr()

        def launch():
            rc = L.die_kern_attention(base, base + 2 * C, base + 4 * C, out.data_ptr(), B, S, H, D, 3 * C, 3 * C,
                                      3 * C, C, float(1 / np.sqrt(D)), torch.cuda.current_stream().cuda_stream,
                                      int(split))
            assert rc == 0, rc

        first = None
        for var in (0, 1, 2):
            K.set_attention_variant(var)
            launch()
            torch.cuda.synchronize()
            res = (K.join_planes(out) if split else out.float()).clone()
            err = float((res.double() - ref).norm() / ref.norm())
            same = "-" if first is None else str(bool(torch.equal(res, first)))
            if first is None:
                first = res
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    launch()
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000 / 20)
            lines.append("| %s | %d | %.2f | %.1e | %s |" % ("fp32 split" if split else "bf16", var,
                                                              statistics.median(ts), err, same))
            print(lines[-1], flush=True)
        K.set_attention_variant(0)
    if a.md:
        open(a.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
