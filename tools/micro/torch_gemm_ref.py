#!/usr/bin/env python3
"""Vendor-library reference for the ResNet50 1x1-conv GEMM shapes: torch.matmul (hipBLASLt) in bf16
and fp32 on the same M x N x K problems the engine's split-fp32 kernels run (tools/micro/gemm_probe*).
Prints a markdown table of us per GEMM (median of hipGraph-free back-to-back launches)."""
import torch

SHAPES = [("s1.reduce", 100352, 64, 256), ("s2.reduce", 25088, 128, 512), ("s3.reduce", 6272, 256, 1024),
          ("s3.expand", 6272, 1024, 256), ("s4.reduce", 1568, 512, 2048), ("s4.expand", 1568, 2048, 512),
          ("s3.reduce.b16", 3136, 256, 1024)]


def bench(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    print("| shape | M | N | K | bf16 us | bf16 TFLOP/s | fp32 us | fp32 TFLOP/s | 3 x bf16 (split-equivalent) us |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, M, N, K in SHAPES:
        out = []
        for dt in (torch.bfloat16, torch.float32):
            x = torch.randn(M, K, device="cuda", dtype=dt)
            w = torch.randn(K, N, device="cuda", dtype=dt)
            o = torch.empty(M, N, device="cuda", dtype=dt)
            us = bench(lambda: torch.matmul(x, w, out=o))
            out.append((us, 2.0 * M * N * K / us * 1e-6))
        print("| %s | %d | %d | %d | %.1f | %.0f | %.1f | %.0f | %.1f |" % (name, M, N, K, out[0][0], out[0][1], out[1][0],
                                                                           out[1][1], 3 * out[0][0]))


if __name__ == "__main__":
    main()
