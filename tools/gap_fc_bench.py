#!/usr/bin/env python3
"""Global pool + FC head kernel (kernels/misc.hip gap_fc_kernel) on ResNet50's head shape: x [B, 49,
2048] split planes, 1000 classes; each a captured hipGraph of 20 launches, median of 5 trials; the
phase-stop knob (set_gap_fc_stop) returns every block after the pooling (1), after the partial
logits (2), after the ticket (3) or runs the whole kernel (0), which splits the time by phase.
Checked against torch float64 first.

  python tools/gap_fc_bench.py [--batch 20] [--md out.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--hw", type=int, default=49)
    ap.add_argument("--C", type=int, default=2048)
    ap.add_argument("--N", type=int, default=1000)
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    import torch

    import die_amd  # noqa: F401
    from die_amd import native
    from die_amd.ops import kernels as K

    B, HW, C, N = a.batch, a.hw, a.C, a.N
    L = native.kernels()
    x = torch.randn(B, HW, C, device="cuda").relu()
    xs = K.split_planes(x)  # [2, B, HW, C]
    Npad, Kpad = (N + 127) // 128 * 128, C
    w = torch.zeros(Npad, Kpad, device="cuda")
    w[:N] = torch.randn(N, C, device="cuda") / C ** 0.5
    ws_ = K.split_planes(w)  # [2, Npad, Kpad]
    bias = torch.randn(N, device="cuda") * 0.1
    out = torch.zeros(B, N, device="cuda")
    wsbuf = torch.zeros(64 << 18, device="cuda")  # 64 MiB
    counters = torch.zeros(1 << 12, dtype=torch.int32, device="cuda")
    ref = x.double().mean(1) @ w[:N].double().T + bias.double()

    def launch():
        rc = L.die_kern_gap_fc(xs.data_ptr(), B, HW, C, 0, ws_.data_ptr(), Npad * Kpad, Kpad, bias.data_ptr(), N, 0,
                               out.data_ptr(), wsbuf.data_ptr(), wsbuf.numel() * 4, counters.data_ptr(),
                               counters.numel(), torch.cuda.current_stream().cuda_stream, 1)
        assert rc == 0, rc

    launch()
    torch.cuda.synchronize()
    err = float((out.double() - ref).norm() / ref.norm())
    lines = ["# gap_fc phases, B=%d HW=%d C=%d N=%d fp32 split (MI355X), rel err %.1e" % (B, HW, C, N, err), "",
             "| stop after | us |", "|---|---:|"]
    for stop, name in ((1, "pooling"), (2, "partial logits"), (3, "ticket"), (0, "whole kernel")):
        L.die_kern_set_gap_fc_stop(stop)
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
        lines.append("| %s | %.2f |" % (name, statistics.median(ts)))
        print(lines[-1], flush=True)
    L.die_kern_set_gap_fc_stop(0)
    # the ticket counters must be back at 0 after whole-kernel launches; stop 3 leaves them counting
    counters.zero_()
    launch()
    torch.cuda.synchronize()
    assert float((out.double() - ref).norm() / ref.norm()) < 1e-5
    if a.md:
        open(a.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
