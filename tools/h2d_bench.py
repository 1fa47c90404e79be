#!/usr/bin/env python3
"""Host->device copy throughput for request-sized pinned buffers (1 MiB, the ResNet JSON text):
back-to-back on one stream, with an event after each copy, round-robin over several streams, and
one large copy.  Decides how the engine stages request inputs."""
import time

import torch


def main():
    n, sz = 64, 1 << 20
    src = [torch.empty(sz, dtype=torch.uint8).pin_memory() for _ in range(n)]
    dst = torch.empty(n * sz, dtype=torch.uint8, device="cuda")
    big = torch.empty(n * sz, dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream() for _ in range(4)]
    evs = [torch.cuda.Event() for _ in range(n)]

    def run(nstreams, events):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            s = streams[i % nstreams]
            with torch.cuda.stream(s):
                dst[i * sz:(i + 1) * sz].copy_(src[i], non_blocking=True)
                if events:
                    evs[i].record(s)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        return n * sz / t / 1e9, t_issue / n * 1e6

    for _ in range(2):
        run(1, False)
    for label, ns, ev in [("1 stream", 1, False), ("1 stream + event/copy", 1, True), ("2 streams", 2, False),
                          ("2 streams + event/copy", 2, True), ("4 streams", 4, False)]:
        r = [run(ns, ev) for _ in range(5)]
        gbs = sorted(x[0] for x in r)[2]
        us = sorted(x[1] for x in r)[2]
        print("%-24s %6.1f GB/s  issue %.1f us/copy" % (label, gbs, us), flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(big, non_blocking=True)
    torch.cuda.synchronize()
    print("%-24s %6.1f GB/s" % ("one 64 MiB copy", 5 * n * sz / (time.perf_counter() - t0) / 1e9))


if __name__ == "__main__":
    main()
