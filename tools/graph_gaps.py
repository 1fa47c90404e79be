#!/usr/bin/env python3
"""Per-forward kernel busy time vs wall span from a rocprofv3 kernel trace.

    python tools/graph_gaps.py gpurun_out/x/prof_kernel_trace.csv [--first conv_stem] [--last N]

A forward is the sequence of kernels on the compute queue from one `--first` kernel (the stem conv)
to the kernel before the next one.  Reports, per forward: kernels, sum of kernel durations, span
(first start -> last end) and the idle gap = span - busy (launch/dependency bubbles inside the
hipGraph), plus the largest individual gaps by kernel pair.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="conv_stem")
    ap.add_argument("--last", type=int, default=50, help="analyse the last N forwards")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if a.first in k[2]]
    fwd = []
    for j, s in enumerate(starts[:-1]):
        seg = ks[s:starts[j + 1]]
        # stop at the forward's last kernel (the FC/GEMM before the next batch's decode kernels)
        fwd.append(seg)
    fwd = fwd[-a.last:]
    gaps = collections.Counter()
    tot_busy = tot_span = 0.0
    n_k = []
    for seg in fwd:
        # only the compute chain: drop kernels overlapping the next batch's PREP (decode/unpack/prep)
        seg = [k for k in seg if not any(t in k[2] for t in ("dec_", "unpack_text", "input_prep", "copy_i64"))]
        busy = sum(e - s for s, e, _ in seg) / 1e3
        span = (seg[-1][1] - seg[0][0]) / 1e3
        tot_busy += busy
        tot_span += span
        n_k.append(len(seg))
        for p, q in zip(seg, seg[1:]):
            g = (q[0] - p[1]) / 1e3
            if g > 0:
                gaps[(p[2][:60], q[2][:60])] += g
    n = max(len(fwd), 1)
    print("forwards analysed: %d, kernels per forward: %s" % (len(fwd), sorted(set(n_k))))
    print("avg busy %.1f us, avg span %.1f us, avg idle inside forward %.1f us (%.1f%%)"
          % (tot_busy / n, tot_span / n, (tot_span - tot_busy) / n, 100 * (tot_span - tot_busy) / max(tot_span, 1e-9)))
    print("largest gaps (avg us per forward):")
    for (p, q), g in gaps.most_common(12):
        print("  %6.2f  %s -> %s" % (g / n, p, q))


if __name__ == "__main__":
    main()
