#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown.

    python tools/prof_summary.py gpurun_out/r1_prof/prof [--model model.onnx --batch 32] > profiles/x.md

With --model, the last complete forward in the trace is mapped op-by-op onto the engine plan
(`die_plan_summary`), giving per-layer time, TFLOP/s and the fused epilogue of each conv.
"""
import argparse
import csv
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="path prefix of the CSVs, e.g. gpurun_out/r1_prof/prof")
    ap.add_argument("--model", default="")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    stats = list(csv.DictReader(open(a.prefix + "_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in stats)
    print("# %s\n" % a.title)
    print("Source: `%s_kernel_stats.csv` (rocprofv3 --kernel-trace --stats).\n" % os.path.basename(a.prefix))
    print("| kernel | calls | total us | avg us | share |\n|---|---:|---:|---:|---:|")
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"])):
        print("| `%s` | %s | %.1f | %.1f | %.1f%% |" % (r["Name"][:110].replace("|", "/"), r["Calls"],
                                                       float(r["TotalDurationNs"]) / 1e3,
                                                       float(r["AverageNs"]) / 1e3,
                                                       100 * float(r["TotalDurationNs"]) / tot))
    print("\nTotal kernel time: %.3f ms\n" % (tot / 1e6))
    if not a.model:
        return
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import die_amd  # noqa: F401
    from die_amd import native

    plan = native.plan_summary(a.model, a.batch)
    ops = plan["ops"]
    trace = list(csv.DictReader(open(a.prefix + "_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = ops[0]["kind"]
    starts = [i for i, r in enumerate(trace) if first in r["Kernel_Name"]]
    fw = None
    for s in reversed(starts):
        # group helper kernels (split-K reduce) with the op that launched them
        grp, i = [], s
        while i < len(trace) and len(grp) < len(ops):
            g = [trace[i]]
            i += 1
            while i < len(trace) and "splitk_epilogue" in trace[i]["Kernel_Name"]:
                g.append(trace[i])
                i += 1
            grp.append(g)
        if len(grp) == len(ops):
            fw = grp
            break
    if fw is None:
        return
    t0 = int(fw[0][0]["Start_Timestamp"])
    t1 = int(fw[-1][-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for g in fw for r in g)
    print("## One forward (batch %d), op by op\n" % a.batch)
    print("Span %.1f us, kernel busy %.1f us (%.0f%%), %d kernels; %s\n" % ((t1 - t0) / 1e3, busy / 1e3,
                                                                          100 * busy / max(1, t1 - t0), len(fw),
                                                                          plan["summary"]))
    print("| # | op | kernel | us | GFLOP | TFLOP/s | N | K | KxK/s | epilogue |\n|---:|---|---|---:|---:|---:|---:|---:|---|---|")
    for i, (g, op) in enumerate(zip(fw, ops)):
        r = g[0]
        us = sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in g) / 1e3
        gf = op.get("gflop", 0.0) * a.batch
        epi = ""
        if op["kind"] == "conv":
            epi = "+".join(k for k in ("relu", "residual", "dual_store") if op.get(k))
        print("| %d | %s | `%s`%s | %.1f | %.2f | %s | %s | %s | %s | %s |" % (
            i, op["name"][:40], r["Kernel_Name"].split("(")[0].replace("void ", "").replace("die::kern::(anonymous namespace)::", "")[-44:],
            " +splitK" if len(g) > 1 else "", us, gf,
            ("%.0f" % (gf / us * 1e3)) if gf else "", op.get("N", ""), op.get("K", ""),
            ("%sx%s/%s" % (op.get("KH"), op.get("KH"), op.get("stride"))) if op["kind"] == "conv" else "", epi))


if __name__ == "__main__":
    main()
