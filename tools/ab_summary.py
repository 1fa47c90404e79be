#!/usr/bin/env python3
"""Summarise tools/ab_ops.sh: total and per-kind forward time (mean over rounds) of the baseline
library against the in-tree one, and the ops that moved most.  usage: ab_summary.py <dir>"""
import glob
import json
import os
import sys


def load(pattern):
    runs = [json.load(open(f)) for f in sorted(glob.glob(pattern))]
    return runs


def main():
    d = sys.argv[1]
    arms = {a: load(os.path.join(d, a + "_*.json")) for a in ("base", "new")}
    if not all(arms.values()):
        print("missing runs")
        return
    print("# Same-box A/B, %s\n" % os.path.basename(d.rstrip("/")))
    print("| arm | totals (us) | mean |")
    print("|---|---|---:|")
    for a, runs in arms.items():
        t = [r["total_us"] for r in runs]
        print("| %s | %s | %.1f |" % (a, " / ".join("%.1f" % x for x in t), sum(t) / len(t)))
    kinds = sorted({o["kind"] for r in arms["base"] for o in r["ops"]})
    print("\n| kind | base us | new us | delta |")
    print("|---|---:|---:|---:|")
    for k in kinds:
        m = {a: sum(sum(o["us"] for o in r["ops"] if o["kind"] == k) for r in runs) / len(runs) for a, runs in arms.items()}
        print("| %s | %.1f | %.1f | %+.1f |" % (k, m["base"], m["new"], m["new"] - m["base"]))
    n = len(arms["base"][0]["ops"])
    rows = []
    for i in range(n):
        b = sum(r["ops"][i]["us"] for r in arms["base"]) / len(arms["base"])
        w = sum(r["ops"][i]["us"] for r in arms["new"]) / len(arms["new"])
        rows.append((w - b, i, arms["base"][0]["ops"][i]["name"][:48], b, w))
    rows.sort()
    print("\n| op | name | base | new | delta |")
    print("|---:|---|---:|---:|---:|")
    for delta, i, name, b, w in rows[:8] + rows[-5:]:
        print("| %d | %s | %.1f | %.1f | %+.1f |" % (i, name, b, w, delta))


if __name__ == "__main__":
    main()
