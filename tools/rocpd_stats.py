#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite results database (`rocprofv3 --kernel-trace
-d DIR -o NAME` writes DIR/NAME_results.db by default): calls, total/avg/min/max us and share of
kernel time, grouped by the demangled kernel name (template arguments kept, namespaces dropped).

  python tools/rocpd_stats.py gpurun_out/r2_31/prof/bench_results.db [--top 30] [--md out.md]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"die::kern::(igemm::)?(\(anonymous namespace\)::)?", "", name)
    n = n.replace("void ", "").split("(")[0] if "(" in n and "<" not in n.split("(")[0][-1:] else n
    n = re.sub(r"\(die::kern::ConvArgs.*$", "", n)
    return n.replace("conv_glds_kernel", "glds").replace("conv_igemm_kernel", "igemm")[:110]


SIDE = ("pk_count", "pk_parse", "copyBuffer", "fillBuffer", "copy_i64", "unpack", "decode")


def forwards(con, first, md):
    """A forward = the compute-stream kernels from one FIRST_KERNEL launch to the next (decode and
    copy kernels, which run on the copy stream under the previous forward, are left out).  span =
    first start -> last end; busy = summed kernel time; gap = span - busy (the compute stream idle
    inside the forward: launch/enqueue delays, not device work)."""
    rows = con.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                       "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    fw, cur = [], None
    for name, b, e in rows:
        if any(k in name for k in SIDE):
            continue
        if first in name:
            if cur:
                fw.append(cur)
            cur = [b, e, 0.0, 0, 0.0]
        if cur is None:
            continue
        cur[1] = max(cur[1], e)
        cur[2] += (e - b) / 1e3
        cur[3] += 1
    if cur:
        fw.append(cur)
    n = max((f[3] for f in fw), default=0)
    fw = [f for f in fw if f[3] == n]  # whole forwards only (autotune launches the first kernel alone)
    if not fw:
        return
    span = sorted((f[1] - f[0]) / 1e3 for f in fw)
    busy = sorted(f[2] for f in fw)
    gap = sorted((f[1] - f[0]) / 1e3 - f[2] for f in fw)
    med = lambda v: v[len(v) // 2]
    line = ("%d forwards of %d kernels: span us median %.1f mean %.1f; kernel-busy median %.1f mean %.1f; "
            "idle inside the forward median %.1f mean %.1f p90 %.1f" % (
                len(fw), n, med(span), sum(span) / len(span), med(busy), sum(busy) / len(busy), med(gap),
                sum(gap) / len(gap), gap[int(0.9 * (len(gap) - 1))]))
    print(line)
    if md:
        open(md + ".forwards.txt", "w").write(line + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", default="")
    ap.add_argument("--forwards", default="", metavar="FIRST_KERNEL",
                    help="also split the trace into forwards, each starting at a kernel whose name contains "
                         "FIRST_KERNEL, and report per-forward span, kernel-busy time and idle gaps")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    if a.forwards:
        forwards(con, a.forwards, a.md)
    rows = con.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                       "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    st = defaultdict(lambda: [0, 0.0, 1e30, 0.0])
    t0, t1 = min(r[1] for r in rows), max(r[2] for r in rows)
    for name, b, e in rows:
        us = (e - b) / 1e3
        s = st[short(name)]
        s[0] += 1
        s[1] += us
        s[2] = min(s[2], us)
        s[3] = max(s[3], us)
    total = sum(v[1] for v in st.values())
    lines = ["| kernel | calls | total us | avg us | min us | max us | share |", "|---|---:|---:|---:|---:|---:|---:|"]
    for k, v in sorted(st.items(), key=lambda kv: -kv[1][1])[: a.top]:
        lines.append("| `%s` | %d | %.0f | %.2f | %.2f | %.2f | %.1f%% |" % (k, v[0], v[1], v[1] / v[0], v[2], v[3],
                                                                            100 * v[1] / total))
    head = ("%d dispatches, %.1f ms of kernel time over a %.1f ms trace window (GPU busy %.0f %%)."
            % (len(rows), total / 1e3, (t1 - t0) / 1e6, 100 * total * 1e3 / max(t1 - t0, 1)))
    text = head + "\n\n" + "\n".join(lines)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
