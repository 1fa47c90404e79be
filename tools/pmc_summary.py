#!/usr/bin/env python3
"""Join rocprofv3 --pmc passes (tools/gpu_r10.sh layout: <dir>/p1..p4/p_counter_collection.csv) into a
per-kernel table for the LAST forward pass of tools/pmc_forward.py.

Derived metrics (gfx950: 256 CUs, 1024 SIMDs; formulas from `rocprofv3 -L`):
  GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (~21k cycles/us); it is divided by 8 first,
  matching the derived formulas' reduce(GRBM_GUI_ACTIVE, max).
  MfmaUtil %  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 1024) * 100
                (a 16x16x32 bf16 MFMA = 16 busy cycles; 100 % = 2.5 PFLOP/s dense bf16)
  Occupancy % = 400 * SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE / 256 / 32
  HBM GB/s    = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B / kernel time   (FETCH_SIZE counts half the bytes
                of wide coalesced reads on gfx950 -> doubled; an estimate, Infinity-Cache hits included)
  L2 hit %    = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  LDS conf    = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (conflict cycles per LDS instruction)
  park/stall/issue % = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over their sum (wave parked
                on s_waitcnt or a barrier / issue-stalled / issuing; disjoint, ~= SQ_WAVE_CYCLES)
  LDS-issue % = SQ_WAIT_INST_LDS over the same sum (a sub-bucket of the stall share)
usage: pmc_summary.py gpurun_out/r10/resnet50 [--title T]
"""
import argparse
import csv
import os
import re
from collections import OrderedDict, defaultdict

SIMDS, CUS, XCDS = 1024, 256, 8  # GRBM_GUI_ACTIVE comes back summed over the 8 XCDs' GRBMs


def load(pass_dir):
    path = os.path.join(pass_dir, "p_counter_collection.csv")
    rows = list(csv.DictReader(open(path)))
    disp = OrderedDict()
    for r in rows:
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "t0": int(r["Start_Timestamp"]),
                                                     "t1": int(r["End_Timestamp"]), "c": defaultdict(float),
                                                     "grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                                                     "agpr": int(r["Accum_VGPR_Count"]), "lds": int(r["LDS_Block_Size"])})
        d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    seq = [v for _, v in sorted(disp.items()) if "die::kern" in v["name"]]
    # the forward starts at its input pass: input_prep, or the stem that fused it
    start = max(i for i, v in enumerate(seq) if "input_prep" in v["name"] or "stem7x7_nchw" in v["name"] or "stem_pool_nchw" in v["name"])
    return seq[start:]


def short(name):
    n = name.replace("die::kern::igemm::(anonymous namespace)::", "").replace("die::kern::(anonymous namespace)::", "")
    n = n.replace("void ", "")
    n = n.split("(")[0]
    return n.replace("conv_igemm_kernel", "igemm").replace("conv_glds_kernel", "glds")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--title", default="")
    ap.add_argument("--note", default="heuristic kernel configs, no graphs")
    a = ap.parse_args()
    passes = [load(os.path.join(a.dir, p)) for p in ("p1", "p2", "p3", "p4") if os.path.isdir(os.path.join(a.dir, p))]
    n = min(len(p) for p in passes)
    lines = ["# rocprofv3 PMC counters: %s" % (a.title or os.path.basename(a.dir.rstrip("/"))), "",
             "One eager forward%s (%s), counters from 4 separate" % (
                 (" at batch " + re.search(r"B=(\d+)", a.title).group(1)) if re.search(r"B=(\d+)", a.title) else "",
                 a.note),
             "`rocprofv3 --kernel-trace --pmc` passes joined by dispatch order. Derived formulas: see tools/pmc_summary.py.",
             "", "| # | kernel | grid | VGPR/AGPR | LDS B | us | MfmaUtil % | Occ % | HBM GB/s (est) | L2 hit % | LDS conf/instr | park/stall/issue % | LDS-issue % |",
             "|---:|---|---:|---|---:|---:|---:|---:|---:|---:|---:|---|---:|"]
    tot = defaultdict(float)
    for i in range(n):
        k = {}
        for p in passes:
            k.update(p[i]["c"])
        d = passes[0][i]
        us = (d["t1"] - d["t0"]) / 1e3
        gui = (k.get("GRBM_GUI_ACTIVE", 0) / XCDS) or 1  # the derived formulas use the per-XCD (max) value
        mfma = 100 * k.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * SIMDS)
        occ = 400 * k.get("SQ_WAVE_CYCLES", 0) / gui / CUS / 32
        us2 = (passes[1][i]["t1"] - passes[1][i]["t0"]) / 1e3 if len(passes) > 1 else us
        us3 = (passes[2][i]["t1"] - passes[2][i]["t0"]) / 1e3 if len(passes) > 2 else us
        rd = 2 * k.get("FETCH_SIZE", 0) * 1024
        wr = k.get("WRITE_SIZE", 0) * 1024
        gbs = (rd / max(us2, 1e-3) + wr / max(us3, 1e-3)) / 1e3
        hit, miss = k.get("TCC_HIT_sum", 0), k.get("TCC_MISS_sum", 0)
        l2 = 100 * hit / (hit + miss) if hit + miss else 0
        ldsc = k.get("SQ_LDS_BANK_CONFLICT", 0) / max(k.get("SQ_INSTS_LDS", 0), 1)
        wa, wi, ac = k.get("SQ_WAIT_ANY", 0), k.get("SQ_WAIT_INST_ANY", 0), k.get("SQ_ACTIVE_INST_ANY", 0)
        ws = max(wa + wi + ac, 1)
        lines.append("| %d | `%s` | %d | %d/%d | %d | %.1f | %.1f | %.0f | %.0f | %.0f | %.2f | %.0f/%.0f/%.0f | %.0f |" % (
            i, short(d["name"]), d["grid"], d["vgpr"], d["agpr"], d["lds"], us, mfma, occ, gbs, l2, ldsc,
            100 * wa / ws, 100 * wi / ws, 100 * ac / ws, 100 * k.get("SQ_WAIT_INST_LDS", 0) / ws))
        tot["us"] += us
        tot["mfma_cyc"] += k.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        tot["gui"] += gui
        tot["bytes"] += rd + wr
    lines += ["", "Whole forward: %.1f us of kernels, MfmaUtil %.1f %% (cycle-weighted), ~%.2f GB moved (%.0f GB/s avg)." % (
        tot["us"], 100 * tot["mfma_cyc"] / (tot["gui"] * SIMDS), tot["bytes"] / 1e9, tot["bytes"] / max(tot["us"], 1) / 1e3)]
    print("\n".join(lines))


if __name__ == "__main__":
    main()
