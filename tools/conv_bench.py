#!/usr/bin/env python3
"""Sweep every (launch config, split-K, fused reduction) of the implicit-GEMM conv kernel over the
unique ResNet50-v2 conv shapes at one batch size and report the best per shape.

Each candidate is timed as a captured hipGraph of `--reps` back-to-back launches (no host launch
gaps), replayed `--trials` times; the median replay / reps is the per-launch time.  The epilogue of
each shape matches the engine's fusion (1x1 reduce / 3x3: bias+ReLU; expand: +residual and the dual
store of the next unit's BN+ReLU; projection: plain).

  python tools/conv_bench.py --batch 16 [--json out.json] [--md out.md]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, count in the network, Cin, Cout, k, stride, H_in, epilogue)
def resnet50_shapes():
    out = []
    widths = [64, 128, 256, 512]
    units = [3, 4, 6, 3]
    H = 56
    cin = 64
    for s, (w, n) in enumerate(zip(widths, units)):
        st = 1 if s == 0 else 2
        Ho = H // st
        o = 4 * w
        out.append(("s%d.u0.reduce" % (s + 1), 1, cin, w, 1, 1, H, "relu"))
        out.append(("s%d.u0.3x3" % (s + 1), 1, w, w, 3, st, H, "relu"))
        out.append(("s%d.u0.expand" % (s + 1), 1, w, o, 1, 1, Ho, "res_dual"))
        out.append(("s%d.u0.proj" % (s + 1), 1, cin, o, 1, st, H, "plain"))
        if n > 1:
            out.append(("s%d.reduce" % (s + 1), n - 1, o, w, 1, 1, Ho, "relu"))
            out.append(("s%d.3x3" % (s + 1), n - 1, w, w, 3, 1, Ho, "relu"))
            out.append(("s%d.expand" % (s + 1), n - 1, w, o, 1, 1, Ho, "res_dual"))
        cin = o
        H = Ho
    out.append(("fc", 1, 2048, 1000, 1, 1, 1, "f32"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--only", default="", help="substring filter on the shape name")
    ap.add_argument("--ref", action="store_true", help="also time torch.matmul (hipBLASLt) on the GEMM view "
                    "and F.conv2d (MIOpen, channels_last) for calibration")
    ap.add_argument("--split", action="store_true", help="fp32 mode: split (hi, lo) planes, 3 MFMAs per pair")
    ap.add_argument("--cold", action="store_true", help="time each launch alone behind a 96 MB L2 scrub "
                    "(eager, events around the conv only): operands come from the Infinity Cache, as inside a forward")
    ap.add_argument("--cfgs", default="", help="comma list of launch configs to try (default: all)")
    ap.add_argument("--splits", default="1,2,4,8,16", help="comma list of split-K factors")
    ap.add_argument("--sk", default="", help="comma list of stream-K block counts to try too (ConvArgs::sk)")
    ap.add_argument("--probe", type=int, default=0, help="ConvArgs::probe: 1 = no operand DMA, 2 = no MFMAs (outputs garbage)")
    ap.add_argument("--dump", action="store_true", help="print every candidate's time (with --only)")
    ap.add_argument("--json", default="")
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    import torch

    import die_amd  # noqa: F401
    from die_amd.ops import kernels as K

    torch.manual_seed(0)
    dev = "cuda"
    scrub = torch.ones(24 << 20, device=dev) if a.cold else None  # 96 MB
    results = []
    for name, count, cin, cout, k, stride, H, epi in resnet50_shapes():
        if a.only and a.only not in name:
            continue
        B = a.batch
        x = (torch.randn(B, H, H, cin, device=dev) * 0.5).to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5
        bias = torch.randn(cout, device=dev) * 0.1
        Ho = (H + 2 * (k // 2) - k) // stride + 1
        kw = dict(bias=bias, stride=stride, pad=k // 2)
        if epi == "relu":
            kw["relu"] = True
        elif epi == "res_dual":
            kw.update(res=torch.randn(B, Ho, Ho, cout, device=dev).to(torch.bfloat16),
                      scale2=torch.rand(cout, device=dev) + 0.5, shift2=torch.randn(cout, device=dev) * 0.1,
                      relu2=True)
        elif epi == "f32":
            kw["out_f32"] = True
        pr = K.ConvProblem(x, w, max_splits=16, split=a.split, **kw)
        nk = (cin * k * k + 63) // 64
        cands = []
        cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else range(K.NUM_CFGS)
        for cfg in cfgs:
            sks = [int(v) for v in a.sk.split(",")] if a.sk else []
            for sp in [int(v) for v in a.splits.split(",")] + [-v for v in sks]:
                if sp > nk or (sp > 1 and cout % 8):
                    continue
                for fused, order in [(f, o) for f in ((False, True) if sp > 1 else (False,)) for o in (1, 2)]:
                    rc = pr.launch(cfg, max(sp, 1), fused, order, sk=max(0, -sp), extra={"probe": a.probe} if a.probe else None)
                    if rc == 1:
                        continue
                    if rc != 0:
                        raise RuntimeError("launch failed %d" % rc)
                    torch.cuda.synchronize()
                    ts = []
                    if a.cold:
                        for _ in range(a.trials):
                            scrub.mul_(1.0001)
                            e0 = torch.cuda.Event(enable_timing=True)
                            e1 = torch.cuda.Event(enable_timing=True)
                            e0.record()
                            pr.launch(cfg, max(sp, 1), fused, order, sk=max(0, -sp), extra={"probe": a.probe} if a.probe else None)
                            e1.record()
                            e1.synchronize()
                            ts.append(e0.elapsed_time(e1) * 1000.0)
                        cands.append((statistics.median(ts), cfg, sp, fused, order))
                        continue
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for _ in range(a.reps):
                            pr.launch(cfg, max(sp, 1), fused, order, sk=max(0, -sp), extra={"probe": a.probe} if a.probe else None)
                    g.replay()
                    torch.cuda.synchronize()
                    for _ in range(a.trials):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        g.replay()
                        e1.record()
                        e1.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1000.0 / a.reps)
                    del g
                    cands.append((statistics.median(ts), cfg, sp, fused, order))
        cands.sort()
        if a.dump:
            for us, cfg, sp, fused, order in cands:
                print("  %-14s cfg %2d (v%d tile %d) %s%s order %d: %7.2f us" % (
                    name, cfg, cfg // 4, cfg % 4, "split %2d" % sp if sp > 0 else "sk %4d" % -sp,
                    "f" if fused else " ", order, us), flush=True)
        ref = {}
        if a.ref:
            def timed(fn):
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(a.reps):
                        fn()
                g.replay()
                torch.cuda.synchronize()
                ts = []
                for _ in range(a.trials):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1000.0 / a.reps)
                return statistics.median(ts)

            Mg = B * Ho * Ho
            A_ = torch.randn(Mg, cin * k * k, device=dev).to(torch.bfloat16)
            W_ = torch.randn(cin * k * k, cout, device=dev).to(torch.bfloat16)
            ref["matmul_us"] = timed(lambda: torch.matmul(A_, W_))
            xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wc = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            try:
                ref["conv2d_us"] = timed(lambda: torch.nn.functional.conv2d(xc, wc, None, stride, k // 2))
            except Exception as ex:  # MIOpen may refuse a shape
                ref["conv2d_error"] = str(ex)[:80]
        best = cands[0]
        by_variant = {}
        for us, cfg, sp, fused, order in cands:
            v = cfg // 4
            if v not in by_variant:
                by_variant[v] = (us, cfg, sp, fused)
        r = dict(name=name, count=count, M=B * Ho * Ho, N=cout, K=cin * k * k, us=best[0], cfg=best[1],
                 splits=best[2], fused=best[3], tflops=pr.flops / best[0] / 1e6, ref=ref,
                 best_per_variant={str(v): dict(us=t[0], cfg=t[1], splits=t[2], fused=t[3])
                                   for v, t in sorted(by_variant.items())},
                 top=[dict(us=round(t[0], 2), cfg=t[1], splits=t[2], fused=t[3], order=t[4]) for t in cands[:16]])
        results.append(r)
        print("%-14s x%d M=%-6d N=%-5d K=%-5d best %7.2f us (cfg %2d split %2d%s) %5.0f TF | per variant: %s" % (
            name, count, r["M"], cout, r["K"], best[0], best[1], best[2], "f" if best[3] else "", r["tflops"],
            " ".join("v%s=%.1f" % (v, t["us"]) for v, t in r["best_per_variant"].items())) +
            ("" if not ref else " | matmul %.1f conv2d %s" % (ref["matmul_us"], "%.1f" % ref["conv2d_us"]
                                                               if "conv2d_us" in ref else "n/a")), flush=True)
    total = sum(r["us"] * r["count"] for r in results)
    print("weighted conv total at batch %d: %.1f us" % (a.batch, total))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(batch=a.batch, total_us=total, shapes=results), f, indent=1)
    if a.md:
        lines = ["# conv kernel sweep, ResNet50-v2 shapes, batch %d (MI355X)" % a.batch, "",
                 ("fp32 split mode. " if a.split else "") +
                 "Best of %d configs x split-K {1..16} x {separate, fused} reduction; hipGraph of %d launches, "
                 "median of %d replays. Weighted total %.1f us." % (K.NUM_CFGS, a.reps, a.trials, total), "",
                 "| shape | x | M | N | K | best us | TFLOP/s | cfg/split | v0 | v1 (2st) | v2 (3st) | v3 (4st) | v4 (6st) | v5 (1st) | v6 (3x3 spatial) |",
                 "|---|---:|---:|---:|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|"]
        for r in results:
            pv = r["best_per_variant"]
            cells = ["%.1f" % pv[str(v)]["us"] if str(v) in pv else "-" for v in range(7)]
            lines.append("| %s | %d | %d | %d | %d | %.1f | %.0f | %d/%d%s | %s |" % (
                r["name"], r["count"], r["M"], r["N"], r["K"], r["us"], r["tflops"], r["cfg"], r["splits"],
                "f" if r["fused"] else "", " | ".join(cells)))
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
