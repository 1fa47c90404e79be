#!/usr/bin/env python3
"""Device time of the captured forward for every batch size 1..max_batch (each runs the graph of
the smallest bucket >= B): ms per batch and us per image, so the batch sizes whose tile grids
spill into another round of blocks (per-image cost steps) show up.  One JSON line per size and
a markdown table.  Usage: bucket_curve.py --arch resnet50 [--lo 12] [--hi 32] [--out PREFIX]"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", choices=["resnet50", "vit_b16"], default="resnet50")
    ap.add_argument("--lo", type=int, default=12)
    ap.add_argument("--hi", type=int, default=32)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--out", default="")
    ap.add_argument("--no-fuse-pairs", action="store_true", help="EngineOptions::fuse_pairs off")
    ap.add_argument("--tune-tail", action="store_true", help="EngineOptions::tune_tail on")
    ap.add_argument("--pair-shared-w", type=int, default=-2,
                    help="measurement: force PairArgs::shared_w for every pair launch (-1 auto, 0 never, 1 always)")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime)

    import die_amd  # noqa: F401
    from die_amd import native

    if a.arch == "vit_b16":
        from die_amd.models import vit as m

        cfg = m.ViTConfig()
    else:
        from die_amd.models import resnet_v2 as m

        cfg = m.ResNetConfig()
    native.kernels().die_kern_set_pair_shared_w(int(a.pair_shared_w))
    path = os.path.join(tempfile.mkdtemp(), a.arch + ".onnx")
    open(path, "wb").write(m.build_onnx(cfg)[0])
    e = native.Engine(path, device="hip", max_batch=a.hi, precision=a.precision,
                      fuse_pairs=not a.no_fuse_pairs, tune_tail=a.tune_tail)
    x = m.synthetic_input(a.hi, cfg, seed=3).reshape(a.hi, -1).astype(np.float32)
    rows = []
    for B in range(a.lo, a.hi + 1):
        for _ in range(3):
            e.run(x[:B])
        i0 = e.refresh_info()
        for _ in range(a.iters):
            e.run(x[:B])
        i1 = e.refresh_info()
        ms = (i1["device_busy_ms"] - i0["device_busy_ms"]) / (i1["batches"] - i0["batches"])
        r = {"batch": B, "device_ms": round(ms, 4), "us_per_image": round(ms * 1e3 / B, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    buckets = e.refresh_info().get("buckets")
    e.close()
    lines = ["# %s %s%s: captured-forward device time per batch size" % (
        a.arch, a.precision, (", unfused pairs" if a.no_fuse_pairs else "") + (", tail split-K tuned" if a.tune_tail else "") + (
            ", pair shared_w %d" % a.pair_shared_w if a.pair_shared_w >= -1 else "")), "",
             "Graph buckets: %s." % buckets, "", "| batch | device ms | us / image |", "|---:|---:|---:|"]
    lines += ["| %d | %.3f | %.1f |" % (r["batch"], r["device_ms"], r["us_per_image"]) for r in rows]
    text = "\n".join(lines) + "\n"
    if a.out:
        open(a.out + ".md", "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
