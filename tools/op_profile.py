#!/usr/bin/env python3
"""Per-op device time of one forward on the HIP engine (events around eager launches of the tuned
kernels), written as a markdown table + JSON.  Usage: op_profile.py --arch resnet50|vit_b16 --batch 32"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", choices=["resnet50", "vit_b16"], default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--tune-warm-input", action="store_true", help="autotune with each conv's producer run first")
    ap.add_argument("--splitk-fused-margin", type=float, default=0.0, help="prefer fused split-K within this fraction")
    ap.add_argument("--splitk-two-kernel", action="store_true", help="allow the two-kernel split-K form")
    ap.add_argument("--no-fuse-pairs", action="store_true", help="unfused expand/reduce convs (EngineOptions::fuse_pairs)")
    ap.add_argument("--ln-xcd", type=int, default=0, help="LayerNorm row order: 1 XCD-affine, 0 natural (default)")
    ap.add_argument("--no-fold-layernorm", action="store_true", help="standalone LayerNorms (EngineOptions::fold_layernorm)")
    ap.add_argument("--tune-in-graph", action="store_true", help="EngineOptions::tune_in_graph")
    ap.add_argument("--no-tune-orders", action="store_true", help="heuristic XCD tile order only (EngineOptions::tune_orders)")
    ap.add_argument("--tune-tail", action="store_true", help="tail split-K candidates too (EngineOptions::tune_tail)")
    ap.add_argument("--tune-streamk", type=int, default=-1, help="EngineOptions::tune_streamk (1 / 0; -1 default)")
    ap.add_argument("--conv-order", type=int, default=0, help="EngineOptions::conv_order (XCD tile order override)")
    ap.add_argument("--no-ln-stats-epilogue", action="store_true",
                    help="LayerNorm statistics launches instead of producer-epilogue partials (EngineOptions::ln_stats_epilogue)")
    ap.add_argument("--fuse-gap-fc", action="store_true", help="global pool and FC head as one launch (EngineOptions::fuse_gap_fc)")
    ap.add_argument("--no-fuse-stem-pool", action="store_true", help="stem and max pool as two launches (EngineOptions::fuse_stem_pool)")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)

    import die_amd  # noqa: F401
    from die_amd import native

    if a.arch == "vit_b16":
        from die_amd.models import vit as m

        cfg = m.ViTConfig()
    else:
        from die_amd.models import resnet_v2 as m

        cfg = m.ResNetConfig()
    d = tempfile.mkdtemp()
    path = os.path.join(d, a.arch + ".onnx")
    open(path, "wb").write(m.build_onnx(cfg)[0])
    native.kernels().die_kern_set_layernorm_xcd(int(a.ln_xcd))
    e = native.Engine(path, device="hip", max_batch=a.batch, precision=a.precision,
                      tune_warm_input=a.tune_warm_input, fuse_pairs=not a.no_fuse_pairs,
                      splitk_fused_margin=a.splitk_fused_margin, splitk_two_kernel=a.splitk_two_kernel,
                      fuse_stem_pool=not a.no_fuse_stem_pool, fuse_gap_fc=a.fuse_gap_fc, fold_layernorm=not a.no_fold_layernorm,
                      ln_stats_epilogue=not a.no_ln_stats_epilogue, tune_in_graph=a.tune_in_graph, conv_order=a.conv_order,
                      tune_orders=not a.no_tune_orders, tune_tail=a.tune_tail,
                      **({} if a.tune_streamk < 0 else {"tune_streamk": bool(a.tune_streamk)}))
    p = e.profile(a.batch, a.iters)
    info = e.refresh_info()
    e.close()
    lines = ["# %s per-op device time, batch %d (MI355X, %s, tuned kernels)" % (a.arch, p["batch"], a.precision), "",
             "Total %.1f us per forward = %.1f TFLOP/s over the whole graph; %.0f images/s device-bound." % (
                 p["total_us"], p["tflops"], p["batch"] / p["total_us"] * 1e6), "",
             "In-graph retune: %s (%s candidates timed in place, %s convs changed)." % (
                 "on" if a.tune_in_graph else "off", info.get("tune_in_graph_timed"), info.get("tune_in_graph_changed")), "",
             "| # | op | kind | us | GFLOP | TFLOP/s | tile/splits |", "|---:|---|---|---:|---:|---:|---|"]
    for i, o in enumerate(p["ops"]):
        ts = ("%d/%d" % (o["tile"], o["splits"]) + ("f" if o.get("fused_splitk") else "") + ("t" if o.get("tail_splitk") else "")) if "tile" in o else ""
        lines.append("| %d | %s | %s | %.1f | %.2f | %.0f | %s |" % (i, o["name"][:48], o["kind"], o["us"], o["gflop"],
                                                                    o["tflops"], ts))
    kinds = {}
    for o in p["ops"]:
        kinds[o["kind"]] = kinds.get(o["kind"], 0) + o["us"]
    lines += ["", "| kind | us | share |", "|---|---:|---:|"]
    for k, v in sorted(kinds.items(), key=lambda kv: -kv[1]):
        lines.append("| %s | %.1f | %.1f%% |" % (k, v, 100 * v / p["total_us"]))
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        open(a.out + ".md", "w").write(text)
        json.dump(p, open(a.out + ".json", "w"), indent=1)


if __name__ == "__main__":
    main()
