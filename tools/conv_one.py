#!/usr/bin/env python3
"""Launch ONE conv shape/config repeatedly (eager, no graph): the target process for rocprofv3
--pmc / --kernel-trace runs on a single kernel.
  python tools/conv_one.py --shape s3.3x3 --batch 16 --cfg 7 --splits 1 [--fused] --iters 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="s3.3x3")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--cfg", type=int, default=7)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    import die_amd  # noqa: F401
    from die_amd.ops import kernels as K
    from conv_bench import resnet50_shapes

    sh = {s[0]: s for s in resnet50_shapes()}[a.shape]
    _, _, cin, cout, k, stride, H, epi = sh
    B = a.batch
    x = (torch.randn(B, H, H, cin, device="cuda") * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
    Ho = (H + 2 * (k // 2) - k) // stride + 1
    kw = dict(bias=torch.randn(cout, device="cuda") * 0.1, stride=stride, pad=k // 2)
    if epi == "relu":
        kw["relu"] = True
    elif epi == "res_dual":
        kw.update(res=torch.randn(B, Ho, Ho, cout, device="cuda").to(torch.bfloat16),
                  scale2=torch.rand(cout, device="cuda") + 0.5, shift2=torch.randn(cout, device="cuda") * 0.1,
                  relu2=True)
    elif epi == "f32":
        kw["out_f32"] = True
    pr = K.ConvProblem(x, w, max_splits=max(1, a.splits), **kw)
    for _ in range(a.iters):
        rc = pr.launch(a.cfg, a.splits, a.fused)
        if rc:
            raise SystemExit("launch failed: %d" % rc)
    torch.cuda.synchronize()
    print("ok", a.shape, "M=%d N=%d K=%d" % (B * Ho * Ho, cout, cin * k * k))


if __name__ == "__main__":
    main()
