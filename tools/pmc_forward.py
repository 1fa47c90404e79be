#!/usr/bin/env python3
"""Driver for rocprofv3 --pmc runs: a few eager ResNet50 (or ViT-B/16) forwards at batch B on the HIP
engine (one dispatch per op, no graphs, so every kernel gets its own counter sample).

usage: pmc_forward.py ARCH B ITERS [fp32|bf16] [tuned]
  tuned: autotune=True against $DIE_TUNE_CACHE, i.e. the production kernel configs (run the tuning
  once without the profiler so the cache is warm; the profiled runs then only look configs up)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    precision = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    tuned = len(sys.argv) > 5 and sys.argv[5] == "tuned"
    import torch  # noqa: F401

    import die_amd  # noqa: F401
    from die_amd import native

    if arch == "vit_b16":
        from die_amd.models import vit as m

        cfg = m.ViTConfig()
    else:
        from die_amd.models import resnet_v2 as m

        cfg = m.ResNetConfig()
    path = os.path.join(tempfile.mkdtemp(), arch + ".onnx")
    open(path, "wb").write(m.build_onnx(cfg)[0])
    e = native.Engine(path, device="hip", max_batch=B, autotune=tuned, use_graphs=False,
                      device_decode=False, precision=precision)
    x = m.synthetic_input(B, cfg).reshape(B, -1)
    for _ in range(iters):
        e.run(x)
    e.close()


if __name__ == "__main__":
    main()
