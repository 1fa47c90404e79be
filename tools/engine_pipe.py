#!/usr/bin/env python3
"""Forward time with and without back-to-back batches: T host threads each call Engine.run (or
run_text, the serving path's decode) in a loop, so with T >= 2 the engine's pipeline slots keep the
compute stream full the way the serving loop does, and with T = 1 every forward runs alone.
Prints one JSON line: device ms per batch (hipGraph MAIN, events around it), wall ms per batch,
GPU busy fraction.  Usage: engine_pipe.py --arch resnet50 --batch 20 --threads 3 [--text]"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", choices=["resnet50", "vit_b16"], default="resnet50")
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--threads", type=int, default=3)
    ap.add_argument("--iters", type=int, default=200, help="batches per thread (timed)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--text", action="store_true", help="run_text: packed JSON text decoded on the device")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--model", default="")
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
    path = a.model
    if not path:
        path = os.path.join(tempfile.mkdtemp(), a.arch + ".onnx")
        open(path, "wb").write(m.build_onnx(cfg)[0])
    e = native.Engine(path, device="hip", max_batch=max(a.batch, 32), precision=a.precision)
    x = m.synthetic_input(a.batch, cfg, seed=1).reshape(a.batch, -1).astype(np.float32)
    texts = [",".join("%.4f" % v for v in row).encode() for row in x] if a.text else None

    def one():
        if texts is not None:
            e.run_text(texts, pack=True)
        else:
            e.run(x)

    def loop(n):
        for _ in range(n):
            one()

    for _ in range(a.warmup):
        one()
    i0 = e.refresh_info()
    ts = [threading.Thread(target=loop, args=(a.iters,)) for _ in range(a.threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    i1 = e.refresh_info()
    nb = i1["batches"] - i0["batches"]
    busy = i1["device_busy_ms"] - i0["device_busy_ms"]
    print(json.dumps({"arch": a.arch, "batch": a.batch, "threads": a.threads, "text": a.text, "batches": nb,
                      "device_ms_per_batch": round(busy / nb, 4), "wall_ms_per_batch": round(wall * 1e3 / nb, 4),
                      "gpu_busy": round(busy / (wall * 1e3), 4), "images_per_s": round(nb * a.batch / wall, 1)}))
    e.close()


if __name__ == "__main__":
    main()
