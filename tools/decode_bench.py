#!/usr/bin/env python3
"""Device JSON decode throughput: B ResNet-sized input_data texts (150528 values) per launch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--styles", default="4dec,repr_f32")
    ap.add_argument("--batches", default="16,32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--packed-only", action="store_true")
    args = ap.parse_args()

    import die_amd  # noqa: F401
    from die_amd import native

    L = native.kernels()
    numel = 150528
    rng = np.random.default_rng(0)
    styles = {
        "4dec": lambda: ",".join("%.4f" % v for v in rng.random(numel)).encode(),
        "repr_f32": lambda: json.dumps([float(v) for v in rng.random(numel).astype(np.float32)])[1:-1].encode(),
    }
    res = {}
    styles = {k: v for k, v in styles.items() if k in args.styles.split(",")}
    for name, gen in styles.items():
        for B in [int(b) for b in args.batches.split(",")]:
            base = [gen() for _ in range(min(4, B))]
            texts = (base * ((B + len(base) - 1) // len(base)))[:B]
            assert len(texts) == B  # one text per sample: the kernels read lens[0..B)
            cap = (numel * 24 + 4095) // 4096 * 4096
            host = np.zeros(B * cap, np.uint8)
            lens = np.array([len(t) for t in texts], np.int64)
            for i, t in enumerate(texts):
                host[i * cap:i * cap + len(t)] = np.frombuffer(t, np.uint8)
            d_text = torch.from_numpy(host).cuda()
            d_lens = torch.from_numpy(lens).cuda()
            out = torch.empty((B, numel), dtype=torch.float32, device="cuda")
            st = torch.empty(2 * B, dtype=torch.int32, device="cuda")
            scratch = torch.empty(int(L.die_decode_scratch_bytes(B, cap)), dtype=torch.uint8, device="cuda")
            s = int(torch.cuda.current_stream().cuda_stream)

            # 4-bit packed copy of the same texts (what the worker uploads): decoded straight from nibbles
            pk = [native.pack_nibbles(t) for t in texts]
            packed_ok = all(p is not None for p in pk)
            if packed_ok:
                hp = np.zeros(B * cap // 2, np.uint8)
                for i, p in enumerate(pk):
                    hp[i * cap // 2:i * cap // 2 + len(p)] = np.frombuffer(p, np.uint8)
                d_packed = torch.from_numpy(hp).cuda()
                d_poffs = torch.arange(B, dtype=torch.int64, device="cuda") * (cap // 2)

            def run(packed=False):
                if packed:
                    rc = L.die_kern_decode_packed(d_text.data_ptr(), 0, d_packed.data_ptr(), d_poffs.data_ptr(), cap,
                                                  d_lens.data_ptr(), B, out.data_ptr(), numel, st.data_ptr(),
                                                  st.data_ptr() + 4 * B, scratch.data_ptr(), s)
                else:
                    rc = L.die_kern_decode(d_text.data_ptr(), 0, cap, d_lens.data_ptr(), B, out.data_ptr(), numel,
                                           st.data_ptr(), st.data_ptr() + 4 * B, scratch.data_ptr(), s)
                assert rc == 0

            for packed in (((True,) if args.packed_only else (False, True)) if packed_ok else (False,)):
                for _ in range(3):
                    run(packed)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run(packed)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1000 / args.iters
                assert int(st[:B].abs().sum()) == 0
                res["%s%s_B%d" % (name, "_packed" if packed else "", B)] = {
                    "us": round(us, 1), "MB": round(lens.sum() / 1e6, 1), "GBps": round(lens.sum() / us / 1e3, 1),
                    "us_per_sample": round(us / B, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
