#!/usr/bin/env python3
"""Host JSON /infer parser throughput: SSE token path vs scalar SWAR path, on ResNet-shaped bodies."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import die_amd  # noqa: E402,F401
from die_amd import native  # noqa: E402


def body(decimals, n=3 * 224 * 224, signed=False, seed=0):
    rng = np.random.default_rng(seed)
    v = rng.random(n)
    if signed:
        v = v * 6 - 3
    return ('{"request_id":"r","input_data":[' + ",".join("%.*f" % (decimals, x) for x in v) + "]}").encode()


out = {}
for name, b in [("4dec_unit", body(4)), ("4dec_signed", body(4, signed=True)), ("7dec_unit", body(7)),
                ("repr_signed", ('{"request_id":"r","input_data":[' + ",".join(repr(float(x)) for x in
                                 np.random.default_rng(1).standard_normal(150528).astype(np.float32)) + "]}").encode())]:
    simd = min(native.parse_bench(b, 20, True) for _ in range(3))
    scal = min(native.parse_bench(b, 20, False) for _ in range(3))
    out[name] = {"bytes": len(b), "simd_us": round(simd, 1), "scalar_us": round(scal, 1),
                 "simd_GBps": round(len(b) / simd / 1e3, 2)}
print(json.dumps(out))
