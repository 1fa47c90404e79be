#!/bin/bash
# live batch (skip bucket padding): numerics, engine forward at odd batch sizes, headline A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r47
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
timeout -k 10 300 python - > $O/live_fwd.txt <<'PY'
import os, sys, numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import torch, die_amd
from die_amd import native
from die_amd.models import resnet_v2 as r
import tempfile
cfg = r.ResNetConfig(); blob, _ = r.build_onnx(cfg)
d = tempfile.mkdtemp(); p = os.path.join(d, "m.onnx"); open(p, "wb").write(blob)
import time
for live in (True, False):
    e = native.Engine(p, device="hip", max_batch=32, live_batch=live)
    for B in (17, 20, 23, 24, 25, 28, 32):
        x = r.synthetic_input(B, cfg).reshape(B, -1)
        for _ in range(5): e.run(x)
        i0 = e.refresh_info(); n0, t0 = i0.get("batches", 0), i0.get("avg_device_ms", 0) * i0.get("batches", 0)
        for _ in range(50): e.run(x)
        i1 = e.refresh_info(); n1, t1 = i1["batches"], i1["avg_device_ms"] * i1["batches"]
        print("live=%d B=%d device ms %.4f" % (live, B, (t1 - t0) / (n1 - n0)), flush=True)
    e.close()
PY
cat $O/live_fwd.txt
i=0
for l in 1 0 1 0; do
  i=$((i+1))
  DIE_LIVE_BATCH=$l timeout -k 10 300 python bench.py --steps 400 --warmup 20 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [live=$l] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3))")"
done
