#!/usr/bin/env python3
"""Diagnose two host-gather DP ranks sharing GPU 0: print a timestamped line at every stage (and
every 5 s while waiting) so a stall names its stage.  Run under `timeout`."""
import json
import os
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
T0 = time.time()


def log(*a):
    print("[%6.2f]" % (time.time() - T0), *a, flush=True)


RANK1 = """
import sys, os, json, time
sys.path.insert(0, {repo!r})
import die_amd
import torch
from die_amd import native
print('R1 start', flush=True)
w = native.Worker({model!r}, node_id='dp-r1', port={port}, reuse_port=True, max_batch=16, cache_capacity=0,
                  engine=dict(device='hip', device_id=0, dp_backend='host', dp_world=2, dp_group={group!r}, dp_rank=1,
                              autotune=False))
print('READY', flush=True)
sys.stdin.readline()
print('HEALTH ' + json.dumps(w.health()), flush=True)
w.stop()
print('R1 stopped', flush=True)
"""


def main():
    import die_amd  # noqa: F401
    import torch  # noqa: F401
    from die_amd import native
    from die_amd.models import resnet_v2 as r

    tmp = "/tmp/dp2probe_%d" % os.getpid()
    os.makedirs(tmp, exist_ok=True)
    cfg = r.tiny_config()
    path = os.path.join(tmp, "tiny.onnx")
    log("building model")
    b, _ = r.build_onnx(cfg)
    with open(path, "wb") as f:
        f.write(b)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_dp2probe_%d" % os.getpid()
    p = subprocess.Popen([sys.executable, "-c", RANK1.format(repo=REPO, model=path, port=port, group=group)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)

    def pump():
        for line in p.stdout:
            log("rank1:", line.decode().rstrip()[:300])
    threading.Thread(target=pump, daemon=True).start()
    log("creating rank 0 worker")
    wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=16, cache_capacity=0,
                       engine={"device": "hip", "dp_world": 2, "dp_group": group, "dp_backend": "host",
                               "autotune": False})
    log("rank 0 worker up", json.dumps(wk.health()["engine"].get("name")))
    x = r.synthetic_input(4, cfg, seed=1).reshape(4, -1)
    for conns, reqs in ((1, 4), (4, 32), (32, 256)):
        log("loadgen", conns, reqs)
        res = native.loadgen(port=port, connections=conns, requests=reqs, payload="full", input_numel=x.shape[1],
                             timeout_ms=20000)
        log("  ok", res["ok"], "failed", res["failed"], res.get("errors"))
    log("stopping")
    wk.stop()
    p.stdin.write(b"stop\n")
    p.stdin.flush()
    p.wait(timeout=30)
    log("done")


if __name__ == "__main__":
    main()
