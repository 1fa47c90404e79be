"""Data-parallel serving (one worker fanning batches over N ranks, one process per rank) on the CPU:
leader = in-process worker, followers = separate processes attached through the shared-memory
DpGroup, host communicator for the output all-gather (SURVEY §2.4 / §2.5 fake-communicator path;
the HIP/RCCL path is tests/test_gpu_dp.py)."""
import json
import os
import subprocess
import sys
import time
import urllib.request

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FOLLOWER = """
import sys, os
sys.path.insert(0, {repo!r}); os.environ['DIE_NO_TORCH'] = '1'
import die_amd
from die_amd import native
f = native.DpFollower({model!r}, {group!r}, {rank}, {world}, max_batch={mb}, device='cpu')
print('served', f.join(), flush=True)
"""


def _spawn_followers(model, group, world, mb):
    env = dict(os.environ, DIE_NO_TORCH="1")
    return [subprocess.Popen([sys.executable, "-c", FOLLOWER.format(repo=REPO, model=model, group=group, rank=r,
                                                                      world=world, mb=mb)],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
            for r in range(1, world)]


def _reap(ps):
    outs = []
    for p in ps:
        try:
            out, _ = p.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out.decode()))
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_dp_worker_cpu(native, models, world):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    group = "die_dp_t%d_%d" % (os.getpid(), world)
    ps = _spawn_followers(path, group, world, 8)
    wk = None
    try:
        wk = native.Worker(path, node_id="dp", max_batch=8,
                           engine={"device": "cpu", "dp_world": world, "dp_group": group})
        h = wk.health()
        assert h["engine"]["dp_world"] == world and h["engine"]["dp_backend"] == "host"
        assert h["engine"]["name"].startswith("dp%d(host)" % world)
        res = native.loadgen(port=wk.port, connections=8, requests=80, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 80 and res["failed"] == 0
        x = r.synthetic_input(4, cfg).reshape(4, -1)
        for i in range(4):
            body = json.dumps({"request_id": "dp%d" % i, "input_data": [float(v) for v in x[i]]}).encode()
            out = json.loads(urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=body),
                                                    timeout=30).read())
            ref = native.cpu_run(path, x[i:i + 1].reshape(1, 3, 64, 64))[0]
            np.testing.assert_allclose(np.array(out["output_data"], np.float32), ref, rtol=1e-5, atol=1e-5)
        h = wk.health()
        assert h["engine"]["dp_batches"] >= 1
        assert h["batch_processor"]["total_requests"] >= 84
    finally:
        if wk is not None:
            wk.stop()
        outs = _reap(ps)
    for rc, out in outs:
        assert rc == 0, out
        assert "served" in out and int(out.split("served")[1].split()[0]) >= 1, out


def test_dp_engine_uneven_shards(native, models):
    """B not divisible by the world size: the last rank pads; rows come back in item order."""
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    world = 2
    group = "die_dp_e%d" % os.getpid()
    ps = _spawn_followers(path, group, world, 8)
    e = None
    try:
        e = native.Engine(path, device="cpu", max_batch=8, dp_world=world, dp_group=group)
        for B in (1, 3, 5, 8):
            x = r.synthetic_input(B, cfg, seed=B).reshape(B, -1)
            got = e.run(x)
            ref = native.cpu_run(path, x.reshape(B, 3, 64, 64))
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    finally:
        if e is not None:
            e.close()
        outs = _reap(ps)
    assert all(rc == 0 for rc, _ in outs), outs


def test_dp_follower_reports_missing_group(native, models):
    path = models["tiny"][0]
    # attach waits for the leader; a follower stopped before the leader appears exits cleanly
    f = native.DpFollower(path, "die_dp_absent_%d" % os.getpid(), 1, 2, device="cpu")
    time.sleep(0.2)
    assert f.status()["running"] is True
    assert f.join(stop=True) == 0
