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


@pytest.mark.parametrize("merge", [False, True])
def test_dp_world1_solo_and_merge(native, models, monkeypatch, merge):
    """A group of one feeds its local engine directly (dp_solo); DIE_DP_FORCE_MERGE=1 keeps the
    sub-batch ring + merge loop N>1 runs.  Both answer like the plain executor, over HTTP too."""
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    if merge:
        monkeypatch.setenv("DIE_DP_FORCE_MERGE", "1")
    else:
        monkeypatch.delenv("DIE_DP_FORCE_MERGE", raising=False)
    group = "die_dp_s%d_%d" % (os.getpid(), merge)
    wk = native.Worker(path, node_id="dp1", max_batch=8, engine={"device": "cpu", "dp_world": 1, "dp_group": group})
    try:
        h = wk.health()
        assert h["engine"]["dp_solo"] is (not merge)
        res = native.loadgen(port=wk.port, connections=8, requests=48, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 48 and res["failed"] == 0
        x = r.synthetic_input(2, cfg).reshape(2, -1)
        for i in range(2):
            body = json.dumps({"request_id": "s%d" % i, "input_data": [float(v) for v in x[i]]}).encode()
            out = json.loads(urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=body),
                                                    timeout=30).read())
            ref = native.cpu_run(path, x[i:i + 1].reshape(1, 3, 64, 64))[0]
            np.testing.assert_allclose(np.array(out["output_data"], np.float32), ref, rtol=1e-5, atol=1e-5)
        h = wk.health()
        assert h["engine"]["dp_batches"] >= 1
        assert (h["engine"]["dp_subbatches_merged"] > 0) is merge
    finally:
        wk.stop()


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


INGEST_RANK = """
import sys, os, json
sys.path.insert(0, {repo!r}); os.environ['DIE_NO_TORCH'] = '1'
import die_amd
from die_amd import native
w = native.Worker({model!r}, node_id='dp-r{rank}', port={port}, reuse_port=True, max_batch={mb},
                  engine=dict(device='cpu', dp_world={world}, dp_group={group!r}, dp_rank={rank}))
print('READY', flush=True)
sys.stdin.readline()
print('HEALTH ' + json.dumps(w.health()), flush=True)
w.stop()
"""


@pytest.mark.parametrize("world", [2, 3])
def test_dp_every_rank_ingests(native, models, world):
    """the DP leader owned all HTTP ingest.  Now every rank listens on the same port
    (SO_REUSEPORT), parses its own connections' requests into the shared arena and queues them as
    sub-batches; the leader merges the queues into DP batches and every rank answers its own."""
    import socket

    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_dp_i%d_%d" % (os.getpid(), world)
    env = dict(os.environ, DIE_NO_TORCH="1")
    ps = [subprocess.Popen([sys.executable, "-c", INGEST_RANK.format(repo=REPO, model=path, rank=k, port=port,
                                                                     mb=8, world=world, group=group)],
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
          for k in range(1, world)]
    wk = None
    try:
        wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=8,
                           engine={"device": "cpu", "dp_world": world, "dp_group": group})
        for p in ps:
            line = p.stdout.readline().decode()
            assert "READY" in line, line + p.stdout.read().decode()
        res = native.loadgen(port=port, connections=24, requests=240, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 240 and res["failed"] == 0, res
        x = r.synthetic_input(3, cfg).reshape(3, -1)
        for i in range(3):  # answers are right whichever rank took the connection
            body = json.dumps({"request_id": "ing%d" % i, "input_data": [float(v) for v in x[i]]}).encode()
            out = json.loads(urllib.request.urlopen(urllib.request.Request("http://127.0.0.1:%d/infer" % port,
                                                                           data=body), timeout=30).read())
            ref = native.cpu_run(path, x[i:i + 1].reshape(1, 3, 64, 64))[0]
            np.testing.assert_allclose(np.array(out["output_data"], np.float32), ref, rtol=1e-5, atol=1e-5)
        h0 = wk.health()
        assert h0["engine"]["dp_rank"] == 0 and h0["engine"]["dp_batches"] >= 1
    finally:
        if wk is not None:
            wk.stop()
        healths = []
        for p in ps:
            try:
                out, _ = p.communicate(b"stop\n", timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
                out, _ = p.communicate()
            healths += [json.loads(l[len("HEALTH "):]) for l in out.decode().splitlines() if l.startswith("HEALTH ")]
    assert len(healths) == world - 1
    parsed = [h0["total_requests"]] + [h["total_requests"] for h in healths]
    assert sum(parsed) >= 243 and all(n > 0 for n in parsed), parsed  # every rank ingested
    merged = h0["engine"]["dp_subbatches_merged"]
    sent = h0["engine"]["dp_subbatches_sent"] + sum(h["engine"]["dp_subbatches_sent"] for h in healths)
    assert merged == sent and merged > h0["engine"]["dp_batches"] / 2
