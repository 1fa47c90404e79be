"""Data-parallel HIP engine on the GPU with the RCCL communicator: weights arrive through
ncclBroadcast, logits leave through ncclAllGather.  A 1-GPU box can only form a world of one rank
(RCCL refuses two ranks on one device), which still runs the whole RCCL path: unique-id exchange
through the DpGroup segment, ncclCommInitRank, broadcast into the parameter arena, all-gather of
logits and decode status, leader D2H of the gathered rows.  Multi-rank DP is covered on the CPU
(tests/test_dp.py) with the same sharding code."""
import json
import os
import urllib.error
import urllib.request

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


@pytest.fixture(params=["solo", "merge", "merge_host"])
def dp_path(request):
    """Engine options of each DP path.  solo: a world of one feeds its local engine directly;
    merge: dp_force_merge keeps the multi-rank sub-batch ring + leader merge loop (what N>1 runs)
    at world=1, RCCL device gather; merge_host: the same with dp_backend "host" (logits + decode
    status through the host segment)."""
    return request.param


DP_OPTS = {"solo": {}, "merge": {"dp_force_merge": True}, "merge_host": {"dp_force_merge": True, "dp_backend": "host"}}


BACKEND = {"solo": "none", "merge": "rccl", "merge_host": "host"}


def test_dp_engine_rccl_world1_matches_plain_engine(native, models, dp_path):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    plain = native.Engine(path, device="hip", max_batch=8, autotune=False)
    dp = native.Engine(path, device="hip", max_batch=8, autotune=False, dp_world=1,
                       dp_group="die_gpu_dp_%s_%d" % (dp_path, os.getpid()), **DP_OPTS[dp_path])
    info = dp.refresh_info()
    # solo: no communicator is formed (its host threads cost the serving path ~13 %)
    assert info["name"].startswith("dp1(%s):hip:gfx950" % BACKEND[dp_path])
    assert info["dp_solo"] is (dp_path == "solo")
    for B in (1, 3, 8):
        x = r.synthetic_input(B, cfg, seed=B).reshape(B, -1)
        np.testing.assert_array_equal(dp.run(x), plain.run(x))
    dp.close()
    plain.close()


def test_dp_worker_rccl_world1_http(native, models, dp_path):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    wk = native.Worker(path, node_id="dp", max_batch=8,
                       engine=dict({"device": "hip", "dp_world": 1,
                                    "dp_group": "die_gpu_dpw_%s_%d" % (dp_path, os.getpid()), "autotune": False},
                                   **DP_OPTS[dp_path]))
    ref_eng = native.Engine(path, device="hip", max_batch=8, autotune=False)
    try:
        h = wk.health()
        assert h["engine"]["dp_backend"] == BACKEND[dp_path]
        assert h["engine"]["dp_device_gather"] is (dp_path == "merge")
        assert h["engine"]["dp_solo"] is (dp_path == "solo")
        res = native.loadgen(port=wk.port, connections=8, requests=64, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 64 and res["failed"] == 0
        # 3-decimal texts: the DP staging items are sized for 4-bit packed bodies of short decimals
        # (dp_arena_plan); 17-digit reprs would take the host-parse path
        x = np.array([[float("%.3f" % v) for v in row] for row in r.synthetic_input(2, cfg).reshape(2, -1)], np.float32)
        for i in range(2):  # device-decoded text through the DP path == plain engine on parsed floats
            body = ('{"request_id": "g%d", "input_data": [%s]}' % (i, ",".join("%.3f" % v for v in x[i]))).encode()
            out = json.loads(urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=body),
                                                    timeout=60).read())
            np.testing.assert_array_equal(np.array(out["output_data"], np.float32), ref_eng.run(x[i:i + 1])[0])
        assert wk.health()["device_decoded"] >= 2
        # decode status travels with the rows: too many values -> the size error, a subnormal
        # (device decode flags it) -> host re-parse, same answer as the plain engine
        vals = [float(v) for v in x[0]]
        body = json.dumps({"request_id": "big", "input_data": vals + [0.5] * 5}).encode()
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=body), timeout=60)
        assert ei.value.code == 500 and b"values" in ei.value.read()
        text = json.dumps({"request_id": "sub", "input_data": vals[:-1] + [7.0]}).replace("7.0]", "1e-45]")
        out = json.loads(urllib.request.urlopen(urllib.request.Request(wk.url + "/infer", data=text.encode()),
                                                timeout=60).read())
        xs = np.array(vals[:-1] + [1e-45], np.float32).reshape(1, -1)
        np.testing.assert_array_equal(np.array(out["output_data"], np.float32), ref_eng.run(xs)[0])
    finally:
        wk.stop()
        ref_eng.close()


def _verify_set(native, path, cfg, k, seed, max_batch=8):
    from die_amd.models import resnet_v2 as r

    x = r.synthetic_input(k, cfg, seed=seed).reshape(k, -1)
    plain = native.Engine(path, device="hip", max_batch=max_batch, autotune=False)
    ref = np.concatenate([plain.run(x[i:i + max_batch]) for i in range(0, k, max_batch)])
    plain.close()
    return x, ref


def test_dp_rccl_world1_concurrent_rows_verified(native, models, dp_path):
    """Every DP path under concurrent load (16 connections, K=12 distinct inputs, cache off so every
    request is computed): multi-row batches from several sub-batches, every answer compared with its
    input's expected logits (fp32 across batch buckets: rel-L2 <= 1e-4)."""
    path, w, cfg = models["tiny"]
    wk = native.Worker(path, node_id="dpv", max_batch=8, cache_capacity=0,
                       engine=dict({"device": "hip", "dp_world": 1, "autotune": False,
                                    "dp_group": "die_gpu_dpv_%s_%d" % (dp_path, os.getpid())}, **DP_OPTS[dp_path]))
    try:
        x, ref = _verify_set(native, path, cfg, 12, seed=21)
        res = native.loadgen(port=wk.port, connections=16, requests=384, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4)
        assert res["ok"] == 384 and res["failed"] == 0, res
        assert res["verified"] == 384 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h = wk.health()
        assert h["cache_hits"] == 0 and h["engine"]["dp_batches"] < 384
    finally:
        wk.stop()


def test_dp_rccl_world1_injected_failure_does_not_hang(native, models):
    """A rank whose batch fails before reaching the device still issues its collectives (shard flag
    cleared), so RCCL never waits on it: the failed batches' requests get 500s, every other answer
    is right, and the worker keeps serving.  The failing rank answers from the gathered rows too
    (only its own shard's items fail, as on the host backend)."""
    path, w, cfg = models["tiny"]
    wk = native.Worker(path, node_id="dpf", max_batch=8, cache_capacity=0,
                       engine={"device": "hip", "dp_world": 1, "autotune": False, "dp_force_merge": True,
                               "fail_batch_every": 3, "dp_group": "die_gpu_dpf_%d" % os.getpid()})
    try:
        x, ref = _verify_set(native, path, cfg, 8, seed=4)
        res = native.loadgen(port=wk.port, connections=8, requests=160, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4, timeout_ms=30000)
        assert res["mismatched"] == 0 and res["failed"] > 0 and res["ok"] > 0, res
        h = wk.health()
        assert h["engine"]["dp_backend"] == "rccl" and h["engine"]["options"]["fail_batch_every"] == 3
        # the failed batches still ran the collectives: their items fail through the gathered shard
        # flag (exactly the failed shard's items, as with the host backend), one count per request
        assert h["engine"]["dp_shard_failed_items"] == res["failed"], (h["engine"], res)
    finally:
        wk.stop()


RANK1 = """
import sys, os, json
sys.path.insert(0, {repo!r})
import die_amd
import torch
from die_amd import native
w = native.Worker({model!r}, node_id='dp-r1', port={port}, reuse_port=True, max_batch=16, cache_capacity=0,
                  engine=dict(device='hip', device_id=1, dp_world=2, dp_group={group!r}, dp_rank=1, autotune=False))
print('READY', flush=True)
sys.stdin.readline()
print('HEALTH ' + json.dumps(w.health()), flush=True)
w.stop()
"""


def _wait_ready(p, timeout=120.0):
    """Wait (bounded) for the rank's READY line.  Runtime notes (e.g. libdrm's missing amdgpu.ids on
    the GPU boxes) can come first, and the rank then waits on stdin, so never read to EOF or block
    without a deadline: raw reads behind select(), the rank killed if it does not come up."""
    import select
    import time

    fd = p.stdout.fileno()
    buf = b""
    end = time.time() + timeout
    while time.time() < end:
        r, _, _ = select.select([fd], [], [], max(0.0, end - time.time()))
        if not r:
            break
        chunk = os.read(fd, 4096)
        if not chunk:
            break
        buf += chunk
        if b"READY" in buf:
            return
    p.kill()
    raise AssertionError("rank never became ready: " + buf.decode(errors="replace")[-2000:])


def test_dp_rccl_two_ranks(native, models):
    """Two RCCL ranks on two GPUs (skipped on a 1-GPU box: RCCL refuses two ranks on one device):
    the follower's weights arrive by ncclBroadcast, both ranks ingest HTTP on the shared port, and
    under 32 concurrent connections (multi-row DP batches merged from both ranks' sub-batches) every
    answer is checked against its input's expected logits -- a shard/gather order mix-up would
    swap rows and show up as a mismatch."""
    import socket
    import subprocess
    import sys

    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path, w, cfg = models["tiny"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_gpu_dp2_%d" % os.getpid()
    p = subprocess.Popen([sys.executable, "-c", RANK1.format(repo=repo, model=path, port=port, group=group)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    wk = None
    x, ref = _verify_set(native, path, cfg, 24, seed=5, max_batch=16)
    try:
        wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=16, cache_capacity=0,
                           engine={"device": "hip", "dp_world": 2, "dp_group": group, "autotune": False})
        _wait_ready(p)
        res = native.loadgen(port=port, connections=32, requests=768, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4)
        assert res["ok"] == 768 and res["failed"] == 0, res
        assert res["verified"] == 768 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h0 = wk.health()
        assert h0["engine"]["dp_backend"] == "rccl" and h0["engine"]["dp_world"] == 2
        assert h0["engine"]["dp_batches"] < 768
    finally:
        if wk is not None:
            wk.stop()
        out, _ = p.communicate(b"stop\n", timeout=120)
    h1 = [json.loads(l[7:]) for l in out.decode().splitlines() if l.startswith("HEALTH ")]
    assert h1 and h1[0]["total_requests"] > 0 and h0["total_requests"] > 0


RANK1_HOST = RANK1.replace("device_id=1, dp_world=2", "device_id=0, dp_backend='host', dp_world=2")


def test_dp_host_two_ranks_one_gpu(native, models):
    """The multi-rank DP flow with real HIP engines on a 1-GPU box: two ranks (processes) share GPU 0
    and gather logits + decode status through the host segment (dp_backend "host"; RCCL itself
    refuses two ranks on one device).  Both ranks ingest HTTP on one port; under 32 concurrent
    connections the leader merges both ranks' sub-batches into multi-row DP batches sharded over the
    two engines, and every answer is checked against its own input's expected logits (a shard or
    gather order mix-up swaps rows and shows up as a mismatch) -- the sharding, merge and answer
    routing that an N-GPU run executes, minus the RCCL calls."""
    import socket
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path, w, cfg = models["tiny"]
    x, ref = _verify_set(native, path, cfg, 24, seed=6, max_batch=16)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_gpu_dph2_%d" % os.getpid()
    p = subprocess.Popen([sys.executable, "-c", RANK1_HOST.format(repo=repo, model=path, port=port, group=group)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    wk = None
    try:
        wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=16, cache_capacity=0,
                           engine={"device": "hip", "dp_world": 2, "dp_group": group, "dp_backend": "host",
                                   "autotune": False})
        _wait_ready(p)
        res = native.loadgen(port=port, connections=32, requests=768, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4, timeout_ms=30000)
        assert res["ok"] == 768 and res["failed"] == 0, res
        assert res["verified"] == 768 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h0 = wk.health()
        assert h0["engine"]["dp_backend"] == "host" and h0["engine"]["dp_world"] == 2
        assert h0["engine"]["dp_batches"] < 768  # multi-row batches were merged
    finally:
        if wk is not None:
            wk.stop()
        out, _ = p.communicate(b"stop\n", timeout=120)
    h1 = [json.loads(l[7:]) for l in out.decode().splitlines() if l.startswith("HEALTH ")]
    assert h1 and h1[0]["total_requests"] > 0 and h0["total_requests"] > 0
