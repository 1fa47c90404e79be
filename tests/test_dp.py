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
    # one OpenMP thread per follower: 8 processes x all-CPU OpenMP teams spin against each other
    # (world 8 on an 8-CPU host: 214 s instead of 3 s)
    env = dict(os.environ, DIE_NO_TORCH="1", OMP_NUM_THREADS="1" if world > 3 else os.environ.get("OMP_NUM_THREADS", ""))
    if not env["OMP_NUM_THREADS"]:
        env.pop("OMP_NUM_THREADS")
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
        # generous client timeout: 3 CPU-executor ranks with full OpenMP teams on a loaded host (pytest -n)
        # can take > 10 s for an 8-request batch; the test is about routing and answers, not speed
        res = native.loadgen(port=wk.port, connections=8, requests=80, payload="full", input_numel=3 * 64 * 64,
                             timeout_ms=120000)
        assert res["ok"] == 80 and res["failed"] == 0, res.get("errors")
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
def test_dp_world1_solo_and_merge(native, models, merge):
    """A group of one feeds its local engine directly (dp_solo); dp_force_merge keeps the
    sub-batch ring + merge loop N>1 runs.  Both answer like the plain executor, over HTTP too."""
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    group = "die_dp_s%d_%d" % (os.getpid(), merge)
    wk = native.Worker(path, node_id="dp1", max_batch=8, engine={"device": "cpu", "dp_world": 1, "dp_group": group,
                                                                "dp_force_merge": merge})
    try:
        h = wk.health()
        assert h["engine"]["dp_solo"] is (not merge) and h["engine"]["dp_force_merge"] is merge
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
        res = native.loadgen(port=port, connections=24, requests=240, payload="full", input_numel=3 * 64 * 64,
                             timeout_ms=60000)
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


# ---- row bookkeeping of a DP batch (csrc/parallel/dp_layout.h): pure functions, any world size ----

def _ref_layout(B, world, per):
    """Independent model: item i -> (rank, slot in that rank's shard)."""
    return [(i // per, i % per) for i in range(B)]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("B", [1, 5, 17, 31, 32, 64, 255])
def test_dp_layout_shards_and_gather_mapping(native, world, B):
    L = native.DpLayout(B, world)
    per = -(-B // world)
    assert L.per == per
    # shards cover [0, B) in rank order without overlap; the tail ranks may be short or empty
    covered = []
    for r in range(world):
        begin, n = L.shard(r)
        assert begin == min(B, r * per) and 0 <= n <= per
        covered += list(range(begin, begin + n))
    assert covered == list(range(B))
    # status tables: rank r's block at r*stride, slot j holds a value naming (r, j); padding and
    # the block's tail (ntok rows, shard flag) hold garbage that must never be read
    for stride in (per, 2 * 32 + 4, 2 * per + 7):
        if stride < per:
            continue
        g = np.full(world * stride, -999, np.int32)
        for r in range(world):
            begin, n = L.shard(r)
            for j in range(n):
                g[r * stride + j] = 1000 * r + j
        got = L.items_from_gathered(g, stride)
        want = [1000 * r + j for r, j in _ref_layout(B, world, per)]
        np.testing.assert_array_equal(got, want)
    # logits: every rank contributes exactly `per` rows, so the rank-major gather is item order
    row_len = 3
    rows = np.arange(world * per * row_len, dtype=np.float32).reshape(world * per, row_len)
    np.testing.assert_array_equal(L.rows_from_gathered(rows, per), rows[:B])


@pytest.mark.parametrize("world,B,failed", [(2, 7, [1]), (3, 8, [0]), (8, 61, [2, 7]), (8, 5, [6])])
def test_dp_layout_failed_rank_fails_only_its_items(native, world, B, failed):
    L = native.DpLayout(B, world)
    rank_ok = [0 if r in failed else 1 for r in range(world)]
    ok = L.item_ok(rank_ok)
    for i in range(B):
        assert ok[i] == (i // L.per not in failed), (i, L.per)


def test_dp_layout_explicit_per(native):
    """The leader fixes `per` for a batch (ceil(B / world)); followers read it from the descriptor."""
    L = native.DpLayout(10, 4, per=3)
    assert [L.shard(r) for r in range(4)] == [(0, 3), (3, 3), (6, 3), (9, 1)]
    L = native.DpLayout(10, 4, per=4)  # a larger bucket: the last rank computes nothing
    assert [L.shard(r) for r in range(4)] == [(0, 4), (4, 4), (8, 2), (10, 0)]


# ---- answers verified under concurrent load (multi-row DP batches, every response checked) ----

def _verify_set(native, path, cfg, k, seed):
    from die_amd.models import resnet_v2 as r

    x = r.synthetic_input(k, cfg, seed=seed).reshape(k, -1)
    ref = np.stack([native.cpu_run(path, x[i:i + 1].reshape(1, 3, 64, 64))[0] for i in range(k)])
    return x, ref


@pytest.mark.parametrize("world", [2, 3, 8])
def test_dp_concurrent_rows_verified(native, models, world):
    """16 concurrent connections over K=12 distinct inputs (cache off, so every request is computed):
    DP batches carry several rows from several sub-batches, and every answer is compared with its
    input's expected logits -- a swapped row or a rank-order mix-up is a mismatch, not a pass."""
    path, w, cfg = models["tiny"]
    group = "die_dp_v%d_%d" % (os.getpid(), world)
    ps = _spawn_followers(path, group, world, 8)
    wk = None
    try:
        wk = native.Worker(path, node_id="dpv", max_batch=8, cache_capacity=0,
                           engine={"device": "cpu", "dp_world": world, "dp_group": group})
        x, ref = _verify_set(native, path, cfg, 12, seed=11)
        res = native.loadgen(port=wk.port, connections=16, requests=192, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-5, timeout_ms=120000)
        assert res["ok"] == 192 and res["failed"] == 0, res
        assert res["verified"] == 192 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h = wk.health()
        assert h["cache_hits"] == 0
        assert h["engine"]["dp_batches"] < 192  # batches carried several rows
    finally:
        if wk is not None:
            wk.stop()
        outs = _reap(ps)
    assert all(rc == 0 for rc, _ in outs), outs


INGEST_RANK_NOCACHE = INGEST_RANK.replace("max_batch={mb},", "max_batch={mb}, cache_capacity=0,")


def test_dp_eight_ranks_every_rank_ingests_verified(native, models):
    """an 8-process rehearsal of the N=8 DP flow.  Eight CPU ranks share one port
    (SO_REUSEPORT), each parses its own connections into the shared arena, the leader merges all
    ranks' sub-batches into DP batches sharded over the 8 ranks (host collective in place of RCCL),
    and EVERY answer is checked against its input's logits."""
    import socket

    from die_amd.models import resnet_v2 as r

    world = 8
    path, w, cfg = models["tiny"]
    k = 16
    x = r.synthetic_input(k, cfg, seed=21).reshape(k, -1)
    ref = np.stack([native.cpu_run(path, x[i:i + 1].reshape(1, 3, 64, 64))[0] for i in range(k)])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_dp_e8_%d" % os.getpid()
    env = dict(os.environ, DIE_NO_TORCH="1", OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, "-c", INGEST_RANK_NOCACHE.format(repo=REPO, model=path, rank=q, port=port,
                                                                             mb=32, world=world, group=group)],
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
          for q in range(1, world)]
    wk = None
    try:
        wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=32, cache_capacity=0,
                           engine={"device": "cpu", "dp_world": world, "dp_group": group})
        for p in ps:
            line = p.stdout.readline().decode()
            assert "READY" in line, line + p.stdout.read().decode()
        res = native.loadgen(port=port, connections=48, requests=480, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4, timeout_ms=120000)
        assert res["ok"] == 480 and res["failed"] == 0, res
        assert res["verified"] == 480 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h0 = wk.health()
        assert h0["engine"]["dp_world"] == world and h0["engine"]["dp_batches"] < 480
    finally:
        if wk is not None:
            wk.stop()
        healths = []
        for p in ps:
            try:
                out, _ = p.communicate(b"stop\n", timeout=120)
            except subprocess.TimeoutExpired:
                p.kill()
                out, _ = p.communicate()
            healths += [json.loads(l[len("HEALTH "):]) for l in out.decode().splitlines() if l.startswith("HEALTH ")]
    assert len(healths) == world - 1
    parsed = [h0["total_requests"]] + [h["total_requests"] for h in healths]
    assert sum(parsed) >= 480 and sum(n > 0 for n in parsed) >= 4, parsed  # the kernel spread the connections
    # every rank asks its engine to pin exactly the shared arena once (one mapping of
    # the same pages per process), timed at start-up; the CPU executor pins nothing
    engines = [h0["engine"]] + [h["engine"] for h in healths]
    arena = int(round(engines[0]["dp_arena_mib"] * (1 << 20)))
    assert all(e["dp_pin_request_bytes"] == arena for e in engines), [e["dp_pin_request_bytes"] for e in engines]
    assert sum(e["dp_pin_request_bytes"] for e in engines) == world * arena
    assert all(e["dp_pinned_bytes"] == 0 for e in engines)
    assert all(0.0 <= e["dp_register_ms"] < 1000.0 for e in engines)


def test_dp_arena_at_eight_ranks_batch_256(native):
    """the shared input arena was sized for the worst-case text (24 B per value):
    10.5 GiB of /dev/shm at 8 ranks x batch 256, pinned by every rank.  Packed texts fit the
    float-sized item, so the same group now needs <= 2 GiB."""
    numel = 3 * 224 * 224
    a = native.dp_arena_plan(numel, 8, max_batch=256, device="hip", device_decode=True, pack_text=True)
    assert a["item_bytes"] == numel * 4
    assert a["bytes"] <= 2 << 30, a
    raw = native.dp_arena_plan(numel, 8, max_batch=256, device="hip", device_decode=True, pack_text=False)
    assert raw["bytes"] > 8 << 30  # the unpacked path keeps the worst-case room
    assert native.dp_arena_plan(numel, 8, max_batch=256, dp_arena_mb=512)["bytes"] == 512 << 20


FAILING_FOLLOWER = """
import sys, os
sys.path.insert(0, {repo!r}); os.environ['DIE_NO_TORCH'] = '1'
import die_amd
from die_amd import native
f = native.DpFollower({model!r}, {group!r}, 1, 2, max_batch=8, device='cpu', fail_batch_every=2)
print('served', f.join(), flush=True)
"""


def test_dp_shard_failure_fails_only_that_shard(native, models):
    """with the host gather a failed rank used to contribute zero rows and zero status,
    and the other ranks answered those rows with ok=true.  Now every rank gathers a shard flag:
    rank 1 fails every 2nd batch (fault injection) and exactly its items get a 500 -- no answer is
    wrong, and the rank-0 items of the same batches still succeed."""
    path, w, cfg = models["tiny"]
    group = "die_dp_f%d" % os.getpid()
    env = dict(os.environ, DIE_NO_TORCH="1")
    p = subprocess.Popen([sys.executable, "-c", FAILING_FOLLOWER.format(repo=REPO, model=path, group=group)],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
    wk = None
    try:
        wk = native.Worker(path, node_id="dpf", max_batch=8, cache_capacity=0,
                           engine={"device": "cpu", "dp_world": 2, "dp_group": group})
        x, ref = _verify_set(native, path, cfg, 8, seed=3)
        res = native.loadgen(port=wk.port, connections=8, requests=160, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-5, timeout_ms=120000)
        assert res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        assert res["failed"] > 0 and res["ok"] > 0, res
        assert res["verified"] == res["ok"]
        h = wk.health()
        assert h["engine"]["dp_shard_failed_items"] > 0
        assert h["errors"] >= res["failed"]
    finally:
        if wk is not None:
            wk.stop()
        out, _ = p.communicate(timeout=60)
    assert p.returncode == 0, out


def test_dp_rejects_mismatched_ranks(native, models):
    """a follower planning another program (here: bf16 vs the leader's fp32)
    must fail the group at join time, before any collective sizes a buffer from its own plan."""
    path, w, cfg = models["tiny"]
    group = "die_dp_m%d" % os.getpid()
    code = FOLLOWER.replace("device='cpu')", "device='cpu', precision='bf16')")
    env = dict(os.environ, DIE_NO_TORCH="1")
    p = subprocess.Popen([sys.executable, "-c", code.format(repo=REPO, model=path, group=group, rank=1, world=2, mb=8)],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
    try:
        with pytest.raises(native.NativeError, match="plans a different program"):
            native.Worker(path, node_id="dpm", max_batch=8, engine={"device": "cpu", "dp_world": 2, "dp_group": group})
    finally:
        out, _ = p.communicate(timeout=60)


def test_dp_two_ranks_concurrent_rows_verified(native, models):
    """Multi-row DP batches merged from BOTH ranks' sub-batches under 32 concurrent connections (CPU
    engines, host gather): every answer is checked against its own input's logits (rel 1e-4: the CPU
    executor's summation order depends on the batch it runs in; a swapped row is off by O(1)), so a
    shard / gather / answer-routing order mix-up shows up as a mismatch -- the flow an N-GPU dp_rccl
    run executes, with the host collective in place of RCCL."""
    import socket

    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    k = 24
    x = r.synthetic_input(k, cfg, seed=9).reshape(k, -1)
    plain = native.Engine(path, device="cpu", max_batch=8)
    ref = np.concatenate([plain.run(x[i:i + 8]) for i in range(0, k, 8)])
    plain.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    group = "die_dp_v2_%d" % os.getpid()
    env = dict(os.environ, DIE_NO_TORCH="1")
    p = subprocess.Popen([sys.executable, "-c", INGEST_RANK.format(repo=REPO, model=path, rank=1, port=port, mb=8,
                                                                   world=2, group=group)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
    wk = None
    try:
        wk = native.Worker(path, node_id="dp-r0", port=port, reuse_port=True, max_batch=8, cache_capacity=0,
                           engine={"device": "cpu", "dp_world": 2, "dp_group": group})
        line = p.stdout.readline().decode()
        assert "READY" in line, line + p.stdout.read().decode()
        res = native.loadgen(port=port, connections=32, requests=384, verify_inputs=x, verify_expected=ref,
                             verify_tol=1e-4, timeout_ms=60000)
        assert res["ok"] == 384 and res["failed"] == 0, res
        assert res["verified"] == 384 and res["mismatched"] == 0 and res["bad_request_id"] == 0, res
        h = wk.health()
        assert h["engine"]["dp_world"] == 2 and h["engine"]["dp_batches"] < 384
    finally:
        if wk is not None:
            wk.stop()
        p.communicate(b"stop\n", timeout=120)
