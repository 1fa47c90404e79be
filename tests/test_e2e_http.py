"""End-to-end serving tests on the CPU engine: gateway + 3 workers in-process on ephemeral ports.

Mirrors the reference's only test strategy (diagnostics.sh / benchmark.py against live processes,
SURVEY §4) and adds what it lacks: API-parity assertions on every key, routing parity with the
reference ring, cache semantics, error bodies, and breaker fail-over/recovery."""
import json
import os
import subprocess
import sys
import time
import urllib.error
import urllib.request

import numpy as np
import pytest

from test_core import py_get, py_ring


def post(url, obj=None, raw=None, timeout=30):
    data = raw if raw is not None else json.dumps(obj).encode()
    req = urllib.request.Request(url, data=data, headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def get(url, timeout=10):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.status, json.loads(r.read())


@pytest.fixture(scope="module")
def cluster(native, models):
    path = models["tiny"][0]
    workers = [native.Worker(path, node_id="w%d" % i, engine={"device": "cpu"}) for i in range(3)]
    names = ["127.0.0.1:%d" % w.port for w in workers]
    gw = native.GatewayServer(names, breaker_timeout_s=0.5)
    yield {"workers": workers, "names": names, "gw": gw, "path": path}
    gw.stop()
    for w in workers:
        w.stop()


def test_infer_through_gateway_api_parity(cluster):
    gw = cluster["gw"]
    st, out = post(gw.url + "/infer", {"request_id": "req_42", "input_data": [1.0, 2.0, 3.0]})
    assert st == 200
    assert set(out) == {"request_id", "output_data", "node_id", "cached", "inference_time_us"}
    assert out["request_id"] == "req_42"
    assert len(out["output_data"]) == 10
    assert out["cached"] is False and out["inference_time_us"] > 0
    # same request id -> same worker -> cache hit with the reference's constant 50 us
    st, out2 = post(gw.url + "/infer", {"request_id": "req_42", "input_data": [1.0, 2.0, 3.0]})
    assert st == 200 and out2["cached"] is True and out2["inference_time_us"] == 50
    assert out2["output_data"] == out["output_data"] and out2["node_id"] == out["node_id"]


def test_routing_matches_reference_ring(cluster):
    names = cluster["names"]
    ring, keys = py_ring(names)
    by_port = {w.port: "w%d" % i for i, w in enumerate(cluster["workers"])}
    for i in range(30):
        rid = "route_%d" % i
        st, out = post(cluster["gw"].url + "/infer", {"request_id": rid, "input_data": [0.1 * i]})
        assert st == 200
        expect = py_get(ring, keys, rid)
        assert out["node_id"] == by_port[int(expect.split(":")[1])]


def test_health_and_stats_keys(cluster):
    st, h = get(cluster["workers"][0].url.replace("127.0.0.1", "127.0.0.1") + "/health")
    assert st == 200
    for k in ["healthy", "node_id", "total_requests", "cache_hits", "cache_size", "cache_hit_rate", "batch_processor"]:
        assert k in h
    for k in ["total_batches", "avg_batch_size", "timeout_batches", "full_batches"]:
        assert k in h["batch_processor"]
    st, s = get(cluster["gw"].url + "/stats")
    assert st == 200 and s["total_workers"] == 3
    nodes = [b["node"] for b in s["circuit_breakers"]]
    assert nodes == sorted(nodes)
    for b in s["circuit_breakers"]:
        assert set(b) >= {"node", "state", "failures", "successes"}


def test_direct_worker_errors(cluster):
    w = cluster["workers"][0]
    st, out = post(w.url + "/infer", raw=b"{not json")
    assert st == 500 and "error" in out
    st, out = post(w.url + "/infer", {"request_id": "x"})
    assert st == 500 and "input_data" in out["error"]
    st, out = post(w.url + "/infer", {"request_id": "x", "input_data": [0.0] * (3 * 64 * 64 + 1)})
    assert st == 500  # oversized input rejected (reference: silently shifts the batch)
    st, out = post(w.url + "/infer", {"input_data": [1.0], "request_id": "ok"})
    assert st == 200


def test_padding_semantics_match_cpu_executor(cluster, native):
    w = cluster["workers"][1]
    x = np.zeros(3 * 64 * 64, np.float32)
    x[:5] = [0.5, 0.25, 0.125, 1.0, 2.0]
    st, out = post(w.url + "/infer", {"request_id": "pad", "input_data": x[:5].tolist()})
    ref = native.cpu_run(cluster["path"], x.reshape(1, 3, 64, 64))[0]
    np.testing.assert_allclose(np.array(out["output_data"], np.float32), ref, rtol=1e-5, atol=1e-5)


def test_concurrent_load_and_batching(cluster, native):
    res = native.loadgen(port=cluster["gw"].port, connections=24, requests=600, payload="ref")
    assert res["ok"] == 600 and res["failed"] == 0
    batches = [w.health()["batch_processor"] for w in cluster["workers"]]
    assert sum(b["total_batches"] for b in batches) > 0


@pytest.mark.parametrize("balance", [True, False])
def test_batch_histogram_and_balance(native, models, balance):
    """/health batch_processor: the per-size histogram accounts for every batch and request, and
    batch_balance (WorkerOptions, default on) cuts a long queue to the mean of the queue and the
    previous batch -- reported as trimmed batches / requests; off, nothing is ever cut (the CPU
    engine has no preferred batch size of its own)."""
    path = models["tiny"][0]
    w = native.Worker(path, node_id="hist", engine={"device": "cpu"}, batch_balance=balance)
    try:
        res = native.loadgen(port=w.port, connections=24, requests=480, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 480, res
        bp = w.health()["batch_processor"]
        h = bp["size_histogram"]
        assert sum(h) == bp["total_batches"]
        assert sum((i + 1) * c for i, c in enumerate(h)) == bp["total_requests"]
        assert bp["trimmed_requests"] >= bp["trimmed_batches"] >= 0
        if not balance:
            assert bp["trimmed_batches"] == 0
    finally:
        w.stop()


def test_full_payload_unique_requests(native, models):
    path = models["tiny"][0]
    w = native.Worker(path, node_id="solo", engine={"device": "cpu"})
    try:
        res = native.loadgen(port=w.port, connections=8, requests=64, payload="full", input_numel=3 * 64 * 64)
        assert res["ok"] == 64, res
        h = w.health()
        assert h["cache_hits"] == 0 and h["cache_size"] == 64
    finally:
        w.stop()


def test_failover_and_breaker_recovery(native, models):
    path = models["tiny"][0]
    workers = [native.Worker(path, node_id="f%d" % i, engine={"device": "cpu"}) for i in range(2)]
    names = ["127.0.0.1:%d" % w.port for w in workers]
    gw = native.GatewayServer(names, breaker_timeout_s=0.5, failure_threshold=5, success_threshold=2,
                              connect_timeout_ms=500, read_timeout_ms=2000)
    try:
        dead_port = workers[0].port
        workers[0].stop()
        dead = "127.0.0.1:%d" % dead_port
        ok = 0
        # ring placement depends on the (random) ports: make sure >= failure_threshold ids hit the dead node
        ring, keys = py_ring(names)
        to_dead = [r for r in ("fo_%d" % i for i in range(2000)) if py_get(ring, keys, r) == dead][:10]
        others = ["fo_%d" % i for i in range(30)]
        for i, rid in enumerate(to_dead + others):
            st, out = post(gw.url + "/infer", {"request_id": rid, "input_data": [float(i)]})
            ok += st == 200
            if st == 200:
                assert out["node_id"] == "f1"
        assert ok == 40  # zero client-visible failures while another worker is healthy
        states = {b["node"]: b for b in gw.stats()["circuit_breakers"]}
        assert states[dead]["state"] == "OPEN"
        # restart a worker on the same port; after the timeout the breaker half-opens and closes
        workers[0] = native.Worker(path, node_id="f0b", port=dead_port, engine={"device": "cpu"})
        time.sleep(0.7)
        ring, keys = py_ring(names)
        rids = [r for r in ("rec_%d" % i for i in range(400)) if py_get(ring, keys, r) == dead][:4]
        for rid in rids:
            st, out = post(gw.url + "/infer", {"request_id": rid, "input_data": [1.0]})
            assert st == 200
        states = {b["node"]: b for b in gw.stats()["circuit_breakers"]}
        assert states[dead]["state"] == "CLOSED"
    finally:
        gw.stop()
        for w in workers:
            w.stop()


def test_all_workers_down_error(native):
    gw = native.GatewayServer(["127.0.0.1:1", "127.0.0.1:2"], connect_timeout_ms=200)
    try:
        st, out = post(gw.url + "/infer", {"request_id": "x", "input_data": [1.0]})
        assert st == 500 and out["error"] == "All workers failed or circuit breakers open"
        st, out = post(gw.url + "/infer", raw=b"[1,2")
        assert st == 500 and "error" in out
    finally:
        gw.stop()


def test_binaries_cli(native, models, tmp_path):
    """worker_node/gateway binaries: positional CLI, MODEL_PATH fallback, graceful SIGTERM."""
    from die_amd import BIN_DIR

    path = models["tiny"][0]
    env = dict(os.environ, MODEL_PATH=path)
    w = subprocess.Popen([os.path.join(BIN_DIR, "worker_node"), "18931", "cliw", "--device", "cpu"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    g = subprocess.Popen([os.path.join(BIN_DIR, "gateway"), "localhost:18931", "--port", "18930"],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        for _ in range(100):
            try:
                st, out = post("http://127.0.0.1:18930/infer", {"request_id": "c1", "input_data": [1.0, 2.0]})
                if st == 200:
                    break
            except Exception:
                time.sleep(0.1)
        assert st == 200 and out["node_id"] == "cliw"
    finally:
        w.terminate()
        g.terminate()
        assert w.wait(timeout=20) == 0
        assert g.wait(timeout=20) == 0
    usage = subprocess.run([os.path.join(BIN_DIR, "worker_node")], capture_output=True, text=True)
    assert usage.returncode == 1 and "Usage" in usage.stderr


def _raw_http(port, payload, timeout=5):
    import socket

    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    try:
        s.sendall(payload)
        data = b""
        while True:
            try:
                chunk = s.recv(65536)
            except socket.timeout:
                break
            if not chunk:
                break
            data += chunk
            if b"\r\n\r\n" in data:
                head, _, body = data.partition(b"\r\n\r\n")
                for line in head.split(b"\r\n"):
                    if line.lower().startswith(b"content-length:") and len(body) >= int(line.split(b":")[1]):
                        return data
        return data
    finally:
        s.close()


@pytest.mark.parametrize("chunk", [b"ffffffffffffffff\r\nXY", b"fffffffffffffffff0\r\nXY", b"7fffffff\r\nXY"])
def test_hostile_chunk_sizes_do_not_kill_server(cluster, chunk):
    """A chunk size near 2^64 used to wrap the bounds check and abort the process."""
    port = int(cluster["gw"].url.rsplit(":", 1)[1])
    req = (b"POST /infer HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + chunk)
    out = _raw_http(port, req, timeout=2)
    assert out == b"" or out.startswith(b"HTTP/1.1 4")
    # the server is still alive and serving
    st, s = get(cluster["gw"].url + "/stats")
    assert st == 200 and s["total_workers"] == 3


def test_chunked_body_over_limit_is_413(cluster):
    port = int(cluster["gw"].url.rsplit(":", 1)[1])
    big = 600 << 20  # above the default 512 MiB body limit
    req = b"POST /infer HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + (b"%x\r\n" % big) + b"abc"
    out = _raw_http(port, req)
    assert out.startswith(b"HTTP/1.1 413"), out[:80]


def test_chunked_request_still_works(cluster):
    port = int(cluster["gw"].url.rsplit(":", 1)[1])
    body = json.dumps({"request_id": "chunky", "input_data": [1.0, 2.0]}).encode()
    half = len(body) // 2
    req = (b"POST /infer HTTP/1.1\r\nHost: x\r\nConnection: close\r\nTransfer-Encoding: chunked\r\n\r\n"
           + b"%x\r\n" % half + body[:half] + b"\r\n" + b"%x\r\n" % (len(body) - half) + body[half:] + b"\r\n0\r\n\r\n")
    out = _raw_http(port, req)
    assert out.startswith(b"HTTP/1.1 200"), out[:200]


def test_malformed_bodies_leave_breakers_closed(cluster):
    """a malformed body that still names a request_id reached every worker and each 500
    counted against its breaker, so five of them opened every breaker.  Workers now mark request
    errors (X-Die-Error: client); the gateway passes them through without failover or failure."""
    gw = cluster["gw"]
    _, before = get(gw.url + "/stats")
    for i in range(12):
        st, out = post(gw.url + "/infer", raw=b'{"request_id": "bad_%d", "input_data": [1.0, oops]}' % i)
        assert st == 500 and "error" in out
        st, out = post(gw.url + "/infer", raw=b'{"request_id": "bad2_%d"}' % i)
        assert st == 500 and "input_data" in out["error"]
    _, s = get(gw.url + "/stats")
    assert all(b["state"] == "CLOSED" for b in s["circuit_breakers"]), s
    assert s["client_errors"] - before.get("client_errors", 0) == 24
    assert s["failovers"] == before["failovers"]
    st, out = post(gw.url + "/infer", {"request_id": "good_after_bad", "input_data": [1.0]})
    assert st == 200


def test_health_io_and_log_counters(cluster):
    """SURVEY §5.5 observability: /health carries per-device I/O counters and logger statistics with
    one schema for every engine; the counters move with traffic."""
    w = cluster["workers"][1]
    _, h0 = get(w.url + "/health")
    for k in ("device_id", "h2d_bytes", "d2h_bytes", "graph_replays", "device_busy_ms", "batches", "images"):
        assert k in h0["io"], k
    for k in ("level", "lines", "suppressed"):
        assert k in h0["log"], k
    for i in range(5):
        st, _ = post(w.url + "/infer", {"request_id": "io_%d" % i, "input_data": [float(i), 2.0, 3.0, 4.5]})
        assert st == 200
    _, h1 = get(w.url + "/health")
    assert h1["io"]["batches"] > h0["io"]["batches"] and h1["io"]["images"] >= h0["io"]["images"] + 5
    assert h1["engine"]["name"].startswith("cpu")
    _, s = get(cluster["gw"].url + "/stats")
    assert "log_lines" in s and "log_lines_suppressed" in s


def _metrics(url):
    with urllib.request.urlopen(url + "/metrics", timeout=10) as r:
        assert r.headers.get("Content-Type", "").startswith("text/plain")
        text = r.read().decode()
    samples = {}
    for line in text.splitlines():
        assert line and not line.startswith(" "), line
        name_labels, value = line.rsplit(" ", 1)
        samples[name_labels] = float(value)
    return text, samples


def test_prometheus_metrics_endpoints(cluster):
    """GET /metrics on worker and gateway: Prometheus text exposition of the /health and /stats
    numbers (one sample per numeric leaf, strings as labels of `<prefix>_info`), moving with traffic."""
    w = cluster["workers"][2]
    text0, m0 = _metrics(w.url)
    key = 'die_worker_total_requests{node="w2"}'
    assert key in m0, text0[:500]
    assert any(k.startswith("die_worker_io_batches{") for k in m0)
    assert any(k.startswith("die_worker_info{") and 'node_id="w2"' in k for k in m0), text0[-300:]
    for i in range(3):
        st, _ = post(w.url + "/infer", {"request_id": "prom_%d" % i, "input_data": [float(i), 1.5]})
        assert st == 200
    _, m1 = _metrics(w.url)
    assert m1[key] >= m0[key] + 3
    gtext, g = _metrics(cluster["gw"].url)
    assert "die_gateway_routed" in g, gtext[:500]
    info = [k for k in g if k.startswith("die_gateway_info")]
    assert info and 'circuit_breakers_0_state="CLOSED"' in info[0], info
    # per-worker breaker entries come from a JSON array: an `index` label each
    assert any("index=" in k for k in g), gtext[:800]


def test_gateway_failure_logging_is_rate_limited(native, models):
    """A dead worker produces one WARN line per second per call site, not one per request (the
    reference flushes two lines per request: SURVEY Q11)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    dead = s.getsockname()[1]
    s.close()
    path = models["tiny"][0]
    live = native.Worker(path, node_id="live", engine={"device": "cpu"})
    names = ["127.0.0.1:%d" % dead, "127.0.0.1:%d" % live.port]
    gw = native.GatewayServer(names, failure_threshold=1000)
    # request ids whose ring primary is the dead worker (the ports are random, so the share of
    # ids that land on it varies run to run): each one is a failure + failover
    ring, keys = py_ring(names)
    ids = [rid for rid in ("rl_%d" % i for i in range(5000)) if py_get(ring, keys, rid) == names[0]][:60]
    try:
        _, s0 = get(gw.url + "/stats")
        for rid in ids:
            st, _ = post(gw.url + "/infer", {"request_id": rid, "input_data": [1.0]})
            assert st == 200
        _, s1 = get(gw.url + "/stats")
        emitted = s1["log_lines"] - s0["log_lines"]
        suppressed = s1["log_lines_suppressed"] - s0["log_lines_suppressed"]
        assert s1["failovers"] - s0["failovers"] >= 60
        assert emitted <= 5 and suppressed > 5, (emitted, suppressed)
    finally:
        gw.stop()
        live.stop()


def test_large_bodies_cross_shared_memory(native, models):
    """Bodies >= 64 KiB reach a co-located worker as an X-Die-Shm descriptor (the gateway received
    them into its shared-memory arena); the answer equals the direct one.  A worker that refuses
    descriptors gets the bytes instead, without a breaker failure."""
    import numpy as np

    path = models["tiny"][0]
    a = native.Worker(path, node_id="shm_a", engine={"device": "cpu"})
    b = native.Worker(path, node_id="shm_b", engine={"device": "cpu"}, accept_shm=False)
    gw = native.GatewayServer(["127.0.0.1:%d" % a.port, "127.0.0.1:%d" % b.port])
    try:
        rng = np.random.default_rng(3)
        seen = set()
        # the ring depends on the workers' (random) ports, and FNV-1a placements can be lopsided for
        # similar ids (e.g. every "big_<i>", i < 96, on one node for some port pairs): pick 8 ids
        # whose primary is each node
        names = ["127.0.0.1:%d" % a.port, "127.0.0.1:%d" % b.port]
        ring, keys = py_ring(names)
        ids = []
        for n in names:
            ids += [rid for rid in ("big_%d" % i for i in range(20000)) if py_get(ring, keys, rid) == n][:8]
        for i, rid in enumerate(ids):
            vals = np.round(rng.random(3 * 64 * 64), 4).tolist()
            body = {"request_id": rid, "input_data": vals}
            st, out = post(gw.url + "/infer", body)
            assert st == 200, out
            seen.add(out["node_id"])
            direct = a if out["node_id"] == "shm_a" else b
            st2, ref = post(direct.url + "/infer", dict(body, request_id="d_%d" % i))
            assert st2 == 200 and ref["output_data"] == out["output_data"]
        assert seen == {"shm_a", "shm_b"}
        _, s = get(gw.url + "/stats")
        assert s["shm_arena_mib"] > 0 and s["shm_forwards"] > 0 and s["byte_forwards"] > 0, s
        assert all(x["state"] == "CLOSED" and x["failures"] == 0 for x in s["circuit_breakers"]), s
        assert a.health()["shm_bodies"] > 0 and b.health()["shm_bodies"] == 0
    finally:
        gw.stop()
        a.stop()
        b.stop()
