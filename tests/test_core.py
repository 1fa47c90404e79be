"""Unit tests of the native control plane (CPU): JSON codec, ring, breaker, cache, batcher."""
import json
import struct
import threading
import time

import numpy as np
import pytest


def py_fnv1a(s: str) -> int:
    h = 2166136261
    for b in s.encode("utf-8"):
        c = b - 256 if b >= 128 else b  # x86 `char` is signed; the reference casts char -> uint32
        h ^= c & 0xFFFFFFFF
        h = (h * 16777619) & 0xFFFFFFFF
    return h


def py_ring(nodes, vnodes=150):
    ring = {}
    for n in nodes:
        for i in range(vnodes):
            ring[py_fnv1a("%s#%d" % (n, i))] = n
    keys = sorted(ring)
    return ring, keys


def py_get(ring, keys, key):
    import bisect

    h = py_fnv1a(key)
    i = bisect.bisect_left(keys, h)
    if i == len(keys):
        i = 0
    return ring[keys[i]]


def test_fnv1a_golden(native):
    for s in ["", "a", "req_1", "localhost:8001#0", "ünïcode", "x" * 100]:
        assert native.fnv1a(s) == py_fnv1a(s)
    assert native.fnv1a("") == 2166136261


def test_ring_matches_reference_algorithm(native):
    nodes = ["localhost:8001", "localhost:8002", "localhost:8003"]
    ring = native.Ring(150)
    for n in nodes:
        ring.add(n)
    pr, keys = py_ring(nodes)
    assert len(ring) == len(pr)
    for i in range(2000):
        k = "req_%d" % i
        assert ring.get(k) == py_get(pr, keys, k)
    # failover order = distinct nodes walking the ring from hash 0
    order = []
    for h in keys:
        if pr[h] not in order:
            order.append(pr[h])
    assert ring.nodes() == order
    ring.remove("localhost:8002")
    assert "localhost:8002" not in ring.nodes()
    assert all(ring.get("req_%d" % i) != "localhost:8002" for i in range(200))


def test_ring_distribution_reasonable(native):
    ring = native.Ring(150)
    for n in ["w1:1", "w2:2", "w3:3"]:
        ring.add(n)
    counts = {}
    for i in range(30000):
        n = ring.get("req_%d" % i)
        counts[n] = counts.get(n, 0) + 1
    assert min(counts.values()) > 5000


def test_empty_ring(native):
    assert native.Ring().get("x") == ""


def test_breaker_state_machine(native):
    b = native.Breaker(5, 2, 30000)
    assert b.state()["state"] == "CLOSED"
    for _ in range(4):
        assert b.allow()
        b.failure()
    assert b.state()["state"] == "CLOSED"
    b.success()  # resets consecutive failures while CLOSED
    assert b.state()["failures"] == 0
    for _ in range(5):
        b.failure()
    assert b.state()["state"] == "OPEN"
    assert not b.allow()
    b.advance(29999)
    assert not b.allow()
    b.advance(1)
    assert b.allow()
    assert b.state()["state"] == "HALF_OPEN"
    assert b.allow()  # unlimited half-open probes, like the reference
    b.success()
    assert b.state()["state"] == "HALF_OPEN"
    b.success()
    st = b.state()
    assert st["state"] == "CLOSED" and st["failures"] == 0


def test_breaker_half_open_failure_reopens(native):
    b = native.Breaker(2, 2, 1000)
    b.failure()
    b.failure()
    assert b.state()["state"] == "OPEN"
    b.advance(1000)
    assert b.allow()
    b.failure()
    assert b.state()["state"] == "OPEN"
    assert not b.allow()  # clock restarted at the half-open failure
    b.advance(1000)
    assert b.allow()


def test_lru_cache(native):
    c = native.Cache(3)
    k = [np.array([i, i + 1, i + 2], np.float32) for i in range(5)]
    for i in range(3):
        c.put(k[i], np.array([i], np.float32))
    assert c.get(k[0])[0] == 0  # promotes k0
    c.put(k[3], np.array([3], np.float32))  # evicts k1 (LRU)
    assert c.get(k[1]) is None
    assert c.get(k[2])[0] == 2
    c.put(k[2], np.array([22], np.float32))  # overwrite
    assert c.get(k[2])[0] == 22
    st = c.stats()
    assert st["size"] == 3
    assert st["hits"] == 3 and st["misses"] == 1
    # keys are full-content: a different value in the middle of a long vector must miss
    big = np.zeros(150528, np.float32)
    c.put(big, np.array([7], np.float32))
    big2 = big.copy()
    big2[1000] = 1.0
    assert c.get(big2) is None
    assert c.get(big.copy())[0] == 7
    # -0.0 and 0.0 differ bitwise (the reference compares floats with ==; documented deviation)
    assert c.get(np.array([0.0, 1.0], np.float32)) is None


def test_lru_cache_hash_is_keyed(native):
    """Inputs built to zero a lane of an unkeyed multiply-mix hash (a 64-bit word equal to the mix
    constant) must not collide: the hash is keyed with a per-process secret and the mix keeps its
    multiplicands (lru_cache.h hash_bytes)."""
    c = native.Cache(8)
    words = np.zeros(8, np.uint64)
    words[1] = np.uint64(0xE7037ED1A0B428DB)  # the former fixed k1 of lane 0
    a, b = words.copy(), words.copy()
    a[0], b[0] = 1, 2
    ka, kb = a.view(np.float32), b.view(np.float32)
    c.put(ka, np.array([1], np.float32))
    assert c.get(kb) is None
    assert c.get(ka.copy())[0] == 1


def test_json_roundtrip(native):
    doc = '{"a":[1,2.5,-3e2,"x\\u00e9\\n"],"b":{"c":null,"d":true,"e":false},"f":-0.0,"g":1e-7}'
    out = json.loads(native.json_roundtrip(doc))
    assert out == json.loads(doc)
    with pytest.raises(native.NativeError):
        native.json_roundtrip('{"a":}')
    with pytest.raises(native.NativeError):
        native.json_roundtrip("[1,2")


@pytest.mark.parametrize("fmt", ["%.4f", "%.9g", "%.3e", "%r"])
def test_parse_infer_floats_exact(native, fmt):
    rng = np.random.default_rng(0)
    vals = (rng.standard_normal(5000) * 10.0 ** rng.integers(-8, 8, 5000)).astype(np.float32)
    if fmt == "%r":
        txt = ",".join(repr(float(v)) for v in vals)
    else:
        txt = ",".join(fmt % float(v) for v in vals)
    body = ('{"request_id": "r-1", "input_data": [%s], "extra": {"k": [1,2]}}' % txt).encode()
    rid, out, n = native.parse_infer(body, 6000)
    assert rid == "r-1" and n == 5000
    ref = np.array([float(s) for s in txt.split(",")], dtype=np.float64).astype(np.float32)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_parse_infer_errors(native):
    with pytest.raises(native.NativeError):
        native.parse_infer(b'{"request_id": "a", "input_data": [1, "x"]}', 10)
    with pytest.raises(native.NativeError):
        native.parse_infer(b'{"request_id": 5, "input_data": [1]}', 10)
    with pytest.raises(native.NativeError):
        native.parse_infer(b'{"request_id": "a", "input_data": [1,]}', 10)
    rid, out, n = native.parse_infer(b'{"input_data":[],"request_id":"z"}', 10)
    assert rid == "z" and n == 0
    # more values than capacity: count reported, extra values dropped
    rid, out, n = native.parse_infer(b'{"request_id":"q","input_data":[1,2,3,4,5]}', 3)
    assert n == 5 and list(out) == [1, 2, 3]


def test_format_floats_roundtrip(native):
    v = np.random.default_rng(1).standard_normal(1000).astype(np.float32)
    s = native.format_floats(v)
    back = np.array(json.loads(s), dtype=np.float32)
    assert np.array_equal(back, v)
    assert native.format_floats(np.array([np.nan, np.inf], np.float32)) == "[null,null]"


def test_batcher_greedy_semantics(native):
    b = native.TestBatcher(max_batch=4, timeout_ms=20, deadline=False, delay_ms=30)
    results = [None] * 20

    def run(i):
        results[i] = b.process(i)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(20)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert results == [2 * i for i in range(20)]
    m = b.metrics()
    assert m["total_requests"] == 20
    assert sum(m["sizes"]) == 20
    assert max(m["sizes"]) <= 4
    assert m["full_batches"] + m["timeout_batches"] == m["total_batches"]
    assert m["full_batches"] == sum(1 for s in m["sizes"] if s == 4)
    assert abs(m["avg_batch_size"] - 20 / m["total_batches"]) < 1e-9
    h = m["size_histogram"]  # batches per size, index 0 = size 1
    assert sum(h) == m["total_batches"] and sum((i + 1) * c for i, c in enumerate(h)) == 20
    assert all(h[s - 1] == m["sizes"].count(s) for s in set(m["sizes"]))
    b.stop()


def test_batcher_size_hook_trims_batches(native):
    """The batch-size hook (the worker wires Engine::preferred_batch into it) may take fewer than
    queued: the rest stay queued, oldest first out, and every request still completes once."""
    b = native.TestBatcher(max_batch=8, timeout_ms=20, deadline=False, delay_ms=30, size_cap=3)
    results = [None] * 20

    def run(i):
        results[i] = b.process(i)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(20)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert results == [2 * i for i in range(20)]
    m = b.metrics()
    assert sum(m["sizes"]) == 20 and max(m["sizes"]) <= 3
    # with 30 ms per batch the queue outgrows the cap, so some batches were cut
    assert m["trimmed_batches"] >= 1 and m["trimmed_requests"] >= m["trimmed_batches"]
    b.stop()


def test_batcher_no_shaping_at_low_load(native):
    """Batch shaping (balance, the engine's size hook) only while the queue holds at least half the
    max batch: a short queue behind a batch of one goes out whole (profiles/r6_batch_policy.md)."""
    b = native.TestBatcher(max_batch=8, timeout_ms=20, deadline=False, delay_ms=60, balance=True, size_cap=2)
    results = [None] * 4

    def run(i):
        results[i] = b.process(i)

    first = threading.Thread(target=run, args=(0,))
    first.start()
    time.sleep(0.02)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(1, 4)]
    for t in ts:
        t.start()
    for t in [first] + ts:
        t.join()
    assert results == [0, 2, 4, 6]
    m = b.metrics()
    assert m["sizes"] == [1, 3], m["sizes"]
    assert m["trimmed_batches"] == 0
    b.stop()


def test_batcher_deadline_waits_for_full_batch(native):
    b = native.TestBatcher(max_batch=8, timeout_ms=200, deadline=True)
    out = []

    def run(i):
        out.append(b.process(i))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    m = b.metrics()
    assert sorted(out) == [2 * i for i in range(8)]
    assert m["sizes"][0] == 8 and m["full_batches"] >= 1
    # a lone request is released by the deadline as a partial ("timeout") batch
    assert b.process(5) == 10
    m = b.metrics()
    assert m["timeout_batches"] >= 1
    b.stop()


def test_batcher_exception_propagates_and_stop_fails_fast(native):
    b = native.TestBatcher(max_batch=4, timeout_ms=5)
    with pytest.raises(native.NativeError, match="negative"):
        b.process(-1)
    assert b.process(3) == 6
    b.stop()
    with pytest.raises(native.NativeError, match="stopped"):
        b.process(1)


# ---- 4-bit text packing for the H2D copy (core/textpack.h) ----

_NIB = b"0123456789,.-+e "


def _pack_ref(t: bytes) -> bytes:
    sym = [_NIB.index(c) for c in t] + ([15] if len(t) % 2 else [])
    return bytes(a | (b << 4) for a, b in zip(sym[0::2], sym[1::2]))


@pytest.mark.parametrize("n", [0, 1, 2, 31, 63, 64, 65, 127, 128, 4095, 4096, 4097, 10001])
def test_pack_nibbles_matches_reference(native, n):
    rng = np.random.default_rng(n)
    t = bytes(rng.choice(list(_NIB), size=n).tolist())
    p = native.pack_nibbles(t)
    assert p == _pack_ref(t)
    assert native.unpack_nibbles(p, n) == t


@pytest.mark.parametrize("bad", [b"E", b"\n", b"\t", b"\r", b"a", b"]", b"\x00", b"\xff", b"/", b":", b"!"])
@pytest.mark.parametrize("pos", [0, 31, 63, 64, 5000, -1])
def test_pack_nibbles_rejects_other_bytes(native, bad, pos):
    t = bytearray(b"0.1234," * 1000)
    t[pos] = bad[0]
    assert native.pack_nibbles(bytes(t)) is None


def test_pack_nibbles_json_dumps_payload(native):
    rng = np.random.default_rng(3)
    x = rng.standard_normal(20000).astype(np.float32)
    t = json.dumps([float(v) for v in x])[1:-1].encode()  # ", " separators, e-notation, negatives
    p = native.pack_nibbles(t)
    assert p is not None and len(p) == (len(t) + 1) // 2
    assert native.unpack_nibbles(p, len(t)) == t
