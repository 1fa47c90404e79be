#!/usr/bin/env python3
"""Reference-compatible load client (same CLI and report layout as the reference benchmark.py,
benchmark.py:222-242 there), reimplemented, plus options the reference lacks.

    python tools/benchmark.py --gateway http://localhost:8000 --requests 10000 --threads 50

Default payload is the reference's: request i sends [a, a+1, a+2] with a = i % 10
(benchmark.py:21-24 there), i.e. ~10 distinct inputs per worker and ~99.7 % cache hits.
Extras: --payload full (ResNet-shaped unique inputs), --keep-alive (one requests.Session per
thread; the reference opens a new connection per request), --json (machine-readable summary).
For throughput ceilings use the C++ client (`distributed-inference-engine-cpp_amd/bin/loadgen`):
Python threads and the GIL cap this one.
"""
import argparse
import json
import statistics
import threading
import time
from collections import Counter

import requests


def make_payload(i, kind, numel, rng_state):
    if kind == "ref":
        a = float(i % 10)
        return {"request_id": "req_%d" % i, "input_data": [a, a + 1.0, a + 2.0]}
    import random

    r = random.Random(rng_state * 1000003 + i)
    return {"request_id": "req_%d" % i, "input_data": [round(r.random(), 4) for _ in range(numel)]}


class Runner:
    def __init__(self, url, n, threads, payload, numel, keep_alive, timeout):
        self.url, self.n, self.threads = url.rstrip("/"), n, threads
        self.payload, self.numel, self.keep_alive, self.timeout = payload, numel, keep_alive, timeout
        self.lat, self.ok, self.errors = [], 0, Counter()
        self.lock = threading.Lock()

    def worker(self, tid, per):
        sess = requests.Session() if self.keep_alive else requests
        for k in range(per):
            i = tid * per + k
            body = make_payload(i, self.payload, self.numel, tid)
            t0 = time.time()
            try:
                r = sess.post(self.url + "/infer", json=body, timeout=self.timeout)
                ms = (time.time() - t0) * 1000
                with self.lock:
                    if r.status_code == 200:
                        self.ok += 1
                        self.lat.append(ms)
                    else:
                        self.errors["HTTP %d" % r.status_code] += 1
            except Exception as e:  # noqa: BLE001 - count every transport failure kind
                with self.lock:
                    self.errors[type(e).__name__] += 1

    def run(self):
        per = self.n // self.threads
        ts = [threading.Thread(target=self.worker, args=(t, per)) for t in range(self.threads)]
        t0 = time.time()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        self.wall = time.time() - t0
        self.total = per * self.threads
        return self

    def summary(self):
        lat = sorted(self.lat)
        pick = lambda q: lat[min(len(lat) - 1, int(len(lat) * q))] if lat else 0.0  # noqa: E731
        return {
            "total_requests": self.total, "successful": self.ok, "failed": self.total - self.ok,
            "total_time": self.wall, "throughput": self.ok / self.wall if self.wall else 0.0,
            "latency": {"mean": statistics.mean(lat) if lat else 0.0, "p50": pick(0.5), "p90": pick(0.9),
                        "p95": pick(0.95), "p99": pick(0.99), "min": lat[0] if lat else 0.0,
                        "max": lat[-1] if lat else 0.0,
                        "stdev": statistics.stdev(lat) if len(lat) > 1 else 0.0},
            "errors": dict(self.errors),
        }


def print_report(s):
    bar = "=" * 70
    print(bar + "\nBENCHMARK RESULTS\n" + bar + "\n")
    print("Throughput")
    print("  Total requests:     %d" % s["total_requests"])
    print("  Successful:         %d" % s["successful"])
    print("  Failed:             %d" % s["failed"])
    print("  Success rate:       %.2f%%" % (100.0 * s["successful"] / max(1, s["total_requests"])))
    print("  Total time:         %.2fs" % s["total_time"])
    print("  Requests/sec:       %.2f\n" % s["throughput"])
    L = s["latency"]
    print("Latency (ms):")
    for k in ("mean", "p50", "stdev", "min", "max"):
        print("  %-19s %.2f" % (("Median" if k == "p50" else k.capitalize()) + ":", L[k]))
    print("\nPercentiles (ms):")
    for k in ("p50", "p90", "p95", "p99"):
        print("  %-19s %.2f" % (k + ":", L[k]))
    if s["errors"]:
        print("\nErrors:")
        for k, v in s["errors"].items():
            print("  %s: %d" % (k, v))
    print(bar)


def system_stats(gateway, workers):
    print("\n" + "=" * 70 + "\nSYSTEM STATISTICS\n" + "=" * 70 + "\n")
    try:
        st = requests.get(gateway + "/stats", timeout=5).json()
        print("Gateway Circuit Breakers:")
        for b in st.get("circuit_breakers", []):
            print("  %s: %s (failures: %s, successes: %s)" % (b["node"], b["state"], b["failures"], b["successes"]))
        print()
    except Exception:  # noqa: BLE001
        pass
    for w in workers:
        try:
            h = requests.get(w + "/health", timeout=5).json()
        except Exception:  # noqa: BLE001
            continue
        bp = h.get("batch_processor", {})
        print("Worker %s (%s):" % (h.get("node_id", "?"), w))
        print("  Total requests:    %s" % h.get("total_requests", 0))
        print("  Cache size:        %s" % h.get("cache_size", 0))
        print("  Cache hits:        %s" % h.get("cache_hits", 0))
        print("  Cache hit rate:    %.2f%%" % (100 * h.get("cache_hit_rate", 0)))
        print("  Avg batch size:    %.2f" % bp.get("avg_batch_size", 0))
        print("  Total batches:     %s" % bp.get("total_batches", 0))
        print("  Full batches:      %s" % bp.get("full_batches", 0))
        print("  Timeout batches:   %s\n" % bp.get("timeout_batches", 0))


def cache_test(gateway):
    def phase(prefix):
        lat = []
        for i in range(100):
            a = float(i % 10)
            t0 = time.time()
            requests.post(gateway + "/infer", json={"request_id": "%s_%d" % (prefix, i),
                                                    "input_data": [a, a + 1, a + 2]}, timeout=10)
            lat.append((time.time() - t0) * 1000)
        return statistics.mean(lat)

    miss = phase("cache_miss")
    time.sleep(1)
    hit = phase("cache_hit")
    print("CACHE TEST: miss-phase mean %.2f ms, hit-phase mean %.2f ms, speedup %.2fx" % (miss, hit, miss / hit))


def main():
    ap = argparse.ArgumentParser(description="Benchmark the distributed inference system")
    ap.add_argument("--gateway", default="http://localhost:8000")
    ap.add_argument("--requests", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=10)
    ap.add_argument("--workers", nargs="+",
                    default=["http://localhost:8001", "http://localhost:8002", "http://localhost:8003"])
    ap.add_argument("--cache-test", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--payload", choices=["ref", "full"], default="ref")
    ap.add_argument("--input-numel", type=int, default=3 * 224 * 224)
    ap.add_argument("--keep-alive", action="store_true")
    ap.add_argument("--timeout", type=float, default=10.0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    if a.cache_test:
        cache_test(a.gateway)
    print("Starting benchmark:\n  Gateway: %s\n  Requests: %d\n  Threads: %d\n" % (a.gateway, a.requests, a.threads))
    s = Runner(a.gateway, a.requests, a.threads, a.payload, a.input_numel, a.keep_alive, a.timeout).run().summary()
    if a.json:
        print(json.dumps(s))
    else:
        print_report(s)
    if not a.no_stats:
        system_stats(a.gateway, a.workers)


if __name__ == "__main__":
    main()
