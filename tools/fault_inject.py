#!/usr/bin/env python3
"""Fault-injection drills for the gateway + worker cluster (BASELINE.json config 3).

Starts real `worker_node` processes and a `gateway` process (the in-tree binaries), drives load with
the C++ `loadgen` binary, injects a fault into one worker while the load runs, and reports the
circuit-breaker timeline read from the gateway's /stats plus the client-visible outcome.

Faults:
  kill    SIGKILL the worker, restart it on the same port after --down-s seconds
  hang    SIGSTOP the worker (requests time out), SIGCONT it after --down-s seconds
  errors  POST /admin/fault {"fail_rate": 1.0} (every /infer returns 500), then reset to 0

    python tools/fault_inject.py --model m.onnx --workers 3 --fault kill --device cpu
Reference behaviour being exercised: src/gateway.cpp:38-61 (primary, then every other node in ring
order), src/circuit_breaker.cpp:12-47 (5 failures -> OPEN, timeout -> HALF_OPEN, 2 successes ->
CLOSED).
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time
import urllib.request

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "distributed-inference-engine-cpp_amd", "bin")


def _get(url, timeout=2.0):
    return json.loads(urllib.request.urlopen(url, timeout=timeout).read())


def _wait_http(url, timeout_s=60.0):
    t0 = time.time()
    while time.time() - t0 < timeout_s:
        try:
            return _get(url, 1.0)
        except Exception:
            time.sleep(0.1)
    raise RuntimeError("timed out waiting for " + url)


class Cluster:
    def __init__(self, model, n_workers=3, device="cpu", base_port=0, breaker_timeout_s=1.0, failure_threshold=5,
                 success_threshold=2, read_timeout_ms=2000, connect_timeout_ms=500, log_dir=None, worker_threads=0,
                 stagger=False, worker_args=()):
        import socket

        def free_port():
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
            s.close()
            return p

        self.model, self.device = model, device
        self.ports = [base_port + i if base_port else free_port() for i in range(n_workers)]
        self.gw_port = base_port + n_workers if base_port else free_port()
        self.log_dir = log_dir
        self.env = dict(os.environ)
        if worker_threads:  # CPU workers share the host: cap each one's OpenMP pool
            self.env["OMP_NUM_THREADS"] = str(worker_threads)
        self.worker_args = list(worker_args)
        self.workers = [None] * n_workers
        # stagger: GPU workers start one at a time (the first fills the autotune cache the others load;
        # HIP workers sharing GPU 0 is the reference's own topology)
        for i in range(n_workers):
            self.start_worker(i)
            if stagger:
                _wait_http("http://127.0.0.1:%d/health" % self.ports[i], 300.0)
        for p in self.ports:
            _wait_http("http://127.0.0.1:%d/health" % p, 300.0)
        args = [os.path.join(BIN, "gateway")] + ["127.0.0.1:%d" % p for p in self.ports] + [
            "--port", str(self.gw_port), "--host", "127.0.0.1", "--breaker-timeout-s", str(breaker_timeout_s),
            "--failure-threshold", str(failure_threshold), "--success-threshold", str(success_threshold),
            "--read-timeout-ms", str(read_timeout_ms), "--connect-timeout-ms", str(connect_timeout_ms)]
        self.gw = subprocess.Popen(args, stdout=self._log("gateway"), stderr=subprocess.STDOUT,
                                   start_new_session=True)
        _wait_http(self.url + "/stats")

    def _log(self, name):
        if not self.log_dir:
            return subprocess.DEVNULL
        os.makedirs(self.log_dir, exist_ok=True)
        return open(os.path.join(self.log_dir, name + ".log"), "ab")

    @property
    def url(self):
        return "http://127.0.0.1:%d" % self.gw_port

    def node(self, i):
        return "127.0.0.1:%d" % self.ports[i]

    def start_worker(self, i):
        args = [os.path.join(BIN, "worker_node"), str(self.ports[i]), "w%d" % i, self.model, "--host", "127.0.0.1",
                "--device", self.device] + self.worker_args
        self.workers[i] = subprocess.Popen(args, stdout=self._log("worker%d" % i), stderr=subprocess.STDOUT,
                                           start_new_session=True, env=self.env)

    def signal(self, i, sig):
        self.workers[i].send_signal(sig)

    def restart(self, i, wait=True):
        self.workers[i].wait(timeout=10)
        self.start_worker(i)
        if wait:
            _wait_http("http://127.0.0.1:%d/health" % self.ports[i], 300.0)

    def stats(self):
        return _get(self.url + "/stats")

    def breaker(self, i):
        for b in self.stats()["circuit_breakers"]:
            if b["node"] == self.node(i):
                return b
        raise KeyError(self.node(i))

    def close(self):
        procs = [self.gw] + [w for w in self.workers if w is not None]
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(signal.SIGCONT)
                    p.terminate()
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


def run_load(port, requests, connections, out, input_numel=0):
    # unique full-size inputs (no cache hits) keep the load running through the fault window;
    # input_numel=0 -> the reference's 3-float payload
    cmd = [os.path.join(BIN, "loadgen"), "--port", str(port), "--requests", str(requests), "--connections",
           str(connections), "--timeout-ms", "20000"]
    cmd += ["--payload", "full", "--input-numel", str(input_numel)] if input_numel else ["--payload", "ref"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    text = r.stdout.decode().strip().splitlines()
    out["result"] = json.loads(text[-1]) if text else {"error": r.stderr.decode()}


def drill(cluster, fault, target=0, down_s=2.0, requests=4000, connections=8, poll_s=0.05, input_numel=0):
    """Inject `fault` into worker `target` under load; return a report dict."""
    out = {}
    th = threading.Thread(target=run_load, args=(cluster.gw_port, requests, connections, out, input_numel))
    th.start()
    timeline = []
    t0 = time.time()

    def sample():
        b = cluster.breaker(target)
        if not timeline or timeline[-1][1] != b["state"]:
            timeline.append((round(time.time() - t0, 3), b["state"]))
        return b

    time.sleep(0.5)
    sample()
    if fault == "kill":
        cluster.signal(target, signal.SIGKILL)
    elif fault == "hang":
        cluster.signal(target, signal.SIGSTOP)
    elif fault == "errors":
        req = urllib.request.Request("http://%s/admin/fault" % cluster.node(target),
                                     data=json.dumps({"fail_rate": 1.0}).encode())
        urllib.request.urlopen(req, timeout=5).read()
    else:
        raise ValueError(fault)
    t_fault = time.time()
    while time.time() - t_fault < down_s:
        sample()
        time.sleep(poll_s)
    if fault == "kill":
        cluster.restart(target)
    elif fault == "hang":
        cluster.signal(target, signal.SIGCONT)
    else:
        req = urllib.request.Request("http://%s/admin/fault" % cluster.node(target),
                                     data=json.dumps({"fail_rate": 0.0}).encode())
        urllib.request.urlopen(req, timeout=5).read()
    t_heal = time.time()
    while th.is_alive():
        sample()
        time.sleep(poll_s)
    th.join()
    # if the load finished before the healed worker saw traffic again, probe it through the gateway
    # with request ids the ring assigns to it (same FNV-1a ring as the gateway)
    probes = 0
    if cluster.breaker(target)["state"] != "CLOSED":
        sys.path.insert(0, REPO)
        import die_amd  # noqa: F401
        from die_amd import native

        ring = native.Ring()
        for i in range(len(cluster.ports)):
            ring.add(cluster.node(i))
        ids = [k for k in ("probe_%d" % j for j in range(5000)) if ring.get(k) == cluster.node(target)]
        deadline = time.time() + 10
        while time.time() < deadline and sample()["state"] != "CLOSED":
            body = json.dumps({"request_id": ids[probes % len(ids)], "input_data": [1.0, 2.0, 3.0]}).encode()
            try:
                urllib.request.urlopen(urllib.request.Request(cluster.url + "/infer", data=body), timeout=10).read()
            except Exception:
                pass
            probes += 1
            time.sleep(0.05)
    b = sample()
    st = cluster.stats()
    return {
        "fault": fault, "target": cluster.node(target), "down_s": down_s,
        "timeline": timeline, "breaker": b,
        "heal_to_closed_s": next((t for t, s in timeline if s == "CLOSED" and t > t_heal - t0), None),
        "probes_after_load": probes, "client": out.get("result"), "gateway": {k: st[k] for k in ("routed", "failovers", "failed") if k in st},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True)
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--fault", choices=["kill", "hang", "errors", "all"], default="all")
    ap.add_argument("--down-s", type=float, default=2.0)
    ap.add_argument("--requests", type=int, default=4000)
    ap.add_argument("--connections", type=int, default=8)
    ap.add_argument("--breaker-timeout-s", type=float, default=1.0)
    ap.add_argument("--input-numel", type=int, default=0, help="full unique payloads of this size (0 = reference 3-float)")
    ap.add_argument("--log-dir", default=None)
    a = ap.parse_args()
    faults = ["kill", "hang", "errors"] if a.fault == "all" else [a.fault]
    reports = []
    c = Cluster(a.model, a.workers, a.device, breaker_timeout_s=a.breaker_timeout_s, log_dir=a.log_dir)
    try:
        for f in faults:
            reports.append(drill(c, f, target=0, down_s=a.down_s, requests=a.requests, connections=a.connections,
                                 input_numel=a.input_numel))
            time.sleep(a.breaker_timeout_s + 0.5)
    finally:
        c.close()
    print(json.dumps(reports, indent=1))


if __name__ == "__main__":
    sys.exit(main())
