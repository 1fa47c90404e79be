"""The event-driven load generator (LoadgenOptions::io_threads > 0: epoll loops instead of a thread
per connection) against a CPU worker: same closed-loop accounting as the threaded client, verify
mode and sampled verification checked answer by answer, a dead port counted as failures."""
import os
import tempfile

import numpy as np
import pytest


@pytest.fixture(scope="module")
def tiny_worker(native):
    from die_amd.models import resnet_v2 as r

    cfg = r.tiny_config()
    d = tempfile.mkdtemp()
    p = os.path.join(d, "t.onnx")
    open(p, "wb").write(r.build_onnx(cfg)[0])
    wk = native.Worker(p, node_id="lg", max_batch=8, cache_capacity=0, engine={"device": "cpu"})
    yield wk, p, cfg
    wk.stop()


@pytest.mark.parametrize("io_threads", [1, 3])
def test_async_full_payload(native, tiny_worker, io_threads):
    wk, p, cfg = tiny_worker
    numel = cfg.in_ch * cfg.image * cfg.image
    res = native.loadgen(port=wk.port, connections=12, requests=300, warmup=24, payload="full", input_numel=numel,
                         io_threads=io_threads)
    assert res["ok"] == 300 and res["failed"] == 0, res
    assert len(res["p99_by_tenth_ms"]) == 10 and len(res["slowest_ms"]) == 10


def test_async_verify_modes(native, tiny_worker):
    from die_amd.models import resnet_v2 as r

    wk, p, cfg = tiny_worker
    x = r.synthetic_input(4, cfg, seed=3).reshape(4, -1)
    ref = native.cpu_run(p, x.reshape(4, cfg.in_ch, cfg.image, cfg.image)).reshape(4, -1)
    res = native.loadgen(port=wk.port, connections=8, requests=160, verify_inputs=x, verify_expected=ref,
                         verify_tol=1e-5, io_threads=2)
    assert res["ok"] == 160 and res["verified"] == 160 and res["mismatched"] == 0 and res["bad_request_id"] == 0
    numel = cfg.in_ch * cfg.image * cfg.image
    res = native.loadgen(port=wk.port, connections=8, requests=200, payload="full", input_numel=numel,
                         verify_every=10, verify_inputs=x, verify_expected=ref, verify_tol=1e-5, io_threads=2,
                         scramble_ids=True)
    assert res["ok"] == 200 and res["verified"] == 20 and res["mismatched"] == 0 and res["bad_request_id"] == 0


def test_async_dead_port_fails_cleanly(native):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()  # nothing listens there
    res = native.loadgen(port=port, connections=4, requests=20, io_threads=2, timeout_ms=2000)
    assert res["ok"] == 0 and res["failed"] == 20
