"""HIP engine end to end on the GPU: whole-model numerics vs the C++ CPU executor and vs torch."""
import json
import time
import urllib.request

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12))


def test_hip_engine_tiny_vs_cpu(native, models):
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["tiny"]
    e = native.Engine(path, device="hip", max_batch=8)
    assert e.info["name"].startswith("hip:gfx950")
    x = r.synthetic_input(5, cfg)
    got = e.run(x.reshape(5, -1))
    ref = native.cpu_run(path, x)
    assert e.info["precision"] == "fp32"  # the default, like the reference's ORT session
    assert rel_l2(got, ref) < 1e-4, rel_l2(got, ref)
    assert (got.argmax(1) == ref.argmax(1)).all()
    # padding invariance: sample 0 alone (bucket 1) == sample 0 inside a batch of 5 (bucket 8); the
    # buckets may use different tuned split-K orders, so equal up to fp32 re-association
    one = e.run(x[:1].reshape(1, -1))
    assert float(np.linalg.norm(one[0] - got[0]) / np.linalg.norm(got[0])) < 1e-4
    e.close()


def test_hip_engine_resnet50_vs_torch(native, models):
    import torch

    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["get_rn50"]()
    e = native.Engine(path, device="hip", max_batch=32)
    info = e.refresh_info()
    assert info["hip_graphs"] is True
    x = r.synthetic_input(8, cfg)
    got = e.run(x.reshape(8, -1))
    with torch.no_grad():
        ref = r.torch_forward(w, x, cfg, device="cuda").cpu().numpy()
    err = rel_l2(got, ref)
    assert err < 1e-4, err
    assert (got.argmax(1) == ref.argmax(1)).all()
    # short input -> zero padded (reference semantics)
    short = e.run(np.array([[1.0, 2.0, 3.0]], np.float32))
    full = np.zeros((1, 3 * 224 * 224), np.float32)
    full[0, :3] = [1, 2, 3]
    np.testing.assert_allclose(short, e.run(full), rtol=0, atol=1e-5)
    e.close()


def test_worker_on_gpu_http(native, models):
    path, w, cfg = models["get_rn50"]()
    wk = native.Worker(path, node_id="gpu0", engine={"device": "hip"})
    try:
        res = native.loadgen(port=wk.port, connections=16, requests=256, warmup=32, payload="full",
                             input_numel=3 * 224 * 224)
        assert res["ok"] == 256, res
        h = wk.health()
        assert h["engine"]["name"].startswith("hip:")
        assert h["batch_processor"]["total_batches"] >= 1
        body = json.dumps({"request_id": "x1", "input_data": [0.5] * 100}).encode()
        req = urllib.request.Request(wk.url + "/infer", data=body, headers={"Content-Type": "application/json"})
        out = json.loads(urllib.request.urlopen(req, timeout=30).read())
        assert out["request_id"] == "x1" and len(out["output_data"]) == 1000 and out["cached"] is False
        out2 = json.loads(urllib.request.urlopen(req, timeout=30).read())
        assert out2["cached"] is True and out2["inference_time_us"] == 50
        assert out2["output_data"] == out["output_data"]
    finally:
        wk.stop()


def test_tune_cache_roundtrip(native, models, tmp_path):
    """Autotune results persist in the tuning file and are reused by the next engine."""
    import time

    path, w, cfg = models["tiny"]
    cache = str(tmp_path / "tune.json")
    t0 = time.time()
    e1 = native.Engine(path, device="hip", max_batch=8, tune_cache=cache)
    t1 = time.time()
    info1 = e1.refresh_info()
    e1.close()
    assert info1["tune_cache_entries_loaded"] == 0
    data = json.load(open(cache))
    assert any(k.startswith("gfx950") for k in data) and sum(len(v) for v in data.values()) > 0
    e2 = native.Engine(path, device="hip", max_batch=8, tune_cache=cache)
    t2 = time.time()
    info2 = e2.refresh_info()
    assert info2["tune_cache_entries_loaded"] > 0
    assert info2["tile_split_at_max_batch"] == info1["tile_split_at_max_batch"]
    x = np.random.default_rng(0).random((3, 3 * 64 * 64), dtype=np.float32)
    assert np.isfinite(e2.run(x)).all()
    e2.close()
    print("engine init with tuning %.2fs, from cache %.2fs" % (t1 - t0, time.time() - t2 + (t2 - t1)))


def test_tune_in_graph(native, models, tmp_path):
    """EngineOptions::tune_in_graph: each conv's isolated-launch front runners are re-timed in place
    inside eager forwards.  The engine reports what it timed, the outputs stay those of the
    untuned engine within the fp32 bar, and the in-place choices persist in the tuning file (a second
    engine with the same file re-times nothing)."""
    path, w, cfg = models["tiny"]
    cache = str(tmp_path / "tune.json")
    x = np.random.default_rng(1).random((5, 3 * 64 * 64), dtype=np.float32)
    ref = native.Engine(path, device="hip", max_batch=8, autotune=False, tune_cache="")
    want = ref.run(x)
    ref.close()
    e1 = native.Engine(path, device="hip", max_batch=8, tune_cache=cache, tune_in_graph=True)
    i1 = e1.refresh_info()
    assert i1["options"]["tune_in_graph"] is True
    assert i1["tune_in_graph_timed"] > 0 and 0 <= i1["tune_in_graph_changed"] <= i1["tune_in_graph_timed"]
    got = e1.run(x)
    e1.close()
    assert np.linalg.norm(got - want) / np.linalg.norm(want) < 1e-5
    data = json.load(open(cache))
    assert any(k.startswith("g") for v in data.values() for k in v)
    e2 = native.Engine(path, device="hip", max_batch=8, tune_cache=cache, tune_in_graph=True)
    i2 = e2.refresh_info()
    assert i2["tune_in_graph_timed"] == 0 and i2["tile_split_at_max_batch"] == i1["tile_split_at_max_batch"]
    e2.close()


def test_efficient_batch_curve(native, models):
    """EngineOptions::efficient_batch: the engine times its captured forward at every batch size at
    start-up and preferred_batch(Q) is the largest B <= Q within efficient_batch_tol of the best
    per-image time over 1..Q; a batch it cuts back still runs correctly at that size.  Off: no curve
    and every queue is taken whole.  (Any-size cuts, efficient_batch_ends off: the default bucket-end
    rule has its own test, tests/test_engine_options.py::test_efficient_batch_bucket_ends.)"""
    path, w, cfg = models["tiny"]
    tol = 0.03
    e = native.Engine(path, device="hip", max_batch=16, autotune=False, tune_cache="", efficient_batch_tol=tol,
                      efficient_batch_ends=False)
    info = e.refresh_info()
    curve = info["batch_curve_ms"]
    assert info["efficient_batch"] is True and len(curve) == 16 and all(c > 0 for c in curve)
    per = [c / (b + 1) for b, c in enumerate(curve)]
    for q in range(1, 17):
        b = e.preferred_batch(q)
        assert 1 <= b <= q
        assert per[b - 1] <= min(per[:q]) * (1 + tol) + 1e-9
        assert all(per[c - 1] > min(per[:q]) * (1 + tol) for c in range(b + 1, q + 1))
    assert e.preferred_batch(40) <= 16
    x = np.random.default_rng(2).random((16, 3 * 64 * 64), dtype=np.float32)
    full = e.run(x)
    b = e.preferred_batch(16)
    part = e.run(x[:b])  # another bucket's graph: its own tile configs, so fp32-close rather than bitwise
    assert np.linalg.norm(part - full[:b]) / np.linalg.norm(full[:b]) < 1e-5
    e.close()
    off = native.Engine(path, device="hip", max_batch=16, autotune=False, tune_cache="", efficient_batch=False)
    assert off.refresh_info()["efficient_batch"] is False and "batch_curve_ms" not in off.refresh_info()
    assert [off.preferred_batch(q) for q in (1, 7, 16)] == [1, 7, 16]
    off.close()


@pytest.mark.parametrize("graphs", [True, False])
def test_branch_streams_bit_identical(native, models, graphs):
    """Projection shortcuts on the side stream (hipGraph branches, or eager fork/join events) give
    exactly the outputs of the in-line schedule (same heuristic kernel configs, no autotune), at
    several buckets and across repeated runs (race screen)."""
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["get_rn50"]()
    base = dict(device="hip", max_batch=32, use_graphs=graphs, autotune=False, tune_cache="")
    a = native.Engine(path, branch_streams=True, **base)
    b = native.Engine(path, branch_streams=False, **base)
    assert a.refresh_info()["branch_streams"] is True and b.refresh_info()["branch_streams"] is False
    for B in (1, 7, 24, 32):
        x = r.synthetic_input(B, cfg, seed=B).reshape(B, -1)
        ya = a.run(x)
        for _ in range(3):
            np.testing.assert_array_equal(ya, a.run(x))
        np.testing.assert_array_equal(ya, b.run(x))
    a.close()
    b.close()


@pytest.mark.parametrize("arch", ["resnet", "vit"])
def test_live_batch_skips_padding_exactly(native, models, arch):
    """A batch runs its bucket's graph; with live_batch the kernels skip the padding samples.  The
    real rows must be bit-identical to computing the whole bucket (same kernel configs)."""
    if arch == "resnet":
        from die_amd.models import resnet_v2 as r

        path, w, cfg = models["get_rn50"]()
    else:
        from die_amd.models import vit as r

        path, w, cfg = models["get_vit"]("tiny")
    base = dict(device="hip", max_batch=32, autotune=False, tune_cache="")
    a = native.Engine(path, live_batch=True, **base)
    b = native.Engine(path, live_batch=False, **base)
    assert a.refresh_info()["live_batch"] is True and b.refresh_info()["live_batch"] is False
    for B in (3, 5, 13, 17, 23, 29, 32):
        x = r.synthetic_input(B, cfg, seed=100 + B).reshape(B, -1)
        ya = a.run(x)
        np.testing.assert_array_equal(ya, b.run(x))
        assert np.isfinite(ya).all()
    a.close()
    b.close()
