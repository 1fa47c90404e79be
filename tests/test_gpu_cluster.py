"""BASELINE config 3 on the GPU: three HIP `worker_node` processes sharing GPU 0 (the reference's own
topology: every worker binds device 0, /root/reference/src/inference_engine.cpp:22-24)
behind the in-tree gateway, ResNet50-shaped 1 MB bodies.  A throughput run (no faults) records
gateway req/s and p50/p99; the kill / hang / errors drills must show zero client-visible failures
and the breaker cycle CLOSED -> OPEN -> HALF_OPEN -> CLOSED (/root/reference/src/gateway.cpp:80-128,
README.md:342-349)."""
import json
import os
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

NUMEL = 3 * 224 * 224


@pytest.fixture(scope="module")
def hip_cluster(models, tmp_path_factory):
    import fault_inject

    path = models["get_rn50"]()[0]
    logs = tmp_path_factory.mktemp("gpu_cluster_logs")
    # read timeout 2 s: a hung (SIGSTOPped) worker must fail requests well inside the drill window
    c = fault_inject.Cluster(path, n_workers=3, device="hip", breaker_timeout_s=1.0, read_timeout_ms=2000,
                             log_dir=str(logs), stagger=True)
    yield c
    c.close()


def test_gateway_throughput_three_hip_workers(hip_cluster):
    import fault_inject

    out = {}
    fault_inject.run_load(hip_cluster.gw_port, 6000, 48, out, input_numel=NUMEL)
    r = out["result"]
    assert r["ok"] == 6000 and r["failed"] == 0, r
    st = hip_cluster.stats()
    assert all(b["state"] == "CLOSED" for b in st["circuit_breakers"])
    rep = {"requests": r["requests"], "rps": r["rps"], "latency_ms": r["latency_ms"], "body_bytes": r["body_bytes"],
           "gateway": {k: st[k] for k in ("routed", "failovers", "failed")}}
    print("CONFIG3_THROUGHPUT " + json.dumps(rep))
    assert r["rps"] > 1000


@pytest.mark.parametrize("fault", ["kill", "hang", "errors"])
def test_fault_drill_hip_workers(hip_cluster, fault):
    import fault_inject

    before = hip_cluster.breaker(0)
    rep = fault_inject.drill(hip_cluster, fault, target=0, down_s=4.0 if fault == "hang" else 3.0, requests=24000,
                             connections=24, input_numel=NUMEL)
    print("CONFIG3_DRILL " + json.dumps({k: rep[k] for k in ("fault", "timeline", "heal_to_closed_s", "client",
                                                                "gateway")}))
    client = rep["client"]
    assert rep["timeline"][0][1] == "CLOSED" and client["wall_s"] > 1.0, rep
    assert client["ok"] == 24000 and client["failed"] == 0, rep
    b = rep["breaker"]
    assert b["opened"] > before["opened"] and b["half_opened"] > before["half_opened"], rep
    assert b["closed"] > before["closed"] and b["state"] == "CLOSED", rep
