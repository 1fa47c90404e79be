"""Process-level fault drills (BASELINE config 3): real worker_node / gateway / loadgen binaries, one
worker killed, hung (SIGSTOP) or erroring while the load runs.  Asserts the reference's resilience
contract: no client-visible failure while another worker is healthy, the target's breaker goes
CLOSED -> OPEN -> HALF_OPEN -> CLOSED, and traffic returns to the healed worker."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.fixture(scope="module")
def cluster(models, tmp_path_factory):
    import fault_inject

    path = models["tiny"][0]
    c = fault_inject.Cluster(path, n_workers=3, device="cpu", breaker_timeout_s=1.0, read_timeout_ms=2000,
                             log_dir=str(tmp_path_factory.mktemp("fault_logs")), worker_threads=2)
    yield c
    c.close()


@pytest.mark.parametrize("fault", ["kill", "hang", "errors"])
def test_fault_drill(cluster, fault):
    import fault_inject

    before = cluster.breaker(0)
    rep = fault_inject.drill(cluster, fault, target=0, down_s=4.0 if fault == "hang" else 2.0, requests=3000,
                             connections=8, input_numel=3 * 64 * 64)
    assert rep["timeline"][0][1] == "CLOSED" and rep["client"]["wall_s"] > 1.0, rep  # fault hit a running load
    client = rep["client"]
    assert client["ok"] == 3000 and client["failed"] == 0, rep
    b = rep["breaker"]
    assert b["opened"] > before["opened"], rep
    assert b["half_opened"] > before["half_opened"] and b["closed"] > before["closed"], rep
    assert b["state"] == "CLOSED", rep
    assert rep["gateway"]["failovers"] > 0
    states = [s for _, s in rep["timeline"]]
    assert "OPEN" in states


def test_diagnostics_script(cluster):
    import subprocess

    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "diagnostics.sh")
    r = subprocess.run(["bash", script, str(cluster.gw_port), " ".join(str(p) for p in cluster.ports)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=120)
    out = r.stdout.decode()
    assert r.returncode == 0, out
    assert "0 failed" in out
