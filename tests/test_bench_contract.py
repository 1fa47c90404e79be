"""bench.py driver contract rehearsed on the CPU: one JSON line on rank 0's stdout, whole-job
aggregate over ranks, N>1 through torch.distributed.run (gloo barriers, 127.0.0.1 rendezvous) --
the same launch line the driver uses for the 8-GPU scaling run, on the host executor."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, timeout=300):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout  # exactly one JSON line, nothing else on stdout
    return json.loads(lines[0])


def _check(out, n, steps, warmup, mode):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == warmup
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    names = {"gateway": "gateway+worker", "http": "worker"}
    assert out["config"]["parallelism"] == "dp%d" % n and out["config"]["mode"] == names.get(mode, mode)
    assert out["failed"] == 0 and out["value"] > 0
    # whole-job aggregate: every rank's requests are counted; a step is STEP_REQ requests per GPU
    assert out["config"]["requests"] == steps * STEP_REQ * n
    if mode == "gateway":
        assert out["gateway"]["failed"] == 0 and set(out["gateway"]["breakers"]) == {"CLOSED"}
        assert out["direct_worker"]["failed"] == 0
        assert out["cache_hits_timed"] == 0  # unique payloads per pass: every timed request was computed
        # BASELINE config 4 after the headline: one DP worker over all ranks, in watchdogged children
        dp = out["dp_rccl"]
        assert "error" not in dp, dp
        assert dp["dp_world"] == n and dp["failed"] == 0 and dp["requests_per_s"] > 0 and dp["dp_solo"] is False


STEP_REQ = 4
ARGS = ["--device", "cpu", "--batch", "2", "--steps", "2", "--warmup", "1", "--connections", "4",
        "--step-requests", str(STEP_REQ)]


@pytest.mark.parametrize("mode", ["gateway", "http", "dp"])
def test_bench_single_rank_cpu(mode):
    out = _run([sys.executable, "bench.py", "--mode", mode] + ARGS)
    _check(out, 1, 2, 1, mode)
    assert out["dtype"] == "fp32"


@pytest.mark.parametrize("mode", ["gateway", "dp"])
def test_bench_two_ranks_torchrun_cpu(mode):
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--mode", mode] + ARGS)
    _check(out, 2, 2, 1, mode)
    assert out["config"]["global_batch"] == 4
    # per-rank breakdown of the multi-GPU number (rank order, each rank's own throughput)
    pr = out["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert all(r["requests_per_s"] > 0 and r["failed"] == 0 for r in pr)


@pytest.mark.parametrize("mode", ["gateway", "dp"])
def test_bench_eight_ranks_torchrun_cpu(mode):
    """the driver's N=8 launch line rehearsed with 8 CPU ranks (gloo, a tiny
    ResNet-v2 so the CPU executor keeps up): gateway mode routes over all 8 workers on ring-balanced
    ports with sampled answer verification; dp mode runs ONE data-parallel worker over 8 ranks."""
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
                "--mode", mode, "--arch", "resnet_tiny", "--device", "cpu", "--batch", "4", "--steps", "2",
                "--warmup", "1", "--connections", "4", "--step-requests", "25", "--no-dp", "--verify-every", "10"],
               timeout=600)
    assert out["n_gpus"] == 8 and out["failed"] == 0 and out["value"] > 0
    assert out["config"]["requests"] == 2 * 25 * 8
    pr = out["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8)) and all(r["failed"] == 0 for r in pr)
    if mode == "dp":
        # per-rank dispatch fairness: the leader takes sub-batches oldest first
        # across ranks, so none waits more than two leader batches
        assert out["dp_max_sub_wait_batches"] is not None and out["dp_max_sub_wait_batches"] <= 2, out
    if mode == "gateway":
        v = out["verify"]
        assert v["verified"] == 8 * 5 and v["mismatched"] == 0 and v["bad_request_id"] == 0, v
        ring = out["ring"]
        # ports balance the ring's arcs (400 ids are too few to pin the routed shares themselves)
        assert ring["balanced_ports"] and len(set(ring["ports"])) == 8 and ring["arc_max_over_fair"] <= 1.1, ring
        assert abs(sum(r["worker_share"] for r in pr) - 1.0) < 1e-3
        assert out["gateway_bytes"]["failed"] == 0 and out["gateway_bytes"]["requests_per_s"] > 0


def test_bench_rejects_gpus_world_mismatch():
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
                        "--mode", "http"] + ARGS, cwd=REPO, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert p.returncode != 0 and "does not match WORLD_SIZE" in p.stderr
