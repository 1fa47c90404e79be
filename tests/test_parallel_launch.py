"""die_amd.parallel.launch: rank parsing, the gloo HostGroup bench.py coordinates through (2 ranks
on the CPU), and the launcher command lines."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rank_info_parses_torchrun_env():
    sys.path.insert(0, ROOT)
    from die_amd.parallel.launch import rank_info

    r = rank_info({"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3", "LOCAL_WORLD_SIZE": "8"})
    assert (r.rank, r.world, r.local_rank, r.local_world) == (3, 8, 3, 8)
    r = rank_info({})
    assert (r.rank, r.world, r.local_rank, r.local_world) == (0, 1, 0, 1)


def test_host_group_single_rank_is_local():
    sys.path.insert(0, ROOT)
    from die_amd.parallel.launch import HostGroup, RankInfo

    g = HostGroup(RankInfo())
    g.barrier()
    assert g.reduce([1.5, 2.0], "max") == [1.5, 2.0]
    assert g.all_gather_object({"a": 1}) == [{"a": 1}]
    assert g.broadcast_object(7) == 7
    g.close()


def test_host_group_two_ranks_gloo():
    code = textwrap.dedent("""
        import json, sys
        sys.path.insert(0, %r)
        import torch  # noqa: F401
        from die_amd.parallel.launch import HostGroup
        g = HostGroup()
        r = g.rank
        g.barrier()
        mx = g.reduce([float(r), 10.0 * r], "max")
        sm = g.reduce([1.0, float(r)], "sum")
        ports = g.all_gather_object(9000 + r)
        b = g.broadcast_object("from%%d" %% r, src=0)
        g.close()
        print(json.dumps(dict(mx=mx, sm=sm, ports=ports, b=b)))
    """ % ROOT)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    import json

    outs = []
    for p in procs:
        o, e = p.communicate(timeout=180)
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for o in outs:
        assert o["mx"] == [1.0, 10.0]
        assert o["sm"] == [2.0, 1.0]
        assert o["ports"] == [9000, 9001]
        assert o["b"] == "from0"


def test_spawn_helpers_build_reference_cli(monkeypatch, tmp_path):
    sys.path.insert(0, ROOT)
    from die_amd.parallel import launch

    seen = {}

    class FakePopen:
        def __init__(self, cmd, **kw):
            seen["cmd"] = cmd
            seen["env"] = kw.get("env")

    monkeypatch.setattr(launch.subprocess, "Popen", FakePopen)
    monkeypatch.setattr(launch, "BIN", str(tmp_path))
    for name in ("worker_node", "gateway"):
        (tmp_path / name).write_text("")
    launch.spawn_dp_worker("m.onnx", 8001, [0, 1, 2, 3], max_batch=128, extra_args=["--precision", "fp32"])
    assert seen["cmd"][1:] == ["8001", "dp-worker", "m.onnx", "--devices", "0,1,2,3", "--max-batch", "128",
                               "--precision", "fp32"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    launch.spawn_gateway(["localhost:8001", "localhost:8002"], port=8000)
    assert seen["cmd"][1:] == ["localhost:8001", "localhost:8002", "--port", "8000"]
