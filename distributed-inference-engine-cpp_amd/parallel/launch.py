"""Process-level helpers for the one-process-per-GPU layout.

The device-side data parallelism lives in C++ (csrc/parallel/dp_group.cpp: the shared-memory
control plane; csrc/parallel/communicator.cpp: RCCL over xGMI).  This module is the host side
around it:
  * rank_info()        RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE of a torchrun launch;
  * HostGroup          a gloo process group for host coordination (barriers, max/sum over ranks,
                       object exchange) -- bench.py times its steps between HostGroup barriers;
  * spawn_dp_worker()  one data-parallel worker over N GPUs (`worker_node --devices ...`: rank 0
                       spawns one process per further GPU, every rank ingests HTTP on the port);
  * spawn_gateway()    the gateway in front of a list of workers.
The reference runs every worker on GPU 0 through ORT (/root/reference/src/inference_engine.cpp:22-24)
and has no multi-GPU layer; these are the MI355X-side additions.
"""
from __future__ import annotations

import os
import subprocess
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(_PKG, "bin")


@dataclass
class RankInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    local_world: int = 1


def rank_info(env=None) -> RankInfo:
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    return RankInfo(rank=int(env.get("RANK", "0")), world=world, local_rank=int(env.get("LOCAL_RANK", "0")),
                    local_world=int(env.get("LOCAL_WORLD_SIZE", str(world))))


class HostGroup:
    """gloo group over the launch's ranks (a no-op group for world == 1).  Host coordination only:
    the GPU collectives of the DP engine run on its own RCCL communicator."""

    def __init__(self, info: Optional[RankInfo] = None):
        self.info = info or rank_info()
        self.dist = None
        if self.info.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.info.rank, world_size=self.info.world)
            self.dist = dist

    @property
    def rank(self) -> int:
        return self.info.rank

    @property
    def world(self) -> int:
        return self.info.world

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def reduce(self, values: Sequence[float], op: str = "max") -> List[float]:
        """Element-wise max or sum of `values` over all ranks (every rank gets the result)."""
        if self.dist is None:
            return [float(v) for v in values]
        import torch

        t = torch.tensor([float(v) for v in values], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(v) for v in t.tolist()]

    def all_gather_object(self, obj: Any) -> List[Any]:
        if self.dist is None:
            return [obj]
        out: List[Any] = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if self.dist is None:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def _bin(name: str) -> str:
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        raise FileNotFoundError("%s not built (run `make` in the repo root)" % path)
    return path


def spawn_dp_worker(model: str, port: int, devices: Sequence[int], node_id: str = "dp-worker",
                    max_batch: int = 256, extra_args: Sequence[str] = (), **popen_kw) -> subprocess.Popen:
    """`worker_node <port> <node_id> <model> --devices d0,d1,...`: one process per GPU; rank 0
    (on devices[0]) spawns the others before touching the GPU.  --max-batch is the whole DP batch
    (each rank's sub-batch is max_batch / len(devices))."""
    cmd = [_bin("worker_node"), str(port), node_id, model, "--devices", ",".join(str(d) for d in devices),
           "--max-batch", str(max_batch)] + list(extra_args)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.Popen(cmd, env=env, **popen_kw)


def spawn_gateway(workers: Sequence[str], port: int = 8000, extra_args: Sequence[str] = (),
                  **popen_kw) -> subprocess.Popen:
    """`gateway host:port ... --port P` in front of `workers` (consistent-hash routing, breakers)."""
    cmd = [_bin("gateway")] + list(workers) + ["--port", str(port)] + list(extra_args)
    return subprocess.Popen(cmd, **popen_kw)
