"""ctypes bindings to the native runtime (`lib/libdie.so`, built by `make` / `__graft_entry__.build`).

Everything performance-relevant runs in C++/HIP; Python only configures and observes it.  Objects
wrap opaque handles; options travel as JSON.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import LIB_DIR

_LIB: Optional[C.CDLL] = None


class NativeError(RuntimeError):
    pass


_READY_CB = C.CFUNCTYPE(None, C.c_void_p)  # loadgen on_ready hook (LoadgenOptions::on_ready)


def lib_path() -> str:
    # DIE_LIB_PATH: another build of the library (same-box A/B measurements, tools/ab_ops.sh)
    return os.environ.get("DIE_LIB_PATH") or os.path.join(LIB_DIR, "libdie.so")


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path):
            raise NativeError("native library missing: %s (run `make -j8` or __graft_entry__.build())" % path)
        # torch wheels bundle their own libamdhip64.so (SONAME libamdhip64.so.7, same as /opt/rocm's).
        # If torch is loaded first, libdie.so's NEEDED libamdhip64.so.7 resolves to torch's copy and
        # the process has ONE HIP runtime; loading libdie.so first and torch later would map a second
        # runtime (torch NEEDs the unversioned name).  So bring torch in first whenever it exists.
        if os.environ.get("DIE_NO_TORCH") != "1":
            try:
                import torch  # noqa: F401
            except Exception:
                pass
        L = C.CDLL(path)
        vp, cp, i64p, f32p = C.c_void_p, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_float)
        errp = C.POINTER(C.c_void_p)

        def sig(name, res, *args):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = list(args)

        sig("die_free", None, vp)
        sig("die_version", cp)
        sig("die_json_roundtrip", vp, cp, errp)
        sig("die_parse_infer", C.c_long, cp, C.c_long, f32p, C.c_long, errp, errp)
        sig("die_format_floats", vp, f32p, C.c_long)
        sig("die_fnv1a", C.c_uint32, cp)
        sig("die_pick_efficient_batch", C.c_int, C.POINTER(C.c_double), C.c_int, C.c_int, C.c_double, C.c_double,
            C.POINTER(C.c_int), C.c_int)
        sig("die_ring_create", vp, C.c_int)
        sig("die_ring_destroy", None, vp)
        sig("die_ring_add", None, vp, cp)
        sig("die_ring_remove", None, vp, cp)
        sig("die_ring_get", vp, vp, cp)
        sig("die_ring_nodes", vp, vp)
        sig("die_ring_size", C.c_long, vp)
        sig("die_breaker_create", vp, C.c_int, C.c_int, C.c_long)
        sig("die_breaker_destroy", None, vp)
        sig("die_breaker_advance", None, vp, C.c_long)
        sig("die_breaker_allow", C.c_int, vp)
        sig("die_breaker_success", None, vp)
        sig("die_breaker_failure", None, vp)
        sig("die_breaker_state", vp, vp)
        sig("die_cache_create", vp, C.c_long)
        sig("die_cache_destroy", None, vp)
        sig("die_cache_put", None, vp, f32p, C.c_long, f32p, C.c_long)
        sig("die_cache_get", C.c_long, vp, f32p, C.c_long, f32p, C.c_long)
        sig("die_cache_stats", vp, vp)
        sig("die_batcher_create", vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int)
        sig("die_batcher_process", C.c_int, vp, C.c_int, errp)
        sig("die_batcher_metrics", vp, vp)
        sig("die_batcher_stop", None, vp)
        sig("die_batcher_destroy", None, vp)
        sig("die_engine_create", vp, cp, cp, errp)
        sig("die_engine_destroy", None, vp)
        sig("die_engine_info", vp, vp)
        sig("die_engine_run", C.c_int, vp, f32p, C.c_long, C.c_long, f32p, errp)
        sig("die_engine_run_text", C.c_int, vp, C.c_char_p, i64p, C.c_long, f32p, C.POINTER(C.c_int), C.c_int, errp)
        sig("die_pack_nibbles", C.c_int, C.c_char_p, C.c_longlong, C.c_char_p)
        sig("die_unpack_nibbles", None, C.c_char_p, C.c_longlong, C.c_char_p)
        sig("die_engine_text_packing", C.c_int, vp)
        sig("die_engine_preferred_batch", C.c_int, vp, C.c_int)
        sig("die_engine_profile", vp, vp, C.c_int, C.c_int)
        sig("die_dp_follower_start", vp, cp, errp)
        sig("die_dp_follower_status", vp, vp)
        sig("die_dp_follower_join", C.c_long, vp, C.c_int)
        sig("die_cpu_run", vp, cp, f32p, i64p, C.c_int, i64p, C.POINTER(C.c_int), errp)
        sig("die_onnx_summary", vp, cp, errp)
        sig("die_worker_create", vp, cp, errp)
        sig("die_worker_port", C.c_int, vp)
        sig("die_worker_health", vp, vp)
        sig("die_worker_stop", None, vp)
        sig("die_worker_destroy", None, vp)
        sig("die_gateway_create", vp, cp, errp)
        sig("die_gateway_port", C.c_int, vp)
        sig("die_gateway_stats", vp, vp)
        sig("die_gateway_stop", None, vp)
        sig("die_gateway_destroy", None, vp)
        sig("die_loadgen_run", vp, cp, errp)
        sig("die_loadgen_run_verify", vp, cp, f32p, C.c_long, f32p, C.c_long, errp)
        sig("die_loadgen_run_cb", vp, cp, f32p, C.c_long, f32p, C.c_long, _READY_CB, errp)
        sig("die_parse_bench", C.c_double, cp, C.c_long, C.c_int, C.c_int)
        i32p = C.POINTER(C.c_int)
        sig("die_dp_shard", C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p)
        sig("die_dp_per", C.c_int, C.c_int, C.c_int)
        sig("die_dp_items_from_gathered", None, C.c_int, C.c_int, C.c_int, i32p, C.c_long, i32p)
        sig("die_dp_rows_from_gathered", None, C.c_int, C.c_int, C.c_int, f32p, C.c_long, C.c_long, f32p)
        sig("die_dp_item_ok", None, C.c_int, C.c_int, C.c_int, i32p, C.POINTER(C.c_ubyte))
        _LIB = L
    return _LIB


def _take_str(p) -> str:
    if not p:
        return ""
    s = C.cast(p, C.c_char_p).value.decode("utf-8", "replace")
    lib().die_free(p)
    return s


def _err_box():
    return C.c_void_p(None)


def _raise_if(err, what: str):
    if err.value:
        raise NativeError("%s: %s" % (what, _take_str(err.value)))
    raise NativeError(what)


def _f32(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


# ---- JSON / parsing -------------------------------------------------------------------------------

def json_roundtrip(text: str) -> str:
    err = _err_box()
    p = lib().die_json_roundtrip(text.encode(), C.byref(err))
    if not p:
        _raise_if(err, "json")
    return _take_str(p)


def parse_infer(body: bytes, cap: int) -> Tuple[str, np.ndarray, int]:
    out = np.zeros(cap, np.float32)
    err, idp = _err_box(), C.c_void_p(None)
    n = lib().die_parse_infer(body, len(body), _f32(out), cap, C.byref(idp), C.byref(err))
    if n < 0:
        _raise_if(err, "parse_infer")
    return _take_str(idp.value), out[: min(n, cap)], n


def parse_bench(body: bytes, iters: int = 20, simd: bool = True) -> float:
    """Average microseconds to parse `body` as an /infer request (host parser benchmark)."""
    return lib().die_parse_bench(body, len(body), iters, int(simd))


def format_floats(v: np.ndarray) -> str:
    v = np.ascontiguousarray(v, np.float32)
    return _take_str(lib().die_format_floats(_f32(v), v.size))


# ---- control plane ------------------------------------------------------------------------------

def _cpulist(text: str) -> List[int]:
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def _cgroup_quota() -> Optional[float]:
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        return None


def bind_local_cpus(device: int = 0, ranks_per_node: int = 1) -> Dict[str, Any]:
    """NUMA placement for one-process-per-GPU serving: restrict this process (and every thread it
    creates afterwards: HTTP reactors, batcher, completion, client) to the CPUs local to its GPU's
    PCIe root (sysfs local_cpulist), so request bodies, pinned staging and DMA stay on the GPU's
    socket, and set DIE_CPUS to this rank's share of the node's CPU budget for thread-pool sizing.
    Needs torch (device -> PCI address); a no-op where sysfs does not say."""
    info: Dict[str, Any] = {"bound": False}
    cur = sorted(os.sched_getaffinity(0))
    quota = _cgroup_quota()
    budget = min(len(cur), int(quota)) if quota else len(cur)
    share = max(4, budget // max(1, ranks_per_node))
    os.environ["DIE_CPUS"] = str(share)
    info["cpu_share"] = share
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        local = _cpulist(open("/sys/bus/pci/devices/%s/local_cpulist" % bdf).read())
    except Exception as e:  # no torch/sysfs: keep the inherited mask
        info["reason"] = str(e)
        return info
    cpus = sorted(set(local) & set(cur))
    info["pci"] = bdf
    if len(cpus) < 8 or len(cpus) == len(cur):
        info["reason"] = "local set %d of %d CPUs" % (len(cpus), len(cur))
        return info
    os.sched_setaffinity(0, cpus)
    info.update(bound=True, cpus=len(cpus))
    return info


def pack_nibbles(text: bytes) -> Optional[bytes]:
    """4-bit packing of number-list text (core/textpack.h); None if a byte is outside the alphabet."""
    dst = C.create_string_buffer((len(text) + 1) // 2 + 1)
    if not lib().die_pack_nibbles(text, len(text), dst):
        return None
    return dst.raw[: (len(text) + 1) // 2]


def unpack_nibbles(packed: bytes, n: int) -> bytes:
    dst = C.create_string_buffer(n + 1)
    lib().die_unpack_nibbles(packed, n, dst)
    return dst.raw[:n]


def pick_efficient_batch(curve_ms, queued: int, tol: float = 0.0, margin: float = 0.02, ends=None) -> int:
    """EngineOptions::efficient_batch policy over a forward-time curve (ms at batch 1, 2, ...);
    ends: the engine's bucket sizes (only they are cut targets)."""
    arr = (C.c_double * (len(curve_ms) + 1))(0.0, *curve_ms)
    e = (C.c_int * len(ends))(*ends) if ends else None
    return lib().die_pick_efficient_batch(arr, len(curve_ms), int(queued), float(tol), float(margin), e,
                                          len(ends) if ends else 0)


def fnv1a(s: str) -> int:
    return lib().die_fnv1a(s.encode())


class Ring:
    def __init__(self, vnodes: int = 150):
        self.h = lib().die_ring_create(vnodes)

    def add(self, n: str):
        lib().die_ring_add(self.h, n.encode())

    def remove(self, n: str):
        lib().die_ring_remove(self.h, n.encode())

    def get(self, k: str) -> str:
        return _take_str(lib().die_ring_get(self.h, k.encode()))

    def nodes(self) -> List[str]:
        return json.loads(_take_str(lib().die_ring_nodes(self.h)))

    def __len__(self):
        return lib().die_ring_size(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().die_ring_destroy(self.h)
            self.h = None


class Breaker:
    """Circuit breaker driven by a fake clock (advance(ms))."""

    def __init__(self, failure_threshold=5, success_threshold=2, timeout_ms=30000):
        self.h = lib().die_breaker_create(failure_threshold, success_threshold, timeout_ms)

    def allow(self) -> bool:
        return bool(lib().die_breaker_allow(self.h))

    def success(self):
        lib().die_breaker_success(self.h)

    def failure(self):
        lib().die_breaker_failure(self.h)

    def advance(self, ms: int):
        lib().die_breaker_advance(self.h, ms)

    def state(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_breaker_state(self.h)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().die_breaker_destroy(self.h)
            self.h = None


class Cache:
    def __init__(self, capacity: int):
        self.h = lib().die_cache_create(capacity)

    def put(self, key: np.ndarray, value: np.ndarray):
        k = np.ascontiguousarray(key, np.float32)
        v = np.ascontiguousarray(value, np.float32)
        lib().die_cache_put(self.h, _f32(k), k.size, _f32(v), v.size)

    def get(self, key: np.ndarray, cap: int = 4096) -> Optional[np.ndarray]:
        k = np.ascontiguousarray(key, np.float32)
        out = np.zeros(cap, np.float32)
        n = lib().die_cache_get(self.h, _f32(k), k.size, _f32(out), cap)
        return None if n < 0 else out[:n]

    def stats(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_cache_stats(self.h)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().die_cache_destroy(self.h)
            self.h = None


class TestBatcher:
    """BatchProcessor<int,int> doubling each request (unit tests)."""

    def __init__(self, max_batch: int, timeout_ms: int, deadline: bool = False, delay_ms: int = 0, size_cap: int = 0,
                 balance: bool = False):
        """size_cap > 0: a batch-size hook (as Engine::preferred_batch) that takes at most size_cap;
        balance: WorkerOptions::batch_balance."""
        self.h = lib().die_batcher_create(max_batch, timeout_ms, int(deadline), delay_ms, size_cap, int(balance))

    def process(self, v: int) -> int:
        err = _err_box()
        r = lib().die_batcher_process(self.h, v, C.byref(err))
        if err.value:
            raise NativeError(_take_str(err.value))
        return r

    def metrics(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_batcher_metrics(self.h)))

    def stop(self):
        lib().die_batcher_stop(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().die_batcher_destroy(self.h)
            self.h = None


# ---- engines ----------------------------------------------------------------------------------------

def engine_options(opts: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """EngineOptions as JSON (csrc/engine/engine.h).  tune_cache "auto" (the default) resolves here:
    $DIE_TUNE_CACHE, else the native default (~/.cache/die_amd/tune.json)."""
    o = dict(opts or {})
    if o.get("tune_cache", "auto") == "auto" and os.environ.get("DIE_TUNE_CACHE"):
        o["tune_cache"] = os.environ["DIE_TUNE_CACHE"]
    return o


class Engine:
    def __init__(self, model_path: str, **opts):
        err = _err_box()
        opts = engine_options(opts)
        self.h = lib().die_engine_create(model_path.encode(), json.dumps(opts).encode(), C.byref(err))
        if not self.h:
            _raise_if(err, "engine")
        self.info = json.loads(_take_str(lib().die_engine_info(self.h)))

    def refresh_info(self) -> Dict[str, Any]:
        self.info = json.loads(_take_str(lib().die_engine_info(self.h)))
        return self.info

    @property
    def input_numel(self) -> int:
        return int(np.prod(self.info["input_shape"]))

    @property
    def output_numel(self) -> int:
        return int(np.prod(self.info["output_shape"]))

    def run(self, x: np.ndarray) -> np.ndarray:
        """x: [B, L] (L <= input numel, zero-padded) -> [B, output numel]."""
        x = np.ascontiguousarray(x, np.float32)
        B = x.shape[0]
        L = int(np.prod(x.shape[1:]))
        out = np.zeros((B, self.output_numel), np.float32)
        err = _err_box()
        if lib().die_engine_run(self.h, _f32(x), B, L, _f32(out), C.byref(err)) != 0:
            _raise_if(err, "engine run")
        return out

    def profile(self, batch: int = 32, iters: int = 10) -> Dict[str, Any]:
        """Per-op device time (µs) of one forward at `batch` (HIP engine; {} for the CPU engine)."""
        return json.loads(_take_str(lib().die_engine_profile(self.h, batch, iters)))

    def preferred_batch(self, queued: int) -> int:
        """Batch size the worker dispatches with `queued` requests waiting (EngineOptions::efficient_batch)."""
        return int(lib().die_engine_preferred_batch(self.h, int(queued)))

    @property
    def text_packing(self) -> bool:
        """True when the engine takes 4-bit packed input text (half the H2D bytes)."""
        return bool(lib().die_engine_text_packing(self.h))

    def run_text(self, texts, pack: bool = False):
        """Device-decode path: `texts` are input_data number lists (bytes, without brackets).
        pack=True uploads them 4-bit packed (as the worker does) when the engine supports it.
        Returns (outputs [B, output numel], status [B]); status 0 = ok, bit 0 = needs the host
        parser, 2 = more values than the model input."""
        B = len(texts)
        blob = b"".join(texts)
        lens = np.array([len(t) for t in texts], np.int64)
        out = np.zeros((B, self.output_numel), np.float32)
        status = np.zeros(B, np.int32)
        err = _err_box()
        rc = lib().die_engine_run_text(self.h, blob, lens.ctypes.data_as(C.POINTER(C.c_int64)), B, _f32(out),
                                       status.ctypes.data_as(C.POINTER(C.c_int)), int(pack), C.byref(err))
        if rc != 0:
            _raise_if(err, "engine run_text")
        return out, status

    def close(self):
        if getattr(self, "h", None):
            lib().die_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cpu_run(model_path: str, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    shape = (C.c_int64 * x.ndim)(*x.shape)
    out_shape = (C.c_int64 * 8)()
    out_rank = C.c_int(0)
    err = _err_box()
    p = lib().die_cpu_run(model_path.encode(), _f32(x), shape, x.ndim, out_shape, C.byref(out_rank), C.byref(err))
    if not p:
        _raise_if(err, "cpu_run")
    shp = tuple(out_shape[i] for i in range(out_rank.value))
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(int(np.prod(shp)),)).copy()
    lib().die_free(p)
    return arr.reshape(shp)


def cpu_run_value(model_path: str, x: np.ndarray, name: str) -> np.ndarray:
    """Intermediate value `name` of a CPU-executor run (debugging / per-op parity tests)."""
    L = lib()
    fn = L.die_cpu_run_value
    fn.restype = C.c_void_p
    fn.argtypes = [C.c_char_p, C.POINTER(C.c_float), C.POINTER(C.c_int64), C.c_int, C.c_char_p,
                   C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_void_p)]
    x = np.ascontiguousarray(x, np.float32)
    shape = (C.c_int64 * x.ndim)(*x.shape)
    out_shape = (C.c_int64 * 8)()
    out_rank = C.c_int(0)
    err = _err_box()
    p = fn(model_path.encode(), _f32(x), shape, x.ndim, name.encode(), out_shape, C.byref(out_rank), C.byref(err))
    if not p:
        _raise_if(err, "cpu_run_value")
    shp = tuple(out_shape[i] for i in range(out_rank.value))
    n = int(np.prod(shp)) if shp else 1
    arr = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n,)).copy()
    L.die_free(p)
    return arr.reshape(shp)


def onnx_summary(model_path: str) -> Dict[str, Any]:
    err = _err_box()
    p = lib().die_onnx_summary(model_path.encode(), C.byref(err))
    if not p:
        _raise_if(err, "onnx_summary")
    return json.loads(_take_str(p))


# ---- servers ------------------------------------------------------------------------------------------

def dp_arena_plan(input_numel: int, world: int, **engine_opts) -> Dict[str, int]:
    """Size of a data-parallel group's shared input arena (engine/dp_engine.cpp dp_arena_plan):
    {item_bytes, items, bytes}; engine_opts as for Engine (max_batch = the whole DP batch)."""
    L = lib()
    fn = L.die_dp_arena_plan
    fn.restype = C.c_int
    fn.argtypes = [C.c_longlong, C.c_char_p, C.c_int, C.POINTER(C.c_longlong)]
    out = (C.c_longlong * 3)()
    if fn(int(input_numel), json.dumps(engine_opts).encode(), int(world), out) != 0:
        raise NativeError("dp_arena_plan failed")
    return {"item_bytes": out[0], "items": out[1], "bytes": out[2]}


class DpLayout:
    """Row bookkeeping of one data-parallel batch (csrc/parallel/dp_layout.h): B items over `world`
    ranks, `per` items per rank (default ceil(B / world)); rank r computes [r*per, min(B, (r+1)*per))."""

    def __init__(self, B: int, world: int, per: int = 0):
        self.B, self.world = B, world
        self.per = per if per > 0 else lib().die_dp_per(B, world)

    def shard(self, r: int) -> Tuple[int, int]:
        begin = C.c_int(0)
        n = lib().die_dp_shard(self.B, self.world, self.per, r, C.byref(begin))
        return begin.value, n

    def items_from_gathered(self, gathered: np.ndarray, stride: int) -> np.ndarray:
        g = np.ascontiguousarray(gathered, np.int32)
        assert g.size >= self.world * stride
        out = np.zeros(self.B, np.int32)
        ip = C.POINTER(C.c_int)
        lib().die_dp_items_from_gathered(self.B, self.world, self.per, g.ctypes.data_as(ip), stride,
                                         out.ctypes.data_as(ip))
        return out

    def rows_from_gathered(self, gathered: np.ndarray, rows_per_rank: int) -> np.ndarray:
        g = np.ascontiguousarray(gathered, np.float32)
        row_len = g.shape[-1]
        assert g.reshape(-1, row_len).shape[0] >= self.world * rows_per_rank
        out = np.zeros((self.B, row_len), np.float32)
        lib().die_dp_rows_from_gathered(self.B, self.world, self.per, _f32(g), rows_per_rank, row_len, _f32(out))
        return out

    def item_ok(self, rank_ok) -> np.ndarray:
        r = np.ascontiguousarray(rank_ok, np.int32)
        assert r.size == self.world
        out = np.zeros(self.B, np.uint8)
        lib().die_dp_item_ok(self.B, self.world, self.per, r.ctypes.data_as(C.POINTER(C.c_int)),
                             out.ctypes.data_as(C.POINTER(C.c_ubyte)))
        return out.astype(bool)


class DpFollower:
    """Data-parallel follower rank (csrc/engine/dp_engine.cpp): attaches to the leader's DpGroup
    `group`, builds its local engine (RCCL communicator for HIP, host communicator for CPU) and
    serves its shard of every batch on a background native thread."""

    def __init__(self, model_path: str, group: str, rank: int, world: int, max_batch: int = 32, **engine):
        eng = engine_options(engine)
        eng.update(dp_group=group, dp_rank=rank, dp_world=world)
        o = dict(model_path=model_path, max_batch=max_batch, engine=eng)
        err = _err_box()
        self.h = lib().die_dp_follower_start(json.dumps(o).encode(), C.byref(err))
        if not self.h:
            _raise_if(err, "dp follower")

    def status(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_dp_follower_status(self.h)))

    def join(self, stop: bool = False) -> int:
        """Wait for the follower to finish (the leader stops the group), or stop it; returns batches served."""
        if not self.h:
            return 0
        n = lib().die_dp_follower_join(self.h, int(stop))
        self.h = None
        return n


class Worker:
    """In-process worker node (HTTP on 127.0.0.1:<port>, port 0 = ephemeral)."""

    def __init__(self, model_path: str, node_id: str = "w1", port: int = 0, **opts):
        o = dict(opts)
        o.update(model_path=model_path, node_id=node_id, port=port, engine=engine_options(opts.get("engine")))
        err = _err_box()
        self.h = lib().die_worker_create(json.dumps(o).encode(), C.byref(err))
        if not self.h:
            _raise_if(err, "worker")
        self.port = lib().die_worker_port(self.h)
        self.url = "http://127.0.0.1:%d" % self.port

    def health(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_worker_health(self.h)))

    def stop(self):
        if getattr(self, "h", None):
            lib().die_worker_stop(self.h)
            lib().die_worker_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


class GatewayServer:
    def __init__(self, workers: Sequence[str], port: int = 0, **opts):
        o = dict(opts)
        o.update(workers=list(workers), port=port)
        err = _err_box()
        self.h = lib().die_gateway_create(json.dumps(o).encode(), C.byref(err))
        if not self.h:
            _raise_if(err, "gateway")
        self.port = lib().die_gateway_port(self.h)
        self.url = "http://127.0.0.1:%d" % self.port

    def stats(self) -> Dict[str, Any]:
        return json.loads(_take_str(lib().die_gateway_stats(self.h)))

    def stop(self):
        if getattr(self, "h", None):
            lib().die_gateway_stop(self.h)
            lib().die_gateway_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass


def loadgen(verify_inputs: Optional[np.ndarray] = None, verify_expected: Optional[np.ndarray] = None,
            on_ready: Optional[Callable[[], None]] = None, **opts) -> Dict[str, Any]:
    """Closed-loop C++ load generator.  With verify_inputs ([K, input_numel]) and verify_expected
    ([K, output_numel]) every request carries one of the K inputs (unique request_id) and every answer
    is checked against its expected row (relative L2 <= verify_tol, 0 = bit-exact): the result adds
    "verified", "mismatched", "bad_request_id" and "max_rel_err".  With payload="full" and
    verify_every=N only every N-th request is such a verified one (zero-padded text: never a cache
    hit); scramble_ids=True prints request numbers scrambled (hash-uniform on the gateway ring);
    io_threads=N > 0 drives the connections from N epoll threads instead of one thread each.
    on_ready() runs once, on this thread, after every connection's payloads are built and the warm-up
    is done, right before the timed phase (the place for a timing barrier)."""
    err = _err_box()
    if on_ready is not None:
        def _cb(_arg):
            on_ready()
        cb = _READY_CB(_cb)  # kept alive for the duration of the call
        xi = xe = None
        k = n_out = 0
        if verify_inputs is not None:
            xi = np.ascontiguousarray(verify_inputs, np.float32).reshape(len(verify_inputs), -1)
            xe = np.ascontiguousarray(verify_expected, np.float32).reshape(len(xi), -1)
            opts = dict(opts, input_numel=xi.shape[1])
            k, n_out = len(xi), xe.shape[1]
        p = lib().die_loadgen_run_cb(json.dumps(opts).encode(), _f32(xi) if xi is not None else None, k,
                                     _f32(xe) if xe is not None else None, n_out, cb, C.byref(err))
        if not p:
            _raise_if(err, "loadgen")
        return json.loads(_take_str(p))
    if verify_inputs is not None:
        xi = np.ascontiguousarray(verify_inputs, np.float32).reshape(len(verify_inputs), -1)
        xe = np.ascontiguousarray(verify_expected, np.float32).reshape(len(xi), -1)
        opts = dict(opts, input_numel=xi.shape[1])
        p = lib().die_loadgen_run_verify(json.dumps(opts).encode(), _f32(xi), len(xi), _f32(xe), xe.shape[1],
                                         C.byref(err))
    else:
        p = lib().die_loadgen_run(json.dumps(opts).encode(), C.byref(err))
    if not p:
        _raise_if(err, "loadgen")
    return json.loads(_take_str(p))


# ---- plan / kernels ---------------------------------------------------------------------------------

def _sig_kernels():
    L = lib()
    if getattr(L, "_kern_sigs", False):
        return L
    u64, i = C.c_uint64, C.c_int
    L.die_plan_summary.restype = C.c_void_p
    L.die_plan_summary.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.die_kern_conv.restype = i
    L.die_kern_conv.argtypes = [C.c_char_p] + [u64] * 9 + [i, u64]
    L.die_kern_input_prep.restype = i
    L.die_kern_conv_pair.restype = i
    L.die_kern_conv_pair.argtypes = [C.c_char_p] + [u64] * 11
    L.die_pair_permute_row.restype = i
    L.die_pair_permute_row.argtypes = [i]
    L.die_kern_input_prep.argtypes = [u64] * 4 + [i] * 5 + [u64, i]
    L.die_kern_pool2d.restype = i
    L.die_kern_pool2d.argtypes = [u64, u64] + [i] * 14 + [u64, i]
    L.die_kern_gap.restype = i
    L.die_kern_gap.argtypes = [u64] * 5 + [i] * 4 + [u64, i]
    L.die_kern_affine.restype = i
    L.die_kern_affine.argtypes = [u64] * 4 + [i, u64, C.c_longlong, i, u64, i]
    L.die_kern_nhwc_to_nchw.restype = i
    L.die_kern_nhwc_to_nchw.argtypes = [u64, u64] + [i] * 4 + [u64, i]
    L.die_kern_stem.restype = i
    L.die_kern_stem.argtypes = [u64] * 4 + [i] * 6 + [u64, i]
    L.die_kern_stem_nchw.restype = i
    L.die_kern_stem_nchw.argtypes = [u64, i] + [u64] * 5 + [i] * 6 + [u64, i, i]
    L.die_kern_gconv.restype = i
    L.die_kern_gconv.argtypes = [C.c_char_p] + [u64] * 5
    L.die_kern_softmax.restype = i
    L.die_kern_softmax.argtypes = [u64, u64, u64, C.c_longlong, i, u64, i]
    L.die_kern_layernorm.restype = i
    L.die_kern_layernorm.argtypes = [u64] * 4 + [C.c_float, C.c_longlong, i, u64, i, i]
    L.die_kern_tokens.restype = i
    L.die_kern_tokens.argtypes = [u64] * 4 + [i] * 3 + [u64, i]
    L.die_kern_gather_rows.restype = i
    L.die_kern_gather_rows.argtypes = [u64, u64] + [i] * 4 + [u64, i]
    L.die_kern_attention.restype = i
    L.die_kern_attention.argtypes = [u64] * 4 + [i] * 8 + [C.c_float, u64, i]
    L.die_kern_set_attention_variant.restype = None
    L.die_kern_set_attention_variant.argtypes = [i]
    L.die_kern_set_decode_variant.restype = None
    L.die_kern_set_decode_variant.argtypes = [i]
    L.die_kern_set_layernorm_xcd.restype = None
    L.die_kern_set_layernorm_xcd.argtypes = [i]
    L.die_kern_set_pair_shared_w.restype = None
    L.die_kern_set_pair_shared_w.argtypes = [i]
    L.die_kern_set_gap_fc_stop.restype = None
    L.die_kern_set_gap_fc_stop.argtypes = [i]
    L.die_kern_gap_fc.restype = i
    L.die_kern_gap_fc.argtypes = [u64] + [i] * 4 + [u64, C.c_longlong, i, u64, i, i, u64, u64, C.c_longlong, u64, i,
                                                      u64, i]
    L.die_decode_scratch_bytes.restype = C.c_longlong
    L.die_decode_scratch_bytes.argtypes = [i, C.c_longlong]
    L.die_kern_decode.restype = i
    L.die_kern_decode.argtypes = [u64, u64, C.c_longlong, u64, i, u64, C.c_longlong, u64, u64, u64, u64]
    L.die_kern_decode_packed.restype = i
    L.die_kern_decode_packed.argtypes = [u64, u64, u64, u64, C.c_longlong, u64, i, u64, C.c_longlong, u64, u64, u64, u64]
    L._kern_sigs = True
    return L


def plan_summary(model_path: str, max_batch: int = 32, side_branches: bool = False,
                 precision: str = "bf16", fuse_pairs: bool = True, fuse_stem_pool: bool = True,
                 fuse_gap_fc: bool = False, fold_layernorm: bool = True,
                 ln_stats_epilogue: bool = True) -> Dict[str, Any]:
    """precision "fp32" plans the split (hi, lo) kernels of the HIP engine's default mode.
    fuse_pairs: expand + next reduce 1x1 convs as one conv_pair op (EngineOptions::fuse_pairs);
    fuse_stem_pool: stem conv + max pool as one stem op (EngineOptions::fuse_stem_pool);
    fuse_gap_fc: global pool + FC head as one gap_fc op (EngineOptions::fuse_gap_fc);
    fold_layernorm: LayerNorms read only by GEMMs compute statistics only (EngineOptions::fold_layernorm);
    ln_stats_epilogue: ... from the epilogue of the GEMM producing their input (EngineOptions::ln_stats_epilogue)."""
    L = _sig_kernels()
    err = _err_box()
    p = L.die_plan_summary(model_path.encode(), max_batch, int(side_branches), int(precision == "fp32"),
                           int(fuse_pairs) | 2 * int(fuse_stem_pool) | 4 * int(fuse_gap_fc) | 8 * int(fold_layernorm)
                           | 16 * int(ln_stats_epilogue), C.byref(err))
    if not p:
        _raise_if(err, "plan")
    return json.loads(_take_str(p))


def plan_report(model_path: str, precision: str = "fp32") -> Dict[str, Any]:
    """Which nodes the HIP planner cannot lower (and why): {"supported", "unsupported": [{node, op,
    error}], "blocked", "text"}.  Runs on the CPU (no GPU needed)."""
    L = lib()
    fn = L.die_plan_report
    fn.restype = C.c_void_p
    fn.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
    err = _err_box()
    p = fn(model_path.encode(), int(precision == "fp32"), C.byref(err))
    if not p:
        _raise_if(err, "plan_report")
    return json.loads(_take_str(p))


def hybrid_partition(model_path: str, max_batch: int = 8, precision: str = "fp32") -> List[Dict[str, Any]]:
    """How a model splits into HIP and CPU-executor segments when some of its nodes cannot be lowered
    (engine/hybrid_engine.cpp; runs on the CPU): [{device, first, last, input, output, gemm_nodes,
    ops}] in execution order."""
    L = lib()
    fn = L.die_hybrid_partition
    fn.restype = C.c_void_p
    fn.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    err = _err_box()
    p = fn(model_path.encode(), int(max_batch), int(precision == "fp32"), C.byref(err))
    if not p:
        _raise_if(err, "hybrid_partition")
    return json.loads(_take_str(p))


def kernels():
    """The raw kernel-launch entry points (see ops/kernels.py for the torch-facing wrappers)."""
    return _sig_kernels()
