"""Headline benchmark: requests/sec (+ p50/p99 latency) of ResNet50-v2 `/infer` on MI355X.

Reference headline (README.md:276-289): 522.64 req/s, p50 84.6 ms at 10k requests /
50 client threads through the gateway (benchmark.py:26-30 -> src/gateway.cpp:176-198 -> worker).
Same topology here (default --mode gateway): every rank runs a worker node on its own GPU (C++
epoll HTTP server, JSON text decoded on the GPU, LRU cache, dynamic batcher at max batch 32, HIP
engine with hipGraph-captured forward passes, fp32 numerics like the reference's ORT session) and
a gateway (consistent-hash routing on request_id over ALL ranks' workers, circuit breakers,
event-driven keep-alive forwarding), driven by a C++ closed-loop client with 50 keep-alive
connections per GPU into that gateway.  Payloads are ResNet-shaped (3x224x224 floats, 4 decimals,
~1.1 MB of JSON) and unique per request, so every request is a real inference (no cache hits).
Weights are random-init (no checkpoint offline).

After the headline (and only reported as extra keys): the same requests straight to the worker
(`direct_worker`), and BASELINE config 4 -- ONE data-parallel worker over all N ranks with RCCL
(weights ncclBroadcast from rank 0, per-batch logits + decode status ncclAllGather over xGMI; at
N=1 the multi-rank merge path is forced so the communicator still forms) -- run in child processes
under a watchdog, as `dp_rccl` ({"error": ...} if it fails or hangs; the headline is never lost).

A "step" = --step-requests (500) requests per GPU, so the driver's `--steps 20` times 10,000
requests per GPU: the reference's run length.  W warmup steps (after engine autotune and graph
capture), then exactly K timed steps bracketed by barrier + torch.cuda.synchronize() (the client's
payload templates are built before the opening barrier: loadgen's on_ready hook); the max wall
time over ranks is the job time and `value` = total successful requests / that time (whole job,
all GPUs).  The same count of requests sent straight to the worker (no gateway hop) is reported as
the extra key `direct_worker`.
"""
import argparse
import json
import os
import resource
import signal
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import die_amd  # noqa: E402,F401  (first: sets the HIP runtime environment before anything touches the GPU)

BASELINE_RPS = 522.64  # BASELINE.md / README.md:282


def _hist_window(h0, h1):
    """Per-size batch counts over the timed window (lifetime histograms h1 - h0, zero-padded)."""
    n = max(len(h0), len(h1))
    h0 = list(h0) + [0] * (n - len(h0))
    h1 = list(h1) + [0] * (n - len(h1))
    return [b - a for a, b in zip(h0, h1)]


def _cpu_quota():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--step-requests", type=int, default=500,
                    help="requests per GPU per step (20 steps = the reference's 10k requests)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--connections", type=int, default=50, help="client connections per GPU (reference: 50 threads)")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="fp32 = the reference's numerics (split bf16 MFMA); bf16 = fast mode")
    ap.add_argument("--mode", choices=["gateway", "http", "dp", "engine"], default="gateway",
                    help="gateway: client -> gateway -> worker per GPU (reference topology); http: client -> "
                         "worker; dp: ONE worker whose batches are sharded over all ranks (RCCL); engine: "
                         "forward-only (a step = one batch)")
    ap.add_argument("--no-direct", action="store_true", help="skip the extra direct-to-worker measurement")
    ap.add_argument("--gw-client-threads", type=int, default=0, help="gateway forwarding loops (0 = auto)")
    ap.add_argument("--worker-http-threads", type=int, default=0, help="worker HTTP reactors (0 = auto: CPU share)")
    ap.add_argument("--gw-http-threads", type=int, default=0, help="gateway HTTP reactors (0 = auto: CPU share)")
    ap.add_argument("--no-local-shm", action="store_true",
                    help="gateway sends co-located workers the body bytes instead of a shared-memory descriptor")
    ap.add_argument("--model", default="", help="existing ONNX file (default: generate --arch)")
    ap.add_argument("--arch", choices=["resnet50", "vit_b16", "resnet_tiny"], default="resnet50",
                    help="resnet50 = headline config 2; vit_b16 = BASELINE config 5 (ViT-B/16, batch 32)")
    ap.add_argument("--pipeline-depth", type=int, default=3)
    ap.add_argument("--exec-streams", type=int, default=1, help="batches executing concurrently on the GPU")
    ap.add_argument("--parse-threads", type=int, default=-1,
                    help="worker body-parse pool (-1 auto, 0 = parse on the HTTP reactors)")
    ap.add_argument("--stage-slots", type=int, default=0,
                    help="early-upload text slots on the device (-1 auto, 0 = copy at batch submit)")
    ap.add_argument("--no-numa", action="store_true", help="keep the inherited CPU affinity (no NUMA binding)")
    ap.add_argument("--no-pace", action="store_true",
                    help="dispatch the next batch as soon as a pipeline slot frees (no just-in-time pacing)")
    ap.add_argument("--tune-warm-input", action="store_true",
                    help="autotune: run each conv's input producer right before every timing (default: L2 scrub only)")
    ap.add_argument("--loadgen-io-threads", type=int, default=0,
                    help="drive the client connections from N epoll threads instead of one thread each "
                         "(same closed loop; less client CPU in the shared CPU share)")
    ap.add_argument("--trace-device", action="store_true",
                    help="sample the engine's per-batch device time every 50 ms during the timed pass (tail attribution)")
    ap.add_argument("--splitk-fused-margin", type=float, default=0.0,
                    help="--splitk-two-kernel only: prefer in-kernel split-K within this fraction of the best")
    ap.add_argument("--splitk-two-kernel", action="store_true",
                    help="autotune may pick the two-kernel split-K form (partials + reduction kernel; EngineOptions)")
    ap.add_argument("--pace-lead-scale", type=float, default=1.0,
                    help="pacing lead: 1 = measured input path + adaptive margin; other values = input path x this")
    ap.add_argument("--branch-streams", action="store_true",
                    help="run the projection-shortcut convs on a side stream (measured slower; off by default)")
    ap.add_argument("--attn-variant", type=int, default=0,
                    help="measurement: streaming attention variant (kernels.h set_attention_variant)")
    ap.add_argument("--decode-variant", type=int, default=0,
                    help="measurement: device JSON decode kernels, 0 symbol-level (default), 1 character-level (round 4)")
    ap.add_argument("--pair-shared-w", type=int, default=-2,
                    help="measurement: force PairArgs::shared_w for every expand+reduce pair launch (-1 auto, "
                         "0 separate W1 / W2 LDS buffers, 1 one shared buffer; -2 = the engine's choice)")
    ap.add_argument("--ln-xcd", type=int, default=0,
                    help="measurement: LayerNorm rows read on the XCD that wrote them (1) or in natural order (0, default)")
    ap.add_argument("--no-fold-layernorm", action="store_true",
                    help="standalone LayerNorms instead of statistics + GEMM-epilogue normalisation "
                         "(EngineOptions::fold_layernorm)")
    ap.add_argument("--no-tune-orders", action="store_true",
                    help="measurement: autotune with the heuristic XCD tile order only (EngineOptions::tune_orders)")
    ap.add_argument("--tune-in-graph", action="store_true",
                    help="after the isolated-launch autotune, time each conv's front runners in place inside "
                         "eager forwards and keep the fastest (EngineOptions::tune_in_graph)")
    ap.add_argument("--no-ln-stats-epilogue", action="store_true",
                    help="measurement: LayerNorm statistics by their own launch instead of the producing "
                         "GEMM's epilogue (EngineOptions::ln_stats_epilogue)")
    ap.add_argument("--fuse-gap-fc", action="store_true",
                    help="global pool and FC head as one launch (EngineOptions::fuse_gap_fc)")
    ap.add_argument("--no-fuse-stem-pool", action="store_true",
                    help="keep ResNet's stem conv and max pool as two launches (EngineOptions::fuse_stem_pool)")
    ap.add_argument("--no-fuse-pairs", action="store_true",
                    help="keep ResNet's expand and next reduce convs as two launches (EngineOptions::fuse_pairs)")
    ap.add_argument("--no-pack-text", action="store_true",
                    help="upload input text as-is instead of 4-bit packed (device decode)")
    ap.add_argument("--tune-tail", action="store_true",
                    help="autotune tail split-K candidates too (EngineOptions::tune_tail)")
    ap.add_argument("--tune-streamk", type=int, default=-1,
                    help="autotune stream-K candidates (EngineOptions::tune_streamk): 1 on, 0 off, -1 engine default")
    ap.add_argument("--no-efficient-batch", action="store_true",
                    help="dispatch everything queued (up to --batch) instead of cutting a batch back to just "
                         "below a per-image device-time step (EngineOptions::efficient_batch)")
    ap.add_argument("--efficient-batch-tol", type=float, default=0.0,
                    help="EngineOptions::efficient_batch_tol: per-image time allowed above the best smaller batch")
    ap.add_argument("--no-efficient-batch-ends", action="store_true",
                    help="EngineOptions::efficient_batch_ends off: any size may be a cut target, not only bucket ends")
    ap.add_argument("--batch-curve-median", action="store_true",
                    help="EngineOptions::batch_curve_median: median of three replay groups per batch size")
    ap.add_argument("--efficient-batch-margin", type=float, default=0.0,
                    help="EngineOptions::efficient_batch_margin: a batch is cut only when a smaller size is "
                         "cheaper per image by more than this fraction")
    ap.add_argument("--no-batch-balance", action="store_true",
                    help="dispatch everything queued instead of the mean of the queue and the previous batch "
                         "(WorkerOptions::batch_balance)")
    ap.add_argument("--parse-spin-us", type=int, default=0,
                    help="idle parse threads poll the queue this long before sleeping (WorkerOptions::parse_spin_us)")
    ap.add_argument("--prep-on-compute", action="store_true",
                    help="measurement: run each batch's decode/prep on the compute stream before its forward "
                         "instead of on the copy stream under the previous forward (EngineOptions::prep_on_compute)")
    ap.add_argument("--no-device-decode", action="store_true",
                    help="parse input_data on the host CPU instead of decoding the JSON text on the GPU")
    ap.add_argument("--device", choices=["hip", "cpu"], default="hip",
                    help="cpu: rehearse the multi-rank contract on the host executor (tests; no GPU)")
    ap.add_argument("--dp-backend", choices=["rccl", "host"], default="rccl",
                    help="--mode dp: gather logits over RCCL (xGMI) or through the host segment")
    ap.add_argument("--dp-force-merge", action="store_true",
                    help="--mode dp at 1 rank: keep the multi-rank merge path (RCCL communicator, collectives)")
    ap.add_argument("--no-dp", action="store_true", help="skip the extra data-parallel (dp_rccl) measurement")
    ap.add_argument("--dp-steps", type=int, default=0, help="timed steps of the dp_rccl measurement (0 = --steps)")
    ap.add_argument("--dp-timeout", type=float, default=240.0, help="watchdog of the dp_rccl measurement (s)")
    ap.add_argument("--verify-every", type=int, default=50,
                    help="every Nth timed request carries one of 8 fixed inputs whose logits the CPU executor "
                         "computed beforehand; its answer is checked (0 = off; a mismatch zeroes the value)")
    ap.add_argument("--no-ring-balance", action="store_true",
                    help="N>1 gateway mode: ephemeral worker ports instead of ring-balanced ones")
    ap.add_argument("--no-gateway-bytes", action="store_true",
                    help="skip the extra pass with bodies re-sent over loopback HTTP (reference gateway hop)")
    ap.add_argument("--conv-order", type=int, default=0,
                    help="measurement: force every conv's XCD tile order (1 N-fastest, 2 M-fastest; EngineOptions)")
    ap.add_argument("--no-result-stream", action="store_true",
                    help="result D2H on the compute stream instead of a side stream (EngineOptions::result_stream)")
    ap.add_argument("--no-ref-client", action="store_true",
                    help="skip the extra run of the reference's own workload (tools/ref_bench.py: Python "
                         "benchmark.py client, 3-float payloads, gateway + 3 workers on this rank's GPU)")
    args = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        # n_gpus and global_batch come from --gpus: a torchrun launch must say how many ranks it has
        ap.error("--gpus %d does not match WORLD_SIZE %s" % (args.gpus, os.environ.get("WORLD_SIZE", "1")))

    # rank 0's stdout carries exactly ONE JSON line: library chatter written to fd 1 while the
    # job runs (RCCL's version banner at communicator init, ROCm runtime notes) goes to stderr.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch  # first: one HIP runtime per process (see native.lib)

    import die_amd  # noqa: F401
    from die_amd import native
    if args.device == "hip" and args.ln_xcd != 0:
        native.kernels().die_kern_set_layernorm_xcd(int(args.ln_xcd))
    if args.device == "hip" and args.decode_variant != 0:
        native.kernels().die_kern_set_decode_variant(int(args.decode_variant))
    if args.device == "hip" and args.attn_variant != 0:
        native.kernels().die_kern_set_attention_variant(int(args.attn_variant))
    if args.device == "hip" and args.pair_shared_w != -2:
        native.kernels().die_kern_set_pair_shared_w(int(args.pair_shared_w))
    from die_amd.parallel.launch import HostGroup

    hg = HostGroup()  # gloo: host-side barriers and reductions over the ranks
    rank, world, local_rank = hg.rank, hg.world, hg.info.local_rank
    hip = args.device == "hip"

    def barrier():
        hg.barrier()
        if hip:
            torch.cuda.synchronize()

    def timed_loadgen(start=None, **kw):
        """One timed client pass: the load generator builds every connection's payload templates and
        finishes its warm-up, then calls back here; the barrier (+ device sync) that opens the timed
        window runs in that callback, so payload construction is never timed.  Returns (result,
        elapsed seconds barrier to barrier, rusage at the start)."""
        t = {}

        def ready():
            barrier()
            t["ru0"] = resource.getrusage(resource.RUSAGE_SELF)
            if start is not None:
                start()
            t["t0"] = time.perf_counter()
        r_ = native.loadgen(on_ready=ready, **kw)
        barrier()
        return r_, time.perf_counter() - t["t0"], t["ru0"]
    if args.arch == "vit_b16":
        from die_amd.models import vit as r

        cfg = r.ViTConfig()
        model_name, fname = "ViT-B/16 (ONNX, generated)", "vit-b16.onnx"
    elif args.arch == "resnet_tiny":  # multi-rank CPU rehearsals only (tests/test_bench_contract.py)
        from die_amd.models import resnet_v2 as r

        cfg = r.tiny_config()
        model_name, fname = "ResNet-v2 tiny (rehearsal)", "resnet-tiny.onnx"
    else:
        from die_amd.models import resnet_v2 as r

        cfg = r.ResNetConfig()
        model_name, fname = "ResNet50-v2-7 (ONNX, generated)", "resnet50-v2-7.onnx"
    model = args.model
    tmpdir = None
    if not model:
        tmpdir = tempfile.mkdtemp(prefix="die_bench_%d_" % rank)
        model = os.path.join(tmpdir, fname)
        blob, _ = r.build_onnx(cfg)
        with open(model, "wb") as f:
            f.write(blob)
    # one process per GPU; ranks wrap onto the visible GPUs (a 1-GPU box can rehearse N=2 in
    # http mode: two independent replicas on one card; RCCL dp mode needs distinct GPUs)
    dev = local_rank % max(1, torch.cuda.device_count()) if hip else 0
    if hip:
        torch.cuda.set_device(dev)
    numa = {"bound": False}
    if hip and not args.no_numa:
        # this rank's threads and host buffers on its GPU's socket
        numa = native.bind_local_cpus(dev, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    B = args.batch
    numel = cfg.in_ch * cfg.image * cfg.image
    extra = {}

    SR = args.step_requests
    # Answer verification: K fixed inputs, logits from the CPU executor (fp32, an
    # independent implementation of the same ONNX graph); the timed pass sends every Nth request as
    # one of them, with its text zero-padded per request so it is computed, never a cache hit.
    verify = None
    if args.verify_every > 0 and args.mode in ("gateway", "http"):
        import numpy as np

        v4 = r.synthetic_input(8, cfg, seed=4242).astype(np.float32)
        vx = v4.reshape(8, -1).copy()
        # plain decimals: the load generator pads them with 0-15 zeros each (unique texts that stay on
        # the device decoder's fast path: no host re-parse, csrc/serve/loadgen.cpp verify_body)
        vx[:, 0], vx[:, 1], vx[:, 2] = 0.5, 0.75, 0.25
        vref = native.cpu_run(model, vx.reshape(v4.shape)).reshape(8, -1)
        verify = dict(verify_inputs=vx, verify_expected=vref, verify_every=args.verify_every,
                      verify_tol=1e-3 if args.precision == "fp32" else 5e-2)
    engine_opts = {"device": args.device, "device_id": dev, "max_batch": B, "precision": args.precision,
                   "pipeline_depth": args.pipeline_depth, "stage_slots": args.stage_slots,
                   "exec_streams": args.exec_streams, "pace": not args.no_pace,
                   "pace_lead_scale": args.pace_lead_scale, "tune_warm_input": args.tune_warm_input,
                   "splitk_fused_margin": args.splitk_fused_margin, "splitk_two_kernel": args.splitk_two_kernel,
                   "result_stream": not args.no_result_stream, "conv_order": args.conv_order,
                   "pack_text": not args.no_pack_text, "branch_streams": args.branch_streams,
                   "device_decode": not args.no_device_decode, "fuse_pairs": not args.no_fuse_pairs,
                   "fuse_stem_pool": not args.no_fuse_stem_pool,
                   "fuse_gap_fc": args.fuse_gap_fc, "fold_layernorm": not args.no_fold_layernorm,
                   "ln_stats_epilogue": not args.no_ln_stats_epilogue, "tune_in_graph": args.tune_in_graph,
                   "tune_orders": not args.no_tune_orders, "prep_on_compute": args.prep_on_compute,
                   "efficient_batch": not args.no_efficient_batch, "tune_tail": args.tune_tail,
                   **({} if args.tune_streamk < 0 else {"tune_streamk": bool(args.tune_streamk)}), "efficient_batch_tol": args.efficient_batch_tol,
                   "efficient_batch_margin": args.efficient_batch_margin,
                   "batch_curve_median": args.batch_curve_median,
                   "efficient_batch_ends": not args.no_efficient_batch_ends}
    if args.mode in ("gateway", "http"):
        # N > 1 behind the gateways: worker ports that balance the consistent-hash ring (routing itself
        # unchanged; parallel/ring_balance.py) -- arbitrary ports leave the busiest of 8 workers with
        # ~1.5x its fair share of the requests
        want_port = 0
        if args.mode == "gateway" and world > 1 and not args.no_ring_balance:
            from die_amd.parallel import ring_balance as rb

            ports = rb.balanced_ports(world, range(20000, 22000), seed=world) if rank == 0 else None
            want_port = hg.broadcast_object(ports, src=0)[rank]
        t_init = time.perf_counter()
        try:
            wk = native.Worker(model, node_id="gpu%d" % local_rank, max_batch=B, engine=engine_opts, port=want_port,
                               parse_threads=args.parse_threads, http_threads=args.worker_http_threads,
                               parse_spin_us=args.parse_spin_us, batch_balance=not args.no_batch_balance)
        except native.NativeError:
            if not want_port:
                raise
            wk = native.Worker(model, node_id="gpu%d" % local_rank, max_batch=B, engine=engine_opts,
                               parse_threads=args.parse_threads, http_threads=args.worker_http_threads,
                               parse_spin_us=args.parse_spin_us, batch_balance=not args.no_batch_balance)
        t_ready = time.perf_counter()
        gw = None
        target_port = wk.port
        if args.mode == "gateway":
            # every rank's gateway routes over every rank's worker (ring on request_id)
            ports = hg.all_gather_object(wk.port)
            gw = native.GatewayServer(["127.0.0.1:%d" % p for p in ports], client_threads=args.gw_client_threads,
                                      local_shm=not args.no_local_shm, http_threads=args.gw_http_threads,
                                      # a CPU-executor batch can outlast the reference's 5 s read timeout
                                      # on a loaded host; the HIP path keeps the reference value
                                      read_timeout_ms=5000 if hip else 120000)
            target_port = gw.port
        # every pass and rank gets its own payload seed: no input recurs across the warm-up, timed and
        # direct passes (cache_hits_timed below proves it); request numbers are printed scrambled
        # (FNV-1a spreads them over the ring like random ids)
        lg = dict(connections=args.connections, payload="full", input_numel=numel, decimals=4, timeout_ms=60000,
                  scramble_ids=True, io_threads=args.loadgen_io_threads)
        native.loadgen(port=target_port, requests=args.warmup * SR, warmup=0, id_prefix="warm%d_" % rank,
                       seed=1000 + rank, **lg)
        h0 = wk.health()
        g0 = gw.stats() if gw else {}
        trace = []
        stop_trace = threading.Event()
        tt = {}

        def _start():
            tt["t0"] = time.perf_counter()
            if args.trace_device:
                # opt-in: sample the engine's batch / busy counters every 50 ms during the timed pass, so a
                # tail late in the pass can be told apart from device slow-down (clocks) or host stalls
                def _sampler():
                    while not stop_trace.wait(0.05):
                        e = wk.health()["engine"]
                        trace.append((time.perf_counter(), e.get("batches", 0), e.get("images", 0),
                                      e.get("avg_device_ms", 0.0)))
                threading.Thread(target=_sampler, daemon=True).start()
        res, elapsed, ru0 = timed_loadgen(start=_start, port=target_port, requests=args.steps * SR, warmup=0,
                                          id_prefix="r%d_" % rank, seed=2000 + rank, **dict(lg, **(verify or {})))
        stop_trace.set()
        t0 = tt["t0"]
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        h1 = wk.health()
        g1 = gw.stats() if gw else {}
        ok = res["ok"]
        failed = res["failed"]
        bp0, bp1 = h0["batch_processor"], h1["batch_processor"]
        nb = bp1["total_batches"] - bp0["total_batches"]
        e0, e1 = h0["engine"], h1["engine"]
        extra = {
            "p50_ms": res["latency_ms"]["p50"], "p99_ms": res["latency_ms"]["p99"],
            "mean_ms": res["latency_ms"]["mean"], "failed": failed,
            # tail attribution: p99 per tenth of the timed pass (by request start) + the slowest requests
            "tail": {"p99_by_tenth_ms": [round(v, 2) for v in res.get("p99_by_tenth_ms", [])],
                     "slowest_ms": res.get("slowest_ms", []), "device_trace": _device_trace(trace, t0)},
            "cache_hits_timed": h1["cache_hits"] - h0["cache_hits"],
            "avg_batch": (bp1["total_requests"] - bp0["total_requests"]) / max(nb, 1),
            # batches cut below the queue: balanced batches (WorkerOptions::batch_balance) and bucket-end
            # sizes (EngineOptions::efficient_batch)
            "trimmed_batches": bp1.get("trimmed_batches", 0) - bp0.get("trimmed_batches", 0),
            "trimmed_requests": bp1.get("trimmed_requests", 0) - bp0.get("trimmed_requests", 0),
            # batches per size over the timed pass: [count at size 1, size 2, ...]
            "batch_size_histogram": _hist_window(bp0.get("size_histogram", []), bp1.get("size_histogram", [])),
            # the engine's start-up forward time per batch size (ms at 1, 2, ...; EngineOptions::efficient_batch)
            "batch_curve_ms": [round(v, 3) for v in e1.get("batch_curve_ms", [])],
            "device_ms_per_batch": _win(e0, e1, "avg_device_ms"), "engine": e1.get("device"),
            "precision": e1.get("precision"),
            "client_connections_per_gpu": args.connections, "body_bytes": res.get("body_bytes"),
            "parse_us_avg": h1.get("parse_us_avg"), "host_cpus": len(os.sched_getaffinity(0)),
            "cpu_quota": _cpu_quota(), "device_decode": e1.get("device_decode"),
            "decode_fallbacks": h1.get("decode_fallbacks"),
            "pipeline_depth": args.pipeline_depth, "exec_streams": e1.get("executors"),
            "worker_init_s": round(t_ready - t_init, 2),
            # engine averages over the timed window only (the engine keeps lifetime totals, which
            # include warm-up and autotune-time batches)
            "copy_wait_ms_per_batch": _win(e0, e1, "avg_copy_wait_ms"),
            "gpu_gap_ms_per_batch": _win(e0, e1, "avg_gpu_gap_ms"),
            "prep_ms_per_batch": _win(e0, e1, "avg_prep_ms"),
            "device_busy_frac": _busy(e0, e1, elapsed), "pace": e1.get("pace"), "pack_text": e1.get("pack_text"),
            "pace_lead_ms": e1.get("avg_pace_lead_ms"), "submit_us_avg": e1.get("staging_diag", {}).get("submit_us_avg"),
            "pace_input_ms": e1.get("pace_input_ms"), "pace_margin_ms": e1.get("pace_margin_ms"),
            "stages_us": {k: round(v["avg_us"], 1) for k, v in h1.get("stages_us", {}).items()},
            "stages_p99_us": {k: round(v.get("p99_us", 0.0), 1) for k, v in h1.get("stages_us", {}).items()},
            "engine_options": e1.get("options"),
            # windowed to the timed pass (histogram differences), 8 buckets per octave
            "stages_window_us": _stage_window(h0.get("stages_us", {}), h1.get("stages_us", {})),
            # host CPU spent per request by this process (client + gateway + worker threads together)
            "cpu_us_per_request": {"user": round((ru1.ru_utime - ru0.ru_utime) * 1e6 / max(1, res["ok"]), 1),
                                   "sys": round((ru1.ru_stime - ru0.ru_stime) * 1e6 / max(1, res["ok"]), 1),
                                   # where sys time can come from: page faults and context switches
                                   "minflt": round((ru1.ru_minflt - ru0.ru_minflt) / max(1, res["ok"]), 2),
                                   "majflt": round((ru1.ru_majflt - ru0.ru_majflt) / max(1, res["ok"]), 3),
                                   "vcsw": round((ru1.ru_nvcsw - ru0.ru_nvcsw) / max(1, res["ok"]), 2),
                                   "ivcsw": round((ru1.ru_nivcsw - ru0.ru_nivcsw) / max(1, res["ok"]), 2)},
        }
        if verify:
            extra["verify"] = {"every": args.verify_every, "inputs": 8, "oracle": "cpu_executor_fp32",
                               "tol": verify["verify_tol"], "verified": res.get("verified", 0),
                               "mismatched": res.get("mismatched", 0), "bad_request_id": res.get("bad_request_id", 0),
                               "max_rel_err": res.get("max_rel_err"),
                               "repeat_period": res.get("verify_repeat_period")}
            # every verified answer computed, never served from the cache: no verify text repeats
            rp = res.get("verify_repeat_period")
            if rp is not None and rp < SR * (args.steps + args.warmup):
                extra["verify"]["error"] = "verify texts repeat after %d requests" % rp
        extra["worker_requests_timed"] = bp1["total_requests"] - bp0["total_requests"]
        if gw:
            extra["gateway"] = {"failovers": g1["failovers"] - g0["failovers"], "failed": g1["failed"] - g0["failed"],
                                "upstream_connections": g1.get("upstream_connections_opened"),
                                "shm_forwards": g1.get("shm_forwards", 0) - g0.get("shm_forwards", 0),
                                "byte_forwards": g1.get("byte_forwards", 0) - g0.get("byte_forwards", 0),
                                "breakers": [b["state"] for b in g1["circuit_breakers"]],
                                # per-stage p50/p99 (warm-up included): where a gateway tail comes from
                                "stages_us": {k: [round(v["p50_us"], 1), round(v["p99_us"], 1)]
                                              for k, v in g1.get("stages_us", {}).items()},
                                "stages_window_us": _stage_window(g0.get("stages_us", {}), g1.get("stages_us", {}))}
            if world > 1:
                from die_amd.parallel import ring_balance as rb

                names = ["127.0.0.1:%d" % p for p in ports]
                ids = [x for k in range(world) for x in rb.request_ids("r%d_" % k, args.steps * SR)]
                extra["ring"] = dict(rb.predict(names, ids), balanced_ports=not args.no_ring_balance,
                                     ports=list(ports),
                                     arc_max_over_fair=round(float(rb.arc_shares(names).max() * world), 3),
                                     # the same routing on the reference's own layout (ports
                                     # 8001.., sequential "req_<i>" ids), next to the tuned deployment
                                     reference_layout=rb.reference_layout(world, args.steps * SR * world))
        if gw and not args.no_direct:
            # informative: the same request count straight to this rank's worker (no gateway hop)
            barrier()
            hd0 = wk.health()
            rd, el, rd0 = timed_loadgen(port=wk.port, requests=args.steps * SR, warmup=0, id_prefix="d%d_" % rank,
                                        seed=3000 + rank, **lg)
            rd1 = resource.getrusage(resource.RUSAGE_SELF)
            hd1 = wk.health()
            n_ok = max(1, rd["ok"])
            extra["direct_worker"] = {"rps_this_rank": rd["ok"] / el, "p50_ms": rd["latency_ms"]["p50"],
                                      "p99_ms": rd["latency_ms"]["p99"], "failed": rd["failed"],
                                      "cpu_us_per_request": {"user": round((rd1.ru_utime - rd0.ru_utime) * 1e6 / n_ok, 1),
                                                             "sys": round((rd1.ru_stime - rd0.ru_stime) * 1e6 / n_ok, 1),
                                                             "minflt": round((rd1.ru_minflt - rd0.ru_minflt) / n_ok, 2),
                                                             "vcsw": round((rd1.ru_nvcsw - rd0.ru_nvcsw) / n_ok, 2),
                                                             "ivcsw": round((rd1.ru_nivcsw - rd0.ru_nivcsw) / n_ok, 2)},
                                      # tail attribution: p99 per tenth of the pass by
                                      # request start, the slowest requests [start ms, latency ms], and the
                                      # worker's stage histograms over this pass only
                                      "p99_by_tenth_ms": [round(v, 2) for v in rd.get("p99_by_tenth_ms", [])],
                                      "slowest_ms": rd.get("slowest_ms", []),
                                      "stages_window_us": _stage_window(hd0.get("stages_us", {}), hd1.get("stages_us", {}))}
        if gw and not args.no_gateway_bytes:
            # the reference's gateway hop: every body re-sent to the worker over loopback HTTP
            # (/root/reference/src/gateway.cpp:99-103) instead of a shared-memory descriptor
            gwb = native.GatewayServer(["127.0.0.1:%d" % p for p in ports], client_threads=args.gw_client_threads,
                                       local_shm=False, http_threads=args.gw_http_threads,
                                       read_timeout_ms=5000 if hip else 120000)
            barrier()
            rb_, elb, _ = timed_loadgen(port=gwb.port, requests=args.steps * SR, warmup=0, id_prefix="b%d_" % rank,
                                        seed=4000 + rank, **lg)
            gs = gwb.stats()
            extra["gateway_bytes"] = {"rps_this_rank": rb_["ok"] / elb, "p50_ms": rb_["latency_ms"]["p50"],
                                      "p99_ms": rb_["latency_ms"]["p99"], "failed": rb_["failed"],
                                      "byte_forwards": gs.get("byte_forwards", 0), "shm_forwards": gs.get("shm_forwards", 0)}
            gwb.stop()
        if gw:
            gw.stop()
        wk.stop()
        if not args.no_dp:
            extra["dp_rccl"] = _dp_child(args, hg, rank, world)
        if hip and args.arch == "resnet50" and args.mode == "gateway" and not args.no_ref_client:
            extra["ref_client"] = _ref_client(hg, rank, dev)
    elif args.mode == "dp":
        # BASELINE config 4: ONE data-parallel worker over all ranks.  Every rank serves HTTP on the
        # same port (SO_REUSEPORT) and parses its own connections' requests; the leader merges the
        # ranks' queued sub-batches into DP batches sharded over the GPUs (RCCL all-gather of logits),
        # and every rank answers its own requests.  Each rank drives its own 50-connection client.
        group = "die_bench_dp_%s" % os.environ.get("MASTER_PORT", str(os.getpid()))
        Btot = B * world
        port = 0
        if rank == 0:
            import socket

            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
            sk.close()
        port = hg.broadcast_object(port, src=0)
        eng_opts = dict(engine_opts, dp_world=world, dp_group=group, dp_rank=rank, dp_backend=args.dp_backend,
                        dp_force_merge=args.dp_force_merge)
        wk = native.Worker(model, node_id="dp-r%d" % rank, port=port, reuse_port=True, max_batch=Btot,
                           engine=eng_opts, parse_threads=args.parse_threads)
        lg = dict(port=port, connections=args.connections, payload="full", input_numel=numel, decimals=4,
                  timeout_ms=60000, io_threads=args.loadgen_io_threads)
        native.loadgen(requests=args.warmup * SR, warmup=0, id_prefix="warm%d_" % rank, seed=1000 + rank, **lg)
        h0 = wk.health()
        res, elapsed, _ = timed_loadgen(requests=args.steps * SR, warmup=0, id_prefix="r%d_" % rank, seed=2000 + rank,
                                        **lg)
        ok, failed = res["ok"], res["failed"]
        h1 = wk.health()
        e1 = h1["engine"]
        extra = {"p50_ms": res["latency_ms"]["p50"], "p99_ms": res["latency_ms"]["p99"],
                 "mean_ms": res["latency_ms"]["mean"], "failed": failed,
                 "cache_hits_timed": h1["cache_hits"] - h0["cache_hits"],
                 "engine": e1.get("device"), "dp_backend": e1.get("dp_backend"), "precision": e1.get("precision"),
                 "dp_solo": e1.get("dp_solo"), "dp_world": e1.get("dp_world"),
                 "dp_shard_failed_items": e1.get("dp_shard_failed_items"),
                 "dp_affinity_restores": e1.get("dp_affinity_restores"), "host_cpus": len(os.sched_getaffinity(0)),
                 "device_ms_per_batch": e1.get("avg_device_ms"),
                 "dp_batches_rank0": e1.get("dp_batches", 0) - h0["engine"].get("dp_batches", 0),
                 "requests_parsed_this_rank": h1["total_requests"] - h0["total_requests"],
                 "client_connections_per_gpu": args.connections,
                 "subbatches_sent_this_rank": e1.get("dp_subbatches_sent", 0) - h0["engine"].get("dp_subbatches_sent", 0),
                 "gpu_gap_ms_per_batch": e1.get("avg_gpu_gap_ms"), "copy_wait_ms_per_batch": e1.get("avg_copy_wait_ms"),
                 "pace_lead_ms": e1.get("avg_pace_lead_ms"), "prep_ms_per_batch": e1.get("avg_prep_ms"),
                 "leader_wait_ms_per_batch": {k: e1.get("dp_%s_wait_ms_per_batch" % k) for k in ("pop", "slot", "pace")},
                 # dispatch fairness: leader batches any rank's sub-batch waited before riding one
                 "dp_max_sub_wait_batches": e1.get("dp_max_sub_wait_batches"),
                 "dp_mean_sub_wait_batches": e1.get("dp_mean_sub_wait_batches"),
                 "submit_us_avg": e1.get("staging_diag", {}).get("submit_us_avg"),
                 "pace_input_ms": e1.get("pace_input_ms"), "pace_margin_ms": e1.get("pace_margin_ms"),
                 "stages_us": {k: round(v["avg_us"], 1) for k, v in h1.get("stages_us", {}).items()}}
        if extra["dp_batches_rank0"]:
            extra["avg_dp_batch"] = world * SR * args.steps / extra["dp_batches_rank0"] if rank == 0 else None
        barrier()  # every rank done with traffic before the leader stops the group
        if rank != 0:
            barrier()
        wk.stop()
        if rank == 0 and world > 1:
            barrier()
    else:
        import numpy as np

        eng = native.Engine(model, **engine_opts)
        x = r.synthetic_input(B, cfg, seed=rank).reshape(B, -1)
        for _ in range(args.warmup):
            eng.run(x)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.run(x)
        barrier()
        elapsed = time.perf_counter() - t0
        ok, failed = args.steps * B, 0
        # device_ms_per_batch: the in-graph forward (hipGraph replay of bucket B, events around it)
        extra = {"engine": eng.refresh_info()["name"], "device_ms_per_batch": eng.info.get("avg_device_ms"),
                 "engine_options": eng.info.get("options"),
                 "tune_in_graph": {"timed": eng.info.get("tune_in_graph_timed"), "changed": eng.info.get("tune_in_graph_changed")}}
        eng.close()

    if world > 1:
        # where the time goes, rank by rank (a SCALE number blends host-CPU partitioning with GPU
        # scaling: each rank's own throughput, latency, batch size, device time and host CPU)
        mine = {"rank": rank, "requests_per_s": round(ok / elapsed, 1) if elapsed > 0 else None,
                "elapsed_s": round(elapsed, 3), "failed": failed}
        for k in ("p50_ms", "p99_ms", "avg_batch", "avg_dp_batch", "device_ms_per_batch", "device_busy_frac",
                  "gpu_gap_ms_per_batch", "cpu_us_per_request", "requests_parsed_this_rank", "worker_requests_timed"):
            if extra.get(k) is not None:
                mine[k] = extra[k]
        if isinstance(extra.get("direct_worker"), dict):
            mine["direct_rps"] = round(extra["direct_worker"].get("rps_this_rank", 0.0), 1)
        mine["numa_cpus"] = numa.get("cpu_share") if isinstance(numa, dict) else None
        per_rank = hg.all_gather_object(mine)
        if rank == 0:
            tot = sum(x.get("worker_requests_timed", 0) for x in per_rank)
            for x in per_rank:  # measured ring share of each rank's worker (ring.shares: predicted)
                if tot and "worker_requests_timed" in x:
                    x["worker_share"] = round(x["worker_requests_timed"] / tot, 4)
            extra["per_rank"] = per_rank
        if isinstance(extra.get("verify"), dict):
            v = extra["verify"]
            v["verified"], v["mismatched"], v["bad_request_id"] = hg.reduce(
                [v["verified"], v["mismatched"], v["bad_request_id"]], "sum")
        if isinstance(extra.get("gateway_bytes"), dict):
            gb = extra["gateway_bytes"]
            gb["requests_per_s"] = hg.reduce([gb.pop("rps_this_rank")], "sum")[0]
            gb["p99_ms"] = hg.reduce([gb["p99_ms"]], "max")[0]
        elapsed = hg.reduce([elapsed], "max")[0]
        ok, failed = hg.reduce([ok, failed], "sum")
        extra["p50_ms"], extra["p99_ms"] = hg.reduce([extra.get("p50_ms", 0.0), extra.get("p99_ms", 0.0)], "max")
    value = ok / elapsed
    v = extra.get("verify")
    if isinstance(v, dict) and (v["mismatched"] or v["bad_request_id"] or not v["verified"] or v.get("error")):
        extra["error"] = "answer verification failed: %s" % (v,)
        value = 0.0  # a wrong answer does not score
    if world == 1 and isinstance(extra.get("gateway_bytes"), dict):
        extra["gateway_bytes"]["requests_per_s"] = extra["gateway_bytes"].pop("rps_this_rank")
    if rank == 0:
        out = {
            "metric": "requests/sec + p50/p99 latency, %s ONNX /infer at 1/2/4/8 MI355X"
                      % ("ResNet50" if args.arch == "resnet50" else "ViT-B/16"),
            "value": value,
            "unit": "requests/s",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1000.0 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / BASELINE_RPS if args.arch == "resnet50" else None,
            "dtype": args.precision if hip else "fp32",
            "data": "synthetic: unique image-shaped JSON payloads (3x224x224 floats, 4 decimals), random-init weights",
            "config": {"model": model_name, "global_batch": B * args.gpus, "seq_len": 0,
                       "parallelism": "dp%d" % args.gpus,
                       "mode": {"gateway": "gateway+worker", "http": "worker"}.get(args.mode, args.mode),
                       "max_batch_per_gpu": B, "requests": int(ok + failed), "connections_per_gpu": args.connections},
        }
        extra["numa"] = numa
        extra["hip_hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
        out.update({k: v for k, v in extra.items() if v is not None})
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    hg.close()


def _device_trace(trace, t0):
    """[t ms, batches, images / batch, device ms / batch] per 50 ms sample interval (--trace-device)."""
    out = []
    for a, b in zip(trace, trace[1:]):
        nb = b[1] - a[1]
        if nb <= 0:
            continue
        dev = (b[3] * b[1] - a[3] * a[1]) / nb  # lifetime averages -> this interval's
        out.append([round((b[0] - t0) * 1e3, 1), nb, round((b[2] - a[2]) / nb, 1), round(dev, 3)])
    return out


def _win(e0, e1, key):
    """Per-batch average of an engine statistic over the timed window: the engine reports lifetime
    averages (total / batches), so window = (avg1*n1 - avg0*n0) / (n1 - n0)."""
    n0, n1 = e0.get("batches", 0), e1.get("batches", 0)
    if key not in e1 or n1 <= n0:
        return e1.get(key)
    return (e1[key] * n1 - e0.get(key, 0.0) * n0) / (n1 - n0)


def _stage_window(s0, s1):
    """p50/p99 (us) of each stage over the window between two /health or /stats snapshots, from
    their histogram buckets (csrc/serve/stage_stats.h: u = ns/1024, u < 8 exact, then 8 buckets per
    octave); {stage: [count, p50, p99]}."""
    def upper(b):
        if b < 8:
            return b + 1.0
        o, sub = (b - 8) // 8 + 3, (b - 8) % 8
        return (1 << o) * (1.0 + (sub + 1) / 8.0)

    out = {}
    for k, v1 in s1.items():
        if not isinstance(v1, dict) or "hist" not in v1:
            continue
        c = {}
        for b, n in v1["hist"]:
            c[b] = c.get(b, 0) + n
        for b, n in s0.get(k, {}).get("hist", []):
            c[b] = c.get(b, 0) - n
        items = sorted((b, n) for b, n in c.items() if n > 0)
        n = sum(x for _, x in items)
        if not n:
            continue

        def pct(q):
            acc = 0
            for b, x in items:
                acc += x
                if acc > q * n:
                    return round(upper(b) * 1.024, 1)
            return round(upper(items[-1][0]) * 1.024, 1)
        out[k] = [n, pct(0.5), pct(0.99)]
    return out


def _busy(e0, e1, elapsed_s):
    """Fraction of the timed window the GPU spent in forward passes (MAIN graphs)."""
    if "device_busy_ms" not in e1 or elapsed_s <= 0:
        return None
    return round((e1["device_busy_ms"] - e0.get("device_busy_ms", 0.0)) / (elapsed_s * 1000.0), 4)


def _ref_client(hg, rank, dev):
    """The reference's own benchmark, as published (README.md:276-294 there: 522.64 req/s, p50
    84.6 ms): its client (Python `requests`, a new connection per request, 50 threads, 10,000
    requests, payload [a, a+1, a+2] with a = i % 10, benchmark.py:18-76 there) through a gateway to 3
    workers on one GPU (tools/ref_bench.py).  Rank 0 only, in a child process under a watchdog;
    returns the client summary and each worker's cache hit rate (None on other ranks)."""
    res = None
    if rank == 0:
        fd, out = tempfile.mkstemp(prefix="die_refclient_", suffix=".json")
        os.close(fd)
        cmd = [sys.executable, os.path.join(REPO, "tools", "ref_bench.py"), "--out", out, "--device", "hip",
               "--device-id", str(dev), "--requests", "10000", "--threads", "50"]
        t0 = time.perf_counter()
        try:
            # own session: on the watchdog the whole group (client, gateway, workers) goes
            p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True)
            try:
                _, se = p.communicate(timeout=420)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                raise
            if p.returncode != 0:
                res = {"error": "ref_bench exited %d: %s" % (p.returncode, se.decode(errors="replace")[-400:])}
            else:
                d = json.load(open(out))
                c = d["client"]
                lat = c.get("latency", {})
                res = {"requests_per_s": c.get("throughput"), "p50_ms": lat.get("p50"), "p99_ms": lat.get("p99"),
                       "mean_ms": lat.get("mean"), "successful": c.get("successful"), "failed": c.get("failed"),
                       "requests": d.get("requests"), "threads": d.get("threads"),
                       "worker_hit_rate": [w.get("cache_hit_rate") for w in d.get("workers", [])],
                       "worker_requests": [w.get("total_requests") for w in d.get("workers", [])],
                       "published": {"requests_per_s": BASELINE_RPS, "p50_ms": 84.60, "p99_ms": 164.29},
                       "vs_published": (c.get("throughput") or 0.0) / BASELINE_RPS,
                       "client": "tools/benchmark.py (reference CLI; python requests, new connection per request)",
                       "topology": "gateway + 3 HIP workers on GPU %d" % dev}
        except subprocess.TimeoutExpired:
            res = {"error": "ref_bench exceeded the 420 s watchdog"}
        except Exception as e:  # noqa: BLE001 (the headline must survive anything here)
            res = {"error": "ref_bench failed: %r" % (e,)}
        finally:
            try:
                os.unlink(out)
            except OSError:
                pass
        res["wall_s"] = round(time.perf_counter() - t0, 1)
    hg.barrier()
    return res


def _dp_child(args, hg, rank, world):
    """BASELINE config 4 after the headline: ONE data-parallel worker over all ranks (RCCL weight
    broadcast + per-batch all-gather; at world 1 the merge path is forced so the communicator forms),
    each rank in a child process on a fresh rendezvous, under a watchdog: a failing or hung DP run
    costs this key, never the headline.  Returns rank 0's result (extra keys of that run)."""
    port = 0
    if rank == 0:
        import socket

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
    port = hg.broadcast_object(port, src=0)
    steps = args.dp_steps or args.steps  # as long as the headline: a short run is dominated by pacing warm-up noise
    cmd = [sys.executable, os.path.abspath(__file__), "--mode", "dp", "--gpus", str(world), "--steps", str(steps),
           "--warmup", str(max(1, args.warmup)), "--step-requests", str(args.step_requests),
           "--batch", str(args.batch), "--connections", str(args.connections), "--precision", args.precision,
           "--arch", args.arch, "--pipeline-depth", str(args.pipeline_depth), "--dp-backend", "rccl",
           "--device", args.device, "--loadgen-io-threads", str(args.loadgen_io_threads)]
    if world == 1:
        cmd.append("--dp-force-merge")
    if args.model:
        cmd += ["--model", args.model]
    # a fresh rendezvous of its own (rank 0's child hosts the store): not torchrun's agent store
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    out = {"error": "no result"}
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True)
    try:
        so, se = p.communicate(timeout=args.dp_timeout)
        if p.returncode == 0 and rank == 0:
            out = json.loads(so.decode().strip().splitlines()[-1])
        elif p.returncode == 0:
            out = {}
        else:
            out = {"error": "dp run exited %d: %s" % (p.returncode, se.decode(errors="replace")[-400:])}
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        out = {"error": "dp run exceeded the %.0f s watchdog" % args.dp_timeout}
    except Exception as e:  # noqa: BLE001 (the headline must survive anything here)
        out = {"error": "dp run failed: %r" % (e,)}
    hg.barrier()
    if rank != 0:
        return None
    keep = ("value", "p50_ms", "p99_ms", "failed", "avg_dp_batch", "dp_backend", "dp_world", "dp_solo",
            "device_ms_per_batch", "engine", "cache_hits_timed", "dp_shard_failed_items", "dp_max_sub_wait_batches",
            "dp_mean_sub_wait_batches", "error")
    res = {k: out[k] for k in keep if k in out}
    if "value" in res:
        res["requests_per_s"] = res.pop("value")
        res["requests"] = out.get("config", {}).get("requests")
    res["wall_s"] = round(time.perf_counter() - t0, 1)
    return res


if __name__ == "__main__":
    main()
