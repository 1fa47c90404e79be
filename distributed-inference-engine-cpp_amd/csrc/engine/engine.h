// Engine interface: what the worker's batcher drives.
//
// Public surface mirrors the reference InferenceEngine (include/inference_engine.h:10-22):
// predict, batchPredict, getInputShape, getOutputShape, getModelPath.  Shapes report dynamic dims
// as 1 like the reference (src/inference_engine.cpp:44-51,62-68).  Beyond parity, engines take
// batches asynchronously (`submit`) so the worker can pipeline H2D / compute / D2H across batches,
// and they own the host staging memory the HTTP layer parses request floats into (pinned host
// memory for the HIP engine, so the H2D copy is a DMA straight from where the JSON was decoded).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../core/json.h"
#include "../onnx/onnx_model.h"

namespace die {

class Communicator;

// A per-sample host buffer of input_numel floats (pinned when the engine is a GPU engine).
struct SampleBuffer {
  float* data = nullptr;
  size_t capacity = 0;  // floats
};

// Pool of equally sized host buffers.  `alloc_fn` provides chunks (pinned or pageable).
class SamplePool {
 public:
  using AllocFn = std::function<void*(size_t bytes)>;
  using FreeFn = std::function<void(void*)>;
  SamplePool(size_t floats_per_sample, AllocFn a = nullptr, FreeFn f = nullptr, size_t chunk = 64);
  ~SamplePool();
  SampleBuffer acquire();
  void release(SampleBuffer b);
  size_t allocated() const { return allocated_; }

 private:
  size_t floats_;
  AllocFn alloc_;
  FreeFn free_;
  size_t chunk_;
  std::mutex mu_;
  std::vector<float*> free_list_;
  std::vector<void*> chunks_;
  size_t allocated_ = 0;
};

struct BatchItem {
  const float* input = nullptr;  // host pointer (usually a SampleBuffer)
  size_t len = 0;                // valid floats; engine zero-pads to input_numel
  // Device decode (engines with text_capacity() > 0): the JSON number-list text of input_data
  // (between '[' and ']') in engine-pinned memory; the engine converts it on the device.
  const char* text = nullptr;
  size_t text_len = 0;
  bool packed = false;  // text is 4-bit packed (core/textpack.h): (text_len + 1) / 2 bytes at `text`
  // Ticket from Engine::stage_text() when the text was already uploaded early (-1 = not staged).
  long staged = -1;
};

struct BatchResult {
  bool ok = true;
  std::string error;
  const float* outputs = nullptr;  // B * output_numel floats, valid during the callback only
  size_t output_numel = 0;
  double wall_us = 0;    // submit -> outputs on host
  double device_us = 0;  // forward time on the device (0 for CPU)
  // Per item, for text items (valid during the callback only; null when the batch had none):
  // status 0 = ok, bit 0 = needs the host parser (unusual token), 2 = more values than the model
  // input; ntok = number of values found.
  const int* status = nullptr;
  const int* ntok = nullptr;
  // Data-parallel engines with a device all-gather: outputs/status hold `gathered` ranks' shards
  // (rank r's rows at [r * B, (r + 1) * B), B = items submitted per rank); status/ntok stride
  // between ranks is `status_stride`.
  int gathered = 1;
  int status_stride = 0;
  // Data parallel: per-rank shard flags (`gathered` entries; 0 = that rank's forward did not run,
  // its rows are garbage).  Null when the engine does not gather.
  const int* rank_ok = nullptr;
};

// BatchResult::status bits (per item)
constexpr int kItemNeedsHostParse = 1;  // unusual token: re-parse on the host and re-dispatch
constexpr int kItemTooManyValues = 2;   // more values than the model input (ntok = count)
constexpr int kItemShardFailed = 4;     // data parallel: the rank computing this item failed

using BatchDone = std::function<void(BatchResult&)>;

class Engine {
 public:
  virtual ~Engine() = default;

  virtual std::string name() const = 0;
  virtual const std::string& getModelPath() const = 0;
  // Batch dim reported as 1 (reference semantics).
  virtual std::vector<int64_t> getInputShape() const = 0;
  virtual std::vector<int64_t> getOutputShape() const = 0;
  size_t input_numel() const;
  size_t output_numel() const;
  int getShardId() const { return shard_id_; }

  // Largest batch one submit() may carry.
  virtual int max_batch() const = 0;
  // Asynchronous batch execution.  Blocks while the engine's pipeline is full (backpressure).
  // `done` runs on an engine thread once outputs are on the host.
  virtual void submit(std::vector<BatchItem> items, BatchDone done) = 0;
  // Block until a submit() would not block.
  virtual void wait_for_slot() {}
  // Pacing for work-conserving batching: the earliest time the next batch should be dispatched.
  // An engine that knows when the batch in flight will drain returns (drain - lead), where lead
  // covers the next batch's copies; dispatching earlier only makes the next batch smaller.
  virtual std::chrono::steady_clock::time_point dispatch_not_before() { return std::chrono::steady_clock::now(); }
  // Batch size to dispatch when `queued` requests are waiting (1 <= result <= queued): an engine
  // whose per-image cost steps up at some batch sizes (tile grids spilling into another round of
  // blocks) may take fewer and leave the rest for the next batch.
  virtual int preferred_batch(int queued) const { return queued; }
  // Drain everything in flight.
  virtual void synchronize() = 0;

  // Host staging allocation for request inputs.
  virtual SamplePool& sample_pool() = 0;
  // Bytes of input_data text a SampleBuffer can carry for device decode (0 = not supported).
  virtual size_t text_capacity() const { return 0; }
  // True when submit() accepts 4-bit packed text items (BatchItem::packed).
  virtual bool text_packing() const { return false; }
  // Early upload for device decode: start copying one request's input text (engine-pinned, from
  // sample_pool()) into device staging now, on a copy stream, so the batch that later carries it
  // does not wait for its H2D.  Returns a ticket for BatchItem::staged, or -1 when the engine does
  // not stage (or staging is full: submit() then copies as usual).  The caller owns the ticket and
  // hands it back with release_staged() after the batch that carried it completed (ran = true: the
  // copy is known to be done), or with ran = false when the request failed or was dropped before
  // its batch ran (the engine then waits for the copy); the pinned text must not change until then.
  virtual long stage_text(const char* text, size_t len, bool packed = false) {
    (void)text;
    (void)len;
    (void)packed;
    return -1;
  }
  virtual void release_staged(long ticket, bool ran) {
    (void)ticket;
    (void)ran;
  }
  // Make host memory DMA-able for this engine (HIP: hipHostRegister); no-op elsewhere.  Returns
  // the bytes actually pinned (0 when the engine needs no pinning).
  virtual size_t register_host_memory(void* p, size_t bytes) {
    (void)p;
    (void)bytes;
    return 0;
  }
  // True when the engine all-gathers outputs across data-parallel ranks itself (RCCL).
  virtual bool device_gather() const { return false; }

  // Synchronous helpers with the reference's padding rules: predict() pads or truncates to the
  // model input (src/inference_engine.cpp:100-103); batchPredict() pads short inputs and, unlike
  // the reference, rejects oversized ones instead of shifting later samples.
  std::vector<float> predict(const std::vector<float>& input);
  std::vector<std::vector<float>> batchPredict(const std::vector<std::vector<float>>& inputs);

  virtual Json stats() const { return Json::object(); }
  // Per-op device timing of one forward at batch B (engines that support it; else empty object).
  virtual Json profile_ops(int B, int iters) {
    (void)B;
    (void)iters;
    return Json::object();
  }

 protected:
  int shard_id_ = 0;
};

struct EngineOptions {
  std::string device = "auto";   // auto | cpu | hip
  int device_id = 0;             // HIP device ordinal
  int max_batch = 32;
  int pipeline_depth = 3;        // batches in flight (HIP); 3 measured +2-4 % over 2 on the fp32 headline
  int exec_streams = 1;          // of those, batches executing concurrently (HIP; 1 = serialised)
  bool use_graphs = true;        // hipGraph per batch bucket (HIP)
  bool autotune = true;          // time (tile, split-K) candidates per conv at start-up (HIP)
  bool device_decode = true;     // accept input_data text and convert it on the GPU (HIP)
  // Early-upload text slots in device memory (stage_text; -1 = auto-sized, 0 = off).  Off by
  // default: at pipeline depth 2 the submit-time copies already overlap the previous batch and
  // measured faster (15.9k vs 13.3k req/s, profiles/r1_staging_ab.md); early upload wins at depth 1.
  int stage_slots = 0;
  // Just-in-time dispatch (HIP, GREEDY batching): hold the next batch until the batch on the GPU is
  // about to drain (dispatch_not_before) instead of dispatching it as soon as a slot frees.
  bool pace = true;
  // 4-bit packed text upload (core/textpack.h) for device decode: half the H2D bytes per request.
  bool pack_text = true;
  // Run independent plan branches (ResNet projection shortcuts) on a second stream (HIP).  Off by
  // default: measured slower (ResNet50 forward 0.79 vs 0.75 ms at batch 16, and the serving
  // headline -15%: the branch's queue competes with the copy streams), profiles/r1_branches_ab.md.
  bool branch_streams = false;
  // Run the PREP part (decode-table fetch, device decode, input prep) on the compute stream right
  // before MAIN instead of on the copy stream beside the previous batch's MAIN.
  bool prep_on_compute = false;
  // Each batch's result D2H (and data-parallel collectives) on a separate stream behind an event
  // after MAIN, instead of on the compute stream ahead of the next batch's MAIN.
  bool result_stream = true;
  // Measurement: force every conv/GEMM's XCD tile order (ConvArgs::order; 0 = autotuned heuristic,
  // 1 = N-fastest: each XCD owns the same row range in every layer, 2 = M-fastest).
  int conv_order = 0;
  // A batch runs the hipGraph of the smallest bucket >= B; with live_batch the kernels read B from
  // the slot's table and skip the work of the bucket's padding samples.
  bool live_batch = true;
  // Autotune results persist here across restarts (keyed by GPU arch + problem shape); "" = off,
  // "auto" = $DIE_TUNE_CACHE or ~/.cache/die_amd/tune.json.
  std::string tune_cache = "auto";
  // bf16 = HIP kernels (bf16 operands, fp32 accumulation); fp32 = CPU executor (device auto/cpu).
  std::string precision = "fp32";  // fp32 (reference parity; split bf16 MFMA on HIP) | bf16 (fast)
  int cpu_threads = 0;
  int shard_id = 0;
  // Data parallel (one process per GPU): dp_world ranks share the DpGroup segment
  // `dp_group`; rank 0 is the leader that owns the worker, ranks >= 1 run run_dp_follower().
  int dp_world = 0;
  int dp_rank = 0;
  std::string dp_group;
  size_t dp_arena_mb = 0;          // input arena size (0 = sized from the model)
  // How HIP ranks gather logits + decode status: "rccl" (ncclAllGather over xGMI, the default) or
  // "host" (through the DpGroup segment; no communicator, every rank loads the weights itself).
  std::string dp_backend = "rccl";
  // A group of one normally feeds its local engine directly (no merge loop, no communicator);
  // true keeps the N>1 path (sub-batch ring, leader merge, collectives) at world=1.
  bool dp_force_merge = false;
  Communicator* dp_comm = nullptr;  // set internally: RCCL communicator handed to the HIP engine

  // ---- HIP tuning knobs (round 2 kept these in DIE_* environment variables; every one is now an
  // option, echoed in the engine's stats()["options"] and the bench JSON) ----
  int copy_streams = 0;           // H2D copy streams (0 = auto: 2 with one executor, else 1)
  int bucket_div = 8;             // batch-bucket steps per octave above 16 (graphs for 18, 20, ..., 32)
  bool coarse_buckets = false;    // sqrt(2) bucket steps throughout (fewer graphs, faster cold start)
  double pace_lead_scale = 1.0;   // != 1: pacing lead = measured input time x this (< 1 dispatches later)
  int completion_poll_us = 0;     // > 0: sleep-poll each batch's D2H event instead of hipEventSynchronize
  bool bn_on_load = false;        // bf16 plans: next unit's BN+ReLU applied on the 1x1 conv operand load
  bool fuse_pairs = true;         // expand conv + next reduce conv -> one CONV_PAIR launch (kernels/conv_pair.hip)
  bool fuse_stem_pool = true;     // stem conv + max pool (+ its BN/ReLU) -> one launch (kernels/stem.hip)
  // global pool + the FC head reading it -> one launch (kernels/misc.hip gap_fc_kernel).  Off: at
  // ResNet50's head (B = 20) the fused kernel's slice hand-off is slower than GAP + split-K GEMM
  // (45.5 vs ~28.7 us, profiles/r4_gap_fc.md)
  bool fuse_gap_fc = false;
  // LayerNorm -> GEMM readers: statistics only, the normalisation in the GEMM epilogue (ViT-B/16
  // B=32: 5,143 -> 5,075 us per forward on one box, profiles/r4_fold_layernorm.md); fp32 mode only
  bool fold_layernorm = true;
  // ... and the statistics of a LayerNorm whose input a GEMM produces come from that GEMM's
  // epilogue (per-64-column partials, ConvArgs::stats_out / row_parts): no statistics launch
  bool ln_stats_epilogue = true;
  bool tune_cold = true;          // autotune with an L2 scrub before each timing (false: back-to-back)
  // after the isolated-launch autotune, time each conv's front runners in place inside eager
  // forwards (input warm from its producer, weights where the previous forward left them) and keep
  // the fastest (hip_engine.hip tune_in_graph)
  bool tune_in_graph = false;
  // autotune the XCD tile order too: the 2- and 4-panel orders (ConvArgs::order 3 / 4) next to the
  // heuristic, for convs that replicate their weights on every XCD (profiles/r5_xcd_panels.md)
  bool tune_orders = true;
  // autotune tail split-K too (ConvArgs::tail): whole tiles for the full 256-tile rounds, fused
  // split-K slices for the tiles of the last partial round only.  Off by default: behind the cold-L2
  // isolated timing it won 3 of ~1,200 ResNet/ViT shapes and left the per-batch-size forward time
  // unchanged (profiles/r5_batch_curve.md)
  bool tune_tail = false;
  // autotune stream-K candidates too (ConvArgs::sk: P = 256 / 512 / 1024 blocks split the tiles x
  // K-steps iterations evenly, cut tiles reduced in-kernel)
  bool tune_streamk = false;
  bool tune_warm_input = false;   // autotune: run each conv's input producer right before every timing
                                  // (measured no better than the scrub alone: profiles/r3_gemm_feed.md §7)
  // Split-K reductions run in-kernel (the last-arriving split block of a tile sums the partials and
  // runs the epilogue: kernels/conv_igemm_impl.h tile_epilogue).  true also lets the autotuner pick
  // the two-kernel form (partials, then splitk_epilogue_kernel: one more graph node per conv).
  bool splitk_two_kernel = false;
  // splitk_two_kernel only: take the fastest in-kernel (fused) split-K candidate when it is within
  // this fraction of the overall best
  float splitk_fused_margin = 0.f;
  // Efficient batch sizes (HIP, graphs): time the captured forward of every batch size once at
  // start-up; with Q requests queued, dispatch the largest B <= Q whose per-image device time is
  // within efficient_batch_tol of the best B' <= Q (ResNet50 fp32: B = 21 costs 19 % more than
  // B = 20 for 5 % more images, profiles/r5_batch_curve.md).  0 = the best itself: a bucket's
  // forward costs about the same at every live size, so that is a bucket's full size (20, 24, ...);
  // measured +2.9 % over 0.03, which let a batch of 25 run bucket 26's graph.
  // A batch is only cut below the queue when a smaller size is faster per image by more than
  // efficient_batch_margin (inside one bucket the curve is flat to within replay noise,
  // so the strict argmin let start-up noise decide whether requests wait a whole forward).
  // Measured (same-box A/B, profiles/r6_batch_policy.md): margin 0.02 and a median-of-groups curve
  // each let batches of 25 (a cheaper-looking bucket-26 graph) break the loop's 24-request rhythm and
  // cost ~4-5 % of the headline, so both stay opt-in and the round-5 strict rule is the default.
  bool efficient_batch = true;
  double efficient_batch_tol = 0.0;
  double efficient_batch_margin = 0.0;
  bool batch_curve_median = false;
  // cut only to bucket ends (the graph sizes), never to a partly empty bucket (pick_efficient_batch)
  bool efficient_batch_ends = true;
  // Fault injection: every Nth batch this engine runs fails before reaching the
  // device (0 = off).  Drives the data-parallel shard-failure tests.
  int fail_batch_every = 0;
};

// Every option as a JSON object (the /health "engine" document and bench.py echo it, so a run's
// configuration can be reconstructed from its output).
Json engine_options_json(const EngineOptions& o);

// EngineOptions::efficient_batch policy over a per-batch-size forward-time curve (ms[b], b = 1..
// max_b; ms[0] unused): with `queued` requests waiting, the batch size to dispatch.  Keeps the whole
// queue unless some smaller size is cheaper per image by more than `margin`; then the largest size
// within `tol` of the cheapest.  With `ends` (the engine's graph bucket sizes, ascending) only bucket
// ends are candidates -- the queue itself only when it is one -- so a batch never runs a bucket's
// graph partly empty (a batch of 25 on the 26-graph broke the serving loop's 24-request rhythm,
// profiles/r6_batch_policy.md).  Pure (CPU-tested through the C API).
int pick_efficient_batch(const double* ms, int max_b, int queued, double tol, double margin, const int* ends = nullptr,
                         int n_ends = 0);

// Factory: HIP engine when a GPU is visible and device != cpu, else the CPU executor (the
// reference's ORT CUDA-EP -> CPU-EP fallback, src/inference_engine.cpp:21-29, made explicit).
std::unique_ptr<Engine> create_engine(const std::string& model_path, const EngineOptions& opt);

std::unique_ptr<Engine> create_cpu_engine(const std::string& model_path, const EngineOptions& opt);
// Data-parallel leader (rank 0): creates the DpGroup, the communicator and the local engine, waits
// for the followers, and shards every submitted batch over the ranks.
std::unique_ptr<Engine> create_dp_engine(const std::string& model_path, const EngineOptions& opt);
// Shared input arena of a data-parallel group (engine/dp_engine.cpp): bytes per staged request,
// requests staged, total bytes (= the /dev/shm segment every rank maps and pins).
struct DpArenaPlan {
  size_t item_bytes = 0, items = 0, bytes = 0;
};
DpArenaPlan dp_arena_plan(size_t input_numel, const EngineOptions& opt, int world);
// Data-parallel follower (rank >= 1): attach, build the local engine on this process's GPU and
// serve shards until the leader stops the group or *stop becomes true.  Returns batches served.
long run_dp_follower(const std::string& model_path, const EngineOptions& opt, const std::atomic<bool>* stop);
// Defined in the HIP translation unit; returns nullptr (with `why` set) when no GPU is usable.
std::unique_ptr<Engine> create_hip_engine(const std::string& model_path, const EngineOptions& opt, std::string* why);
// The same for a model already in memory (`label` names it in stats / getModelPath).
std::unique_ptr<Engine> create_hip_engine_model(const std::string& label, onnx::Model model, const EngineOptions& opt,
                                                std::string* why);
// Hybrid HIP + CPU execution (engine/hybrid_engine.cpp), the reference's per-node execution-provider
// fallback (/root/reference/src/inference_engine.cpp:21-31: ORT places the nodes the CUDA EP cannot
// run on the CPU EP): the graph is cut at tensors that carry all live state, each piece runs on the
// HIP engine if the planner lowers it and it holds GEMM work, else on the CPU executor.
struct HybridSegment {
  bool hip = false;
  int first = 0, last = -1;        // node range [first, last] in the model's topological order
  std::string input, output;       // the cut tensors it reads / produces
  int convs = 0;                   // Conv / Gemm / MatMul nodes
  std::vector<int64_t> in_shape;   // per sample, batch dim = 1
};
std::vector<HybridSegment> hybrid_partition(const onnx::Model& m, int max_batch, bool split);
// nullptr when the graph needs no CPU island (or no GPU is usable: `why`).
std::unique_ptr<Engine> create_hybrid_engine(const std::string& model_path, const EngineOptions& opt, std::string* why);

}  // namespace die
