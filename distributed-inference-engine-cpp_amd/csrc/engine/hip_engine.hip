// HIP execution engine for MI355X (gfx950).
//
// Replaces the reference's ONNX Runtime session (src/inference_engine.cpp:16-87 construction,
// :134-209 batchPredict).  One engine owns one GPU:
//  * the ONNX graph is lowered once (hip_plan.cpp) to ~60 fused device ops; all packed weights
//    live in one device blob and all activations in one planned arena, both resident in HBM;
//  * request inputs are parsed by the HTTP layer straight into pinned host buffers handed out by
//    this engine (SamplePool backed by hipHostMalloc), so H2D is a DMA from the parse target;
//  * a batch runs on three streams: H2D copies, the forward (a hipGraph captured per batch
//    bucket and pipeline slot), D2H of the logits; `pipeline_depth` slots let batch k+1's copies
//    overlap batch k's forward;
//  * a completion thread waits for each slot's D2H event in FIFO order and runs the callback.
#include <pthread.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <chrono>
#include <condition_variable>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <sstream>
#include <cstring>
#include <deque>
#include <iostream>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "../kernels/kernels.h"
#include "engine.h"
#include "hip_plan.h"
#include "../core/log.h"
#include "../core/trace.h"
#include "../parallel/comm.h"

namespace die {

#define HIP_CHECK(expr)                                                                                     \
  do {                                                                                                      \
    hipError_t e_ = (expr);                                                                                 \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + " failed: " + hipGetErrorString(e_)); \
  } while (0)

namespace {

class HipEngine : public Engine {
 public:
  HipEngine(const std::string& path, const EngineOptions& opt) : HipEngine(path, onnx::load_onnx(path), opt) {}
  // `model` given in memory (a segment of a hybrid HIP + CPU partition); `path` labels it
  HipEngine(const std::string& path, onnx::Model model, const EngineOptions& opt) : path_(path), opt_(opt) {
    shard_id_ = opt.shard_id;
    dev_ = opt.device_id;
    HIP_CHECK(hipSetDevice(dev_));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, dev_));
    arch_ = prop.gcnArchName;
    if (arch_.find("gfx950") == std::string::npos)
      throw std::runtime_error("HIP engine is built for gfx950 (MI355X); device reports " + arch_);
    max_batch_ = std::max(1, opt.max_batch);
    depth_ = std::max(1, std::min(opt.pipeline_depth, 4));
    // fp32 (the reference's ORT numerics): split hi/lo bf16 operands on the matrix cores
    plan_ = build_plan(model, max_batch_, opt.branch_streams && opt.exec_streams <= 1, opt.precision == "fp32", opt.bn_on_load,
                       opt.fuse_pairs, opt.fuse_stem_pool, opt.fuse_gap_fc, opt.fold_layernorm,
                       opt.ln_stats_epilogue);
    sp_ = plan_.split ? 1 : 0;
    while (n_prep_ops_ < plan_.ops.size() && plan_.ops[n_prep_ops_].kind == PlanOp::INPUT_PREP) {
      prep_out_ids_.push_back(plan_.ops[n_prep_ops_].out);
      ++n_prep_ops_;
    }
    in_numel_ = plan_.input_numel;
    out_numel_ = plan_.output_numel;

    comm_ = opt.dp_comm;
    dp_world_ = comm_ ? comm_->world() : 1;
    HIP_CHECK(hipMalloc(&params_, std::max<size_t>(plan_.params.size(), 256)));
    // Executors: n_exec_ compute streams, each with its own activation arena, split-K workspace and
    // tile counters, so n_exec_ batches run on the GPU at once (slot s -> executor s % n_exec_).  At
    // serving batch sizes (~16) every conv is latency-bound and leaves most CUs idle; a second
    // batch in flight fills them.  Data-parallel ranks keep one (RCCL collectives in one order).
    n_exec_ = comm_ ? 1 : std::max(1, std::min({opt.exec_streams, depth_, kMaxExec}));
    arena_bytes_ = std::max<size_t>(plan_.arena_bytes, 256);
    for (int e = 0; e < n_exec_; ++e) {
      HIP_CHECK(hipMalloc(&arenas_[e], arena_bytes_));
      HIP_CHECK(hipStreamCreateWithFlags(&s_exec_[e], hipStreamNonBlocking));
    }
    s_compute_ = s_exec_[0];
    // Streams = hardware queues: the executor streams (graphs + the small result D2H) and copy
    // streams (early uploads, submit-time copies, PREP).  HIP gives a process GPU_MAX_HW_QUEUES
    // queues; more streams than that share queues (serialising copies behind kernels).  The engine
    // stays within four (1 executor + 2 copy streams [+ prep/side], or 2 + 1), and the serving
    // processes raise the limit to 8 (configure_hip_runtime_env) so that an RCCL communicator's
    // internal streams do not push the engine's onto shared queues (profiles/r3_rccl_hw_queues.md).
    // Two executors time-slice the compute queues instead of overlapping (forwards 1.8x longer).
    n_copy_streams_ = n_exec_ > 1 ? 1 : kStageStreams;
    if (opt.copy_streams > 0) n_copy_streams_ = std::min(kStageStreams, opt.copy_streams);
    for (int i = 0; i < n_copy_streams_; ++i) HIP_CHECK(hipStreamCreateWithFlags(&s_stage_[i], hipStreamNonBlocking));
    // side-branch stream (plan ops with join >= 0): the fourth and last queue; only with one executor
    branches_ = opt.branch_streams && n_exec_ == 1;
    // the fourth queue: side branches, or a dedicated PREP stream when texts are uploaded early
    if (!branches_ && n_exec_ == 1 && opt.device_decode && opt.stage_slots != 0 && !comm_)
      HIP_CHECK(hipStreamCreateWithFlags(&s_prep_, hipStreamNonBlocking));
    // Result stream: each batch's logits / status D2H (and, data parallel, its collectives) wait on
    // an event after MAIN instead of queueing on the compute stream, so the next batch's MAIN starts
    // right behind this one's (the copies are blit kernels that otherwise sit between two graphs).
    if (opt.result_stream) HIP_CHECK(hipStreamCreateWithFlags(&s_out_, hipStreamNonBlocking));
    prep_on_compute_ = opt.prep_on_compute;
    use_live_ = opt.live_batch;
    lead_scale_ = std::max(0.0, opt.pace_lead_scale);
    completion_poll_us_ = std::max(0, opt.completion_poll_us);
    if (branches_) {
      HIP_CHECK(hipStreamCreateWithFlags(&s_side_, hipStreamNonBlocking));
      HIP_CHECK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    }
    if (!comm_ || comm_->rank() == 0)
      HIP_CHECK(hipMemcpy(params_, plan_.params.data(), plan_.params.size(), hipMemcpyHostToDevice));
    if (comm_) {  // data parallel: every rank gets the packed weights from rank 0 over xGMI
      const auto tb = std::chrono::steady_clock::now();
      comm_->broadcast(params_, plan_.params.size(), 0, s_compute_);
      HIP_CHECK(hipStreamSynchronize(s_compute_));
      weight_bcast_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count();
      DIE_LOG(INFO, "dp rank " << comm_->rank() << ": weight broadcast " << plan_.params.size() / 1048576.0
                                     << " MiB in " << weight_bcast_ms_ << " ms (" << comm_->backend() << ")");
    }
    if (opt.device_decode) text_cap_ = (in_numel_ * 24 + 4095) / 4096 * 4096;  // up to 23 chars + separator per value
    if (text_cap_) {
      // One device text arena: n_stage_ early-upload slots (stage_text) followed by max_batch
      // fallback slots per pipeline slot (texts copied at submit).  Decode finds sample i at
      // offs[i].  Data-parallel ranks get their shards through the DP arena instead.
      n_stage_ = opt.stage_slots >= 0 ? opt.stage_slots : std::min(1024, std::max(256, 8 * max_batch_));
      if (comm_) n_stage_ = 0;
      HIP_CHECK(hipMalloc(&d_text_, text_cap_ * (static_cast<size_t>(n_stage_) + static_cast<size_t>(depth_) * max_batch_)));
      // 4-bit packed texts (BatchItem::packed; early-uploaded or copied at submit) land here, slot
      // for slot like d_text_; the decode kernels expand them in registers (no character copy in HBM).
      // Data-parallel ranks take packed texts too: the ingesting rank packs into the DP arena.
      if (opt.pack_text)
        HIP_CHECK(hipMalloc(&d_packed_, text_cap_ / 2 * (static_cast<size_t>(n_stage_) + static_cast<size_t>(depth_) * max_batch_)));
      stage_ev_.resize(n_stage_);
      stage_seq_.assign(n_stage_, 0);
      stage_packed_.assign(n_stage_, 0);
      stage_stream_.assign(n_stage_, 0);
      stage_state_.assign(n_stage_, kIssued);
      for (int t = 0; t < n_stage_; ++t) {
        HIP_CHECK(hipEventCreateWithFlags(&stage_ev_[t], hipEventDisableTiming));
        stage_free_.push_back(n_stage_ - 1 - t);
      }
    }
    slots_.resize(depth_);
    for (auto& sl : slots_) {
      if (text_cap_) HIP_CHECK(hipMalloc(&sl.d_scratch, kern::decode_scratch_bytes(max_batch_, text_cap_)));
      // [lens x max_batch][text offsets x max_batch][packed-text offsets x max_batch (-1 = raw)]
      HIP_CHECK(hipMalloc(&sl.d_lens, sizeof(long long) * table_len()));
      HIP_CHECK(hipMemset(sl.d_lens, 0xFF, sizeof(long long) * max_batch_));  // all -1: no text samples
      HIP_CHECK(hipMemset(sl.d_lens + max_batch_, 0, sizeof(long long) * max_batch_));
      HIP_CHECK(hipMemset(sl.d_lens + 2 * max_batch_, 0xFF, sizeof(long long) * max_batch_));
      HIP_CHECK(hipMalloc(&sl.d_status, sizeof(int) * status_len()));
      HIP_CHECK(hipMemset(sl.d_status, 0, sizeof(int) * status_len()));
      if (comm_) {
        HIP_CHECK(hipMalloc(&sl.d_gather, sizeof(float) * out_numel_ * max_batch_ * dp_world_));
        HIP_CHECK(hipMalloc(&sl.d_gstatus, sizeof(int) * status_len() * dp_world_));
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.h_gather), sizeof(float) * out_numel_ * max_batch_ * dp_world_,
                                hipHostMallocDefault));
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.h_gstatus), sizeof(int) * status_len() * dp_world_,
                                hipHostMallocDefault));
        HIP_CHECK(hipEventCreateWithFlags(&sl.ev_gather, hipEventDisableTiming));
      }
      // host-coherent: the graph's first kernel reads it directly (see encode_forward)
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.h_lens), sizeof(long long) * table_len(),
                              hipHostMallocCoherent | hipHostMallocMapped));
      HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&sl.h_lens_dev), sl.h_lens, 0));
      for (int i = 0; i < max_batch_; ++i) {  // no text samples until a submit says otherwise
        sl.h_lens[i] = -1;
        sl.h_lens[max_batch_ + i] = 0;
        sl.h_lens[2 * max_batch_ + i] = -1;
      }
      sl.h_lens[live_index()] = max_batch_;  // live batch: every sample of the bucket until a submit
      HIP_CHECK(hipMemcpy(sl.d_lens + live_index(), sl.h_lens + live_index(), sizeof(long long), hipMemcpyHostToDevice));
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.h_status), sizeof(int) * 2 * max_batch_, hipHostMallocDefault));
      HIP_CHECK(hipMalloc(&sl.d_in, sizeof(float) * in_numel_ * max_batch_));
      HIP_CHECK(hipMalloc(&sl.d_out, sizeof(float) * out_numel_ * max_batch_));
      HIP_CHECK(hipMemset(sl.d_in, 0, sizeof(float) * in_numel_ * max_batch_));
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.h_out), sizeof(float) * out_numel_ * max_batch_,
                              hipHostMallocDefault));
      for (auto& ev : sl.ev_h2d) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&sl.ev_d2h, hipEventDisableTiming | hipEventBlockingSync));
      HIP_CHECK(hipEventCreateWithFlags(&sl.ev_main, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&sl.ev_prep, hipEventDisableTiming));
      for (int id : prep_out_ids_) {
        void* pbuf = nullptr;
        HIP_CHECK(hipMalloc(&pbuf, std::max<size_t>(plan_.bufs[id].bytes_per_sample * max_batch_, 256)));
        sl.d_prep.push_back(pbuf);
      }
    }
    // Batch buckets ~sqrt(2) apart up to 16 (1, 2, 4, 6, 8, 12, 16), eighth steps above
    // (18, 20, ..., 32, 36, ...): a batch runs the graph of the smallest bucket >= B, and the
    // serving loop's batches (17-24 at the headline load) get kernels tuned within 2 of their size
    // (fp32 headline A/B: sqrt(2) steps 13.1-13.2k, quarter steps 13.6-13.7k, eighth steps
    // 13.9-14.1k req/s; profiles/r2_state.md).  EngineOptions::bucket_div = steps per octave above
    // 16; coarse_buckets: sqrt(2) steps throughout.
    const bool coarse = opt.coarse_buckets;
    const int fine = std::max(1, opt.bucket_div);
    for (int b = 1; b < max_batch_; b *= 2) {
      buckets_.push_back(b);
      if (b >= 16 && !coarse) {
        for (int q = 1; q < fine; ++q)
          if (b + q * b / fine < max_batch_) buckets_.push_back(b + q * b / fine);
      } else if (b >= 4 && b + b / 2 < max_batch_) {
        buckets_.push_back(b + b / 2);
      }
    }
    buckets_.push_back(max_batch_);
    est_ms_.assign(buckets_.size(), 0.0);

    pool_ = std::make_unique<SamplePool>(
        std::max(in_numel_, text_cap_ / sizeof(float)),
        [](size_t bytes) -> void* {
          void* p = nullptr;
          if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
          return p;
        },
        [](void* p) { (void)hipHostFree(p); }, 32);

    ws_bytes_ = kern::kSplitKWorkspaceBytes;  // split-K / GAP_FC partials (choose_splits / autotune stay within it)
    // zero page for the LDS-DMA conv loads: padding pixels and M-tail rows (a whole K row)
    size_t zeros_bytes = 4096;
    for (const PlanOp& op : plan_.ops)
      if (op.kind == PlanOp::CONV) zeros_bytes = std::max<size_t>(zeros_bytes, (static_cast<size_t>(op.conv.Kpad) + 64) * 2);
    HIP_CHECK(hipMalloc(&zeros_, zeros_bytes));
    HIP_CHECK(hipMemset(zeros_, 0, zeros_bytes));
    for (int e = 0; e < n_exec_; ++e) {
      HIP_CHECK(hipMalloc(&wss_[e], ws_bytes_));
      HIP_CHECK(hipMalloc(&counterss_[e], sizeof(int) * kCounters));  // fused split-K tile counters
      HIP_CHECK(hipMemset(counterss_[e], 0, sizeof(int) * kCounters));
    }
    if (branches_) {  // a branch running beside the main chain needs its own split-K scratch
      HIP_CHECK(hipMalloc(&ws_side_, ws_bytes_));
      HIP_CHECK(hipMalloc(&counters_side_, sizeof(int) * kCounters));
      HIP_CHECK(hipMemset(counters_side_, 0, sizeof(int) * kCounters));
    }
    ws_ = wss_[0];
    // Validate every op eagerly at the largest bucket, tune, then capture one graph per
    // (bucket, slot).
    for (int s = 0; s < depth_; ++s) encode_forward(max_batch_, s, s_compute_);
    HIP_CHECK(hipStreamSynchronize(s_compute_));
    if (opt.autotune) autotune();
    if (opt.use_graphs) {
      graphs_.assign(buckets_.size() * depth_, nullptr);
      prep_graphs_.assign(buckets_.size() * depth_, nullptr);
      auto capture = [&](int B, int s, Part part) {
        hipGraph_t g;
        HIP_CHECK(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
        encode_forward(B, s, s_compute_, nullptr, part);
        HIP_CHECK(hipStreamEndCapture(s_compute_, &g));
        hipGraphExec_t ge;
        HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        HIP_CHECK(hipGraphDestroy(g));
        return ge;
      };
      for (size_t bi = 0; bi < buckets_.size(); ++bi)
        for (int s = 0; s < depth_; ++s) {
          prep_graphs_[bi * depth_ + s] = capture(buckets_[bi], s, PREP);
          graphs_[bi * depth_ + s] = capture(buckets_[bi], s, MAIN);
        }
      HIP_CHECK(hipGraphLaunch(prep_graphs_.back(), s_compute_));
      // warm the graph path once
      HIP_CHECK(hipGraphLaunch(graphs_.back(), s_compute_));
      HIP_CHECK(hipStreamSynchronize(s_compute_));
      // (data parallel too: the leader's merge takes the local curve's sizes -- the MAIN graphs hold
      // no collectives, so each rank times its own forward)
      if (opt.efficient_batch && n_exec_ == 1) measure_batch_curve();
    }
    for (auto& e : tev_) HIP_CHECK(hipEventCreate(&e));
    completion_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "die-complete");
      completion_loop();
    });
    if (n_stage_)
      stager_ = std::thread([this] {
        pthread_setname_np(pthread_self(), "die-stager");
        stager_loop();
      });
  }

  ~HipEngine() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (completion_.joinable()) completion_.join();
    {
      std::lock_guard<std::mutex> g(stage_mu_);
      stage_stop_ = true;  // the stager drains its queue first (queued tickets still get issued)
    }
    stage_cv_.notify_all();
    if (stager_.joinable()) stager_.join();
    (void)hipSetDevice(dev_);
    (void)hipDeviceSynchronize();
    for (auto ge : graphs_)
      if (ge) (void)hipGraphExecDestroy(ge);
    for (auto ge : prep_graphs_)
      if (ge) (void)hipGraphExecDestroy(ge);
    for (auto ev : stage_ev_) (void)hipEventDestroy(ev);
    for (auto ev : tev_)
      if (ev) (void)hipEventDestroy(ev);
    for (auto st : s_stage_)
      if (st) (void)hipStreamDestroy(st);
    (void)hipFree(d_text_);
    (void)hipFree(d_packed_);
    for (auto& sl : slots_) {
      (void)hipFree(sl.d_in);
      (void)hipFree(sl.d_out);
      (void)hipFree(sl.d_scratch);
      (void)hipFree(sl.d_lens);
      (void)hipFree(sl.d_status);
      (void)hipHostFree(sl.h_lens);
      (void)hipHostFree(sl.h_status);
      if (comm_) {
        (void)hipFree(sl.d_gather);
        (void)hipFree(sl.d_gstatus);
        (void)hipHostFree(sl.h_gather);
        (void)hipHostFree(sl.h_gstatus);
        (void)hipEventDestroy(sl.ev_gather);
      }
      (void)hipHostFree(sl.h_out);
      for (auto ev : sl.ev_h2d) (void)hipEventDestroy(ev);
      (void)hipEventDestroy(sl.ev_d2h);
      (void)hipEventDestroy(sl.ev_main);
      (void)hipEventDestroy(sl.ev_prep);
      for (void* pbuf : sl.d_prep) (void)hipFree(pbuf);
    }
    pool_.reset();
    for (void* p : registered_) (void)hipHostUnregister(p);
    (void)hipFree(params_);
    (void)hipFree(zeros_);
    for (int e = 0; e < n_exec_; ++e) {
      (void)hipFree(arenas_[e]);
      (void)hipFree(wss_[e]);
      (void)hipFree(counterss_[e]);
      (void)hipStreamDestroy(s_exec_[e]);
    }
    if (s_prep_) (void)hipStreamDestroy(s_prep_);
    if (s_out_) (void)hipStreamDestroy(s_out_);
    if (branches_) {
      (void)hipFree(ws_side_);
      (void)hipFree(counters_side_);
      (void)hipEventDestroy(ev_fork_);
      (void)hipEventDestroy(ev_join_);
      (void)hipStreamDestroy(s_side_);
    }
  }

  std::string name() const override { return "hip:" + arch_ + ":" + std::to_string(dev_); }
  const std::string& getModelPath() const override { return path_; }
  std::vector<int64_t> getInputShape() const override { return plan_.input_shape; }
  std::vector<int64_t> getOutputShape() const override { return plan_.output_shape; }
  int max_batch() const override { return max_batch_; }
  SamplePool& sample_pool() override { return *pool_; }
  size_t text_capacity() const override { return text_cap_; }
  bool text_packing() const override { return d_packed_ != nullptr; }
  bool device_gather() const override { return comm_ != nullptr; }
  size_t register_host_memory(void* p, size_t bytes) override {
    HIP_CHECK(hipSetDevice(dev_));
    HIP_CHECK(hipHostRegister(p, bytes, hipHostRegisterDefault));
    registered_.push_back(p);
    return bytes;
  }

  // Early upload: reactor threads only queue the request; ONE stager thread issues every staged
  // copy (no HIP API traffic from the HTTP threads competing with the batcher's graph launches and
  // the completion thread's waits -- measured: issuing from 16 reactors cost ~15% throughput).
  long stage_text(const char* text, size_t len, bool packed) override {
    if (!text_cap_ || n_stage_ == 0 || len == 0 || len > text_cap_ || (packed && !d_packed_)) return -1;
    int t;
    {
      std::lock_guard<std::mutex> g(stage_mu_);
      if (stage_free_.empty() || stage_stop_) return -1;
      t = stage_free_.back();
      stage_free_.pop_back();
      stage_state_[t] = kQueued;
      stage_packed_[t] = packed;
      stage_q_.push_back(StageReq{t, text, len, packed});
    }
    stage_cv_.notify_one();
    staged_total_.fetch_add(1, std::memory_order_relaxed);
    return t;
  }

  void release_staged(long t, bool ran) override {
    if (t < 0 || t >= n_stage_) return;
    if (!ran) {  // the pinned source may be reused after this: wait for an unconsumed copy
      if (wait_staged(static_cast<int>(t)) == kIssued) {
        (void)hipSetDevice(dev_);
        (void)hipEventSynchronize(stage_ev_[t]);
      }
    }
    std::lock_guard<std::mutex> g(stage_mu_);
    stage_free_.push_back(static_cast<int>(t));
  }

  void wait_for_slot() override {
    std::unique_lock<std::mutex> lk(mu_);
    slot_cv_.wait(lk, [&] { return inflight_ < depth_ || stop_; });
  }

  void submit(std::vector<BatchItem> items, BatchDone done) override {
    const int B = static_cast<int>(items.size());
    if (B == 0) {
      BatchResult r;
      done(r);
      return;
    }
    if (B > max_batch_) {
      BatchResult r;
      r.ok = false;
      r.error = "batch of " + std::to_string(B) + " exceeds max_batch " + std::to_string(max_batch_);
      done(r);
      return;
    }
    std::lock_guard<std::mutex> submit_guard(submit_mu_);
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      slot_cv_.wait(lk, [&] { return inflight_ < depth_ || stop_; });
      if (stop_) {
        BatchResult r;
        r.ok = false;
        r.error = "engine stopped";
        done(r);
        return;
      }
      ++inflight_;
      slot = next_slot_;
      next_slot_ = (next_slot_ + 1) % depth_;
    }
    TraceRange tr_submit("engine.submit(h2d+graph)");
    {
      // paced dispatch that arrives after the predicted drain of the batch in flight: the GPU idled
      std::lock_guard<std::mutex> g(pace_mu_);
      if (pace_armed_) {
        pace_armed_ = false;
        const double late = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - pace_drain_).count();
        if (late > 0.03) margin_ms_ = std::min(margin_ms_ + 0.5 * late, 1.0);
      }
    }
    Job job;
    job.slot = slot;
    job.B = B;
    job.done = std::move(done);
    job.t0 = std::chrono::steady_clock::now();
    try {
      HIP_CHECK(hipSetDevice(dev_));
      if (opt_.fail_batch_every > 0 && ++nth_batch_ % opt_.fail_batch_every == 0)
        throw std::runtime_error("injected batch failure (fail_batch_every)");
      Slot& sl = slots_[slot];
      job.ev = static_cast<int>((job_seq_++ % kTimingJobs) * kEvPerJob);
      job.bi = static_cast<int>(bucket_index(B));
      HIP_CHECK(hipEventRecord(tev_[job.ev + 5], s_prep_ ? s_prep_ : s_stage_[0]));  // input path starts (pacing model)
      bool any_text = false;
      long long* h_offs = sl.h_lens + max_batch_;
      long long* h_poffs = sl.h_lens + 2 * max_batch_;
      int wait_ticket[kStageStreams];  // per copy stream, the staged copy issued last covers the earlier ones
      bool copied[kStageStreams] = {};  // submit-time copies issued on that stream
      for (auto& w : wait_ticket) w = -1;
      int rr = 0;
      for (int i = 0; i < B; ++i) {
        h_offs[i] = 0;
        h_poffs[i] = -1;
        if (items[i].text) {
          if (!text_cap_ || items[i].text_len > text_cap_) throw std::runtime_error("input text exceeds device decode capacity");
          if (items[i].packed && !d_packed_) throw std::runtime_error("engine does not take packed text");
          const long t = items[i].staged;
          const auto tw0 = std::chrono::steady_clock::now();
          const bool issued = t >= 0 && t < n_stage_ && wait_staged(static_cast<int>(t)) == kIssued;
          if (t >= 0) {
            diag_submit_wait_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tw0).count();
            if (issued && hipEventQuery(stage_ev_[t]) != hipSuccess) diag_not_ready_++;
          }
          if (issued) {  // already uploaded (raw, or packed: decoded straight from its packed slot)
            h_offs[i] = static_cast<long long>(t) * static_cast<long long>(text_cap_);
            if (stage_packed_[t]) h_poffs[i] = static_cast<long long>(t) * static_cast<long long>(text_cap_ / 2);
            int& w = wait_ticket[stage_stream_[t]];
            if (w < 0 || stage_seq_[t] > stage_seq_[w]) w = static_cast<int>(t);
          } else if (items[i].packed) {
            const size_t idx = static_cast<size_t>(n_stage_) + static_cast<size_t>(slot) * max_batch_ + i;
            h_offs[i] = static_cast<long long>(idx * text_cap_);
            h_poffs[i] = static_cast<long long>(idx * (text_cap_ / 2));
            const int si = rr++ % n_copy_streams_;
            HIP_CHECK(hipMemcpyAsync(d_packed_ + idx * (text_cap_ / 2), items[i].text, (items[i].text_len + 1) / 2,
                                     hipMemcpyHostToDevice, s_stage_[si]));
            h2d_bytes_.fetch_add(static_cast<long long>((items[i].text_len + 1) / 2), std::memory_order_relaxed);
            copied[si] = true;
          } else {
            const size_t idx = static_cast<size_t>(n_stage_) + static_cast<size_t>(slot) * max_batch_ + i;
            h_offs[i] = static_cast<long long>(idx * text_cap_);
            const int si = rr++ % n_copy_streams_;
            HIP_CHECK(hipMemcpyAsync(d_text_ + idx * text_cap_, items[i].text, items[i].text_len, hipMemcpyHostToDevice,
                                     s_stage_[si]));
            h2d_bytes_.fetch_add(static_cast<long long>(items[i].text_len), std::memory_order_relaxed);
            copied[si] = true;
          }
          sl.h_lens[i] = static_cast<long long>(items[i].text_len);
          any_text = true;
          continue;
        }
        sl.h_lens[i] = -1;
        const size_t n = std::min(items[i].len, in_numel_);
        float* dst = sl.d_in + static_cast<size_t>(i) * in_numel_;
        const int si = rr++ % n_copy_streams_;
        if (n) HIP_CHECK(hipMemcpyAsync(dst, items[i].input, n * sizeof(float), hipMemcpyHostToDevice, s_stage_[si]));
        h2d_bytes_.fetch_add(static_cast<long long>(n * sizeof(float)), std::memory_order_relaxed);
        if (n < in_numel_) HIP_CHECK(hipMemsetAsync(dst + n, 0, (in_numel_ - n) * sizeof(float), s_stage_[si]));
        copied[si] = true;
      }
      sl.h_lens[live_index()] = use_live_ ? B : max_batch_;
      for (int i = B; i < max_batch_; ++i) {
        sl.h_lens[i] = -1;
        h_offs[i] = 0;
        h_poffs[i] = -1;
      }
      job.has_text = any_text;
      size_t bi = 0;
      while (buckets_[bi] < B) ++bi;
      // PREP (decode-table fetch from host-coherent memory, device decode, input prep) runs on copy
      // stream 0 behind this batch's copies, overlapping the previous batch's MAIN on the compute
      // stream; MAIN waits for it.  Timing events come from a ring (a job's events outlive its slot's
      // reuse): pre = compute stream done with earlier work, fwd0/fwd1 around MAIN, p0/p1 around PREP.
      // PREP runs on its own stream when there is one (early upload: the stager's copies for later
      // batches must not queue behind this batch's decode on a copy stream), else on copy stream 0
      hipStream_t ps = s_prep_ ? s_prep_ : s_stage_[0];
      hipStream_t cs = s_exec_[slot % n_exec_];
      for (int si = s_prep_ ? 0 : 1; si < kStageStreams; ++si)
        if (copied[si]) {
          HIP_CHECK(hipEventRecord(sl.ev_h2d[si], s_stage_[si]));
          HIP_CHECK(hipStreamWaitEvent(ps, sl.ev_h2d[si], 0));
        }
      bool used_staged = false;
      for (int w : wait_ticket)
        if (w >= 0) {
          HIP_CHECK(hipStreamWaitEvent(ps, stage_ev_[w], 0));
          used_staged = true;
        }
      if (used_staged) staged_used_.fetch_add(1, std::memory_order_relaxed);
      HIP_CHECK(hipEventRecord(tev_[job.ev + 6], ps));  // all input copies landed
      if (prep_on_compute_) {
        // PREP in line on the compute stream, after the previous MAIN: only the copies need lead
        HIP_CHECK(hipEventRecord(sl.ev_prep, ps));
        HIP_CHECK(hipEventRecord(tev_[job.ev], cs));
        HIP_CHECK(hipStreamWaitEvent(cs, sl.ev_prep, 0));
        ps = cs;
      }
      HIP_CHECK(hipEventRecord(tev_[job.ev + 3], ps));
      if (!prep_graphs_.empty()) {
        HIP_CHECK(hipGraphLaunch(prep_graphs_[bi * depth_ + slot], ps));
        graph_replays_.fetch_add(1, std::memory_order_relaxed);
      } else {
        encode_forward(buckets_[bi], slot, ps, nullptr, PREP);
      }
      HIP_CHECK(hipEventRecord(tev_[job.ev + 4], ps));
      if (!prep_on_compute_) {
        HIP_CHECK(hipEventRecord(sl.ev_prep, ps));
        HIP_CHECK(hipEventRecord(tev_[job.ev], cs));
        HIP_CHECK(hipStreamWaitEvent(cs, sl.ev_prep, 0));
      }
      HIP_CHECK(hipEventRecord(tev_[job.ev + 1], cs));
      if (!graphs_.empty()) {
        HIP_CHECK(hipGraphLaunch(graphs_[bi * depth_ + slot], cs));
        graph_replays_.fetch_add(1, std::memory_order_relaxed);
      } else {
        encode_forward(buckets_[bi], slot, cs, nullptr, MAIN);
      }
      HIP_CHECK(hipEventRecord(tev_[job.ev + 2], cs));
      if (comm_) {
        // this rank's shard ran: its flag travels with the status rows, so the other ranks answer
        // this shard's items from the gathered rows (flag 0: they fail them; see the catch below)
        HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sl.d_status + rank_ok_index()), 1, 1, cs));
        dp_collectives(sl, B, result_stream(sl, cs));
        job.has_text = text_cap_ > 0;
      } else {
        hipStream_t os = result_stream(sl, cs);
        HIP_CHECK(hipMemcpyAsync(sl.h_out, sl.d_out, sizeof(float) * out_numel_ * B, hipMemcpyDeviceToHost, os));
        d2h_bytes_.fetch_add(static_cast<long long>(sizeof(float) * out_numel_ * B), std::memory_order_relaxed);
        if (any_text) {
          HIP_CHECK(hipMemcpyAsync(sl.h_status, sl.d_status, sizeof(int) * 2 * max_batch_, hipMemcpyDeviceToHost, os));
          d2h_bytes_.fetch_add(static_cast<long long>(sizeof(int) * 2 * max_batch_), std::memory_order_relaxed);
        }
        HIP_CHECK(hipEventRecord(sl.ev_d2h, os));
      }
    } catch (const std::exception& e) {
      job.error = e.what();
      if (comm_ && !dp_issued_) {
        // The other ranks' collectives are waiting for this rank's: issue them anyway with the
        // shard flag cleared (a rank that skipped them would hang the whole group), so they fail
        // this shard's items and answer the rest.
        try {
          Slot& sl = slots_[slot];
          hipStream_t cs = s_exec_[slot % n_exec_];
          HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sl.d_status + rank_ok_index()), 0, 1, cs));
          dp_collectives(sl, B, result_stream(sl, cs));
          job.dp_gathered = true;
          job.has_text = text_cap_ > 0;
        } catch (const std::exception&) {
        }
      }
    }
    dp_issued_ = false;
    diag_submit_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - job.t0).count();
    {
      std::lock_guard<std::mutex> g(mu_);
      if (job.error.empty()) {
        last_ev_ = job.ev;
        last_bi_ = job.bi;
      }
      jobs_.push_back(std::move(job));
      ++callbacks_running_;
    }
    cv_.notify_all();
  }

  // Just-in-time dispatch.  With the GPU busy on batch k, dispatching batch k+1 as soon as a slot
  // frees makes it carry only what queued during k's submit; holding it until k is about to drain
  // lets it absorb the requests that arrive meanwhile (bigger batches, better MFMA occupancy).
  // Estimate: k's MAIN start (observed through its event) + the EMA device time of k's bucket - lead,
  // where lead (next batch's copies + prep) adapts to the GPU idle time measured before each MAIN.
  std::chrono::steady_clock::time_point dispatch_not_before() override {
    using clk = std::chrono::steady_clock;
    const auto now = clk::now();
    if (!opt_.pace || n_exec_ > 1 || graphs_.empty()) return now;
    int ev, bi;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (inflight_ == 0 || last_ev_ < 0) return now;
      ev = last_ev_;
      bi = last_bi_;
    }
    double est, lead, in_ms;
    {
      std::lock_guard<std::mutex> g(pace_mu_);
      est = est_ms_[bi];
      lead = lead_ms_;
      in_ms = input_ms_;
    }
    if (est <= 0.0 || est <= lead) return now;
    (void)hipSetDevice(dev_);
    const auto give_up = now + std::chrono::milliseconds(20);
    hipError_t q;
    while ((q = hipEventQuery(tev_[ev + 1])) == hipErrorNotReady) {  // k's MAIN has not started yet
      if (clk::now() > give_up) return clk::now();
      std::this_thread::sleep_for(std::chrono::microseconds(15));
    }
    if (q != hipSuccess || hipEventQuery(tev_[ev + 2]) != hipErrorNotReady) return clk::now();  // k drained
    const auto t0 = clk::now();
    const auto drain = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double, std::milli>(est));
    const auto t = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double, std::milli>(est - (lead_scale_ == 1.0 ? lead : in_ms * lead_scale_)));
    {
      std::lock_guard<std::mutex> g(pace_mu_);
      pace_drain_ = drain;
      pace_armed_ = true;
    }
    paced_batches_++;
    return t;
  }

  // EngineOptions::efficient_batch: the largest B <= queued whose per-image device time (the
  // start-up curve) is within efficient_batch_tol of the best B' <= queued.  Per-image time falls
  // with B except where a layer's tile grid spills into one more round of blocks (ResNet50 fp32:
  // 61.6 us per image at B = 20, 69.6 at 21, profiles/r5_batch_curve.md), so this only ever cuts a
  // batch back to just below such a step; the requests left over lead the next batch.
  // A cut needs a smaller size cheaper per image by more than efficient_batch_margin (inside a
  // bucket the curve is flat to within replay noise).
  int preferred_batch(int queued) const override {
    return pick_efficient_batch(batch_ms_.empty() ? nullptr : batch_ms_.data(), max_batch_, queued,
                                opt_.efficient_batch_tol, opt_.efficient_batch_margin,
                                opt_.efficient_batch_ends ? buckets_.data() : nullptr, static_cast<int>(buckets_.size()));
  }

  void synchronize() override {
    std::unique_lock<std::mutex> lk(mu_);
    slot_cv_.wait(lk, [&] { return inflight_ == 0 && callbacks_running_ == 0; });
  }

  Json stats() const override {
    Json j = Json::object();
    j["device"] = name();
    j["batches"] = static_cast<long long>(batches_.load());
    j["images"] = static_cast<long long>(images_.load());
    const long long nb = batches_.load();
    j["avg_device_ms"] = nb ? device_ms_total_.load() / nb : 0.0;
    // per-GPU I/O and activity counters
    j["device_id"] = dev_;
    j["h2d_bytes"] = h2d_bytes_.load();
    j["d2h_bytes"] = d2h_bytes_.load();
    j["graph_replays"] = graph_replays_.load();
    j["device_busy_ms"] = device_ms_total_.load();
    // per batch: compute stream waiting for the batch's PREP (copies + decode) / idle before it was submitted
    j["avg_copy_wait_ms"] = nb ? copy_wait_ms_total_.load() / nb : 0.0;
    j["avg_gpu_gap_ms"] = nb ? gpu_gap_ms_total_.load() / nb : 0.0;
    j["avg_prep_ms"] = nb ? prep_ms_total_.load() / nb : 0.0;  // decode + input prep, on the copy stream
    j["options"] = engine_options_json(opt_);
    j["pace"] = opt_.pace && n_exec_ == 1 && !comm_ && !graphs_.empty();
    j["pack_text"] = d_packed_ != nullptr;
    j["branch_streams"] = branches_;
    j["prep_on_compute"] = prep_on_compute_;
    j["completion_poll_us"] = completion_poll_us_;
    j["live_batch"] = use_live_;
    j["paced_batches"] = static_cast<long long>(paced_batches_.load());
    {
      std::lock_guard<std::mutex> g(pace_mu_);
      j["avg_pace_lead_ms"] = nb ? lead_ms_total_ / nb : 0.0;
      j["pace_input_ms"] = input_ms_;
      j["pace_margin_ms"] = margin_ms_;
    }
    j["hip_graphs"] = !graphs_.empty();
    j["efficient_batch"] = !batch_ms_.empty();
    if (!batch_ms_.empty()) {
      Json c = Json::array();  // device ms of the captured forward at batch 1, 2, ..., max_batch
      for (size_t b = 1; b < batch_ms_.size(); ++b) c.push_back(batch_ms_[b]);
      j["batch_curve_ms"] = c;
    }
    j["pipeline_depth"] = depth_;
    j["executors"] = n_exec_;
    j["copy_streams"] = n_copy_streams_;
    j["plan"] = plan_.summary();
    j["precision"] = sp_ ? "fp32" : "bf16";
    j["gflop_per_image"] = plan_.flops_per_sample / 1e9;
    j["arena_mib"] = static_cast<double>(plan_.arena_bytes) / (1 << 20);
    j["pinned_samples"] = static_cast<long long>(pool_->allocated());
    j["device_decode"] = text_cap_ > 0;
    j["dp_rank"] = comm_ ? comm_->rank() : 0;
    j["dp_weight_broadcast_ms"] = weight_bcast_ms_;
    j["dp_collective_ops"] = dp_collective_ops_.load();
    j["text_capacity"] = static_cast<long long>(text_cap_);
    j["stage_slots"] = n_stage_;
    j["staged_uploads"] = staged_total_.load();
    j["batches_with_staged"] = staged_used_.load();
    {
      const long long st = std::max<long long>(1, staged_total_.load());
      Json d = Json::object();
      d["stager_issue_us_avg"] = diag_issue_ns_.load() / 1e3 / st;
      d["submit_wait_us_avg"] = diag_submit_wait_ns_.load() / 1e3 / st;
      d["staged_not_ready_at_submit"] = diag_not_ready_.load();
      d["submit_us_avg"] = diag_submit_ns_.load() / 1e3 / std::max<long long>(1, batches_.load());
      j["staging_diag"] = d;
    }
    j["autotuned"] = !tune_.empty();
    j["tuned_conv_us_at_max_batch"] = tuned_conv_us_;
    j["tune_in_graph_timed"] = in_graph_timed_;      // candidates timed in place (EngineOptions::tune_in_graph)
    j["tune_in_graph_changed"] = in_graph_changed_;  // convs whose in-place winner differs from the isolated one
    j["tune_cache_entries_loaded"] = tune_cache_hits_;
    if (!tune_.empty()) {
      Json t = Json::array();
      for (size_t oi = 0; oi < plan_.ops.size(); ++oi)
        if (plan_.ops[oi].kind == PlanOp::CONV) {
          const Tune& x = tune_.back()[oi];
          t.push_back(std::to_string(x.tile) + "/" + std::to_string(x.splits) + (x.fused ? "f" : "") +
                      (x.order == 2 ? "m" : x.order == 1 ? "n" : "") + (x.tail ? "t" : "") +
                      (x.sk ? "k" + std::to_string(x.sk) : ""));
        }
      j["tile_split_at_max_batch"] = t;
    }
    return j;
  }

  struct Tune {
    int tile = 0;
    int splits = 1;
    bool fused = false;  // split-K reduced in-kernel by the last split block (else a second kernel)
    int order = 0;       // ConvArgs::order (0 heuristic, 1 N-fastest, 2 M-fastest)
    int tail = 0;        // ConvArgs::tail (> 0: split-K on the last partial round's tiles only)
    int sk = 0;          // ConvArgs::sk (> 0: stream-K launch of sk blocks; splits/tail unused)
  };

  // ---- autotune persistence (kernel configs cached in a tuning file) ----
  std::string tune_cache_path() const {
    std::string p = opt_.tune_cache;
    if (p == "auto") {  // (the Python layer resolves $DIE_TUNE_CACHE before it gets here)
      if (const char* h = std::getenv("HOME")) p = std::string(h) + "/.cache/die_amd/tune.json";
      else p.clear();
    }
    return p;
  }
  size_t load_tune_cache(const std::string& path, std::map<std::string, std::pair<Tune, double>>& out) const {
    if (path.empty()) return 0;
    std::ifstream f(path);
    if (!f) return 0;
    try {
      std::stringstream ss;
      ss << f.rdbuf();
      const Json j = Json::parse(ss.str());
      const Json* arch = j.find(arch_);
      if (!arch) return 0;
      for (const auto& kv : arch->as_object()) {
        const auto& a = kv.second.as_array();
        if (a.size() < 4) continue;
        out[kv.first] = {Tune{static_cast<int>(a[0].as_int()), static_cast<int>(a[1].as_int()), a[2].as_bool(),
                              a.size() > 4 ? static_cast<int>(a[4].as_int()) : 0,
                              a.size() > 5 ? static_cast<int>(a[5].as_int()) : 0,
                              a.size() > 6 ? static_cast<int>(a[6].as_int()) : 0},
                         a[3].as_double()};
      }
    } catch (const std::exception&) {
      return 0;  // unreadable cache: retune
    }
    return out.size();
  }
  void save_tune_cache(const std::string& path, const std::map<std::string, std::pair<Tune, double>>& shapes) const {
    if (path.empty()) return;
    try {
      Json root = Json::object();
      {
        std::ifstream f(path);
        if (f) {
          std::stringstream ss;
          ss << f.rdbuf();
          root = Json::parse(ss.str());
        }
      }
      Json arch = root.find(arch_) ? *root.find(arch_) : Json::object();
      for (const auto& kv : shapes) {
        Json a = Json::array();
        a.push_back(kv.second.first.tile);
        a.push_back(kv.second.first.splits);
        a.push_back(kv.second.first.fused);
        a.push_back(kv.second.second);
        a.push_back(kv.second.first.order);
        a.push_back(kv.second.first.tail);
        a.push_back(kv.second.first.sk);
        arch[kv.first] = a;
      }
      root[arch_] = arch;
      const auto slash = path.rfind('/');
      if (slash != std::string::npos) {  // no shell: this process owns a GPU context
        std::error_code ec;
        std::filesystem::create_directories(path.substr(0, slash), ec);
      }
      const std::string tmp = path + ".tmp" + std::to_string(getpid());
      {
        std::ofstream o(tmp);
        o << root.dump();
      }
      std::rename(tmp.c_str(), path.c_str());
    } catch (const std::exception&) {
    }
  }

  void* buf_ptr(int id, int s) {
    Slot& sl = slots_[s];
    if (id == -2) return sl.d_in;
    if (id == -3) return sl.d_out;
    if (id < 0) return nullptr;
    for (size_t k = 0; k < prep_out_ids_.size(); ++k)
      if (prep_out_ids_[k] == id) return sl.d_prep[k];
    return arenas_[s % n_exec_] + plan_.bufs[id].offset;
  }
  const float* prm_ptr(size_t off) const {
    return off == SIZE_MAX ? nullptr : reinterpret_cast<const float*>(params_ + off);
  }

  kern::ConvArgs conv_args(const PlanOp& op, int B, int s) {
    kern::ConvArgs a = op.conv;
    a.B = B;
    a.M = B * a.Ho * a.Wo;
    a.x = static_cast<const uint16_t*>(buf_ptr(op.in, s));
    a.w = reinterpret_cast<const uint16_t*>(params_ + op.w_off);
    a.bias = prm_ptr(op.bias_off);
    a.res = static_cast<const uint16_t*>(buf_ptr(op.in2, s));
    a.out = static_cast<uint16_t*>(buf_ptr(op.out, s));
    a.out_f32 = static_cast<float*>(buf_ptr(op.out_f32, s));
    a.scale2 = prm_ptr(op.s2_off);
    a.shift2 = prm_ptr(op.b2_off);
    a.out2 = static_cast<uint16_t*>(buf_ptr(op.out2, s));
    a.zeros = zeros_;
    a.counters = counterss_[s % n_exec_];
    a.counters_n = kCounters;
    a.live = slots_[s].d_lens + live_index();
    a.in_scale = prm_ptr(op.in_scale_off);
    a.in_shift = prm_ptr(op.in_shift_off);
    a.in_relu = op.in_relu;
    const float* in3 = op.in3 >= 0 ? static_cast<const float*>(buf_ptr(op.in3, s)) : nullptr;
    a.row_stats = op.in3_parts ? nullptr : in3;
    a.row_parts = op.in3_parts ? in3 : nullptr;
    a.ln_eps = op.eps;
    a.stats_out = op.out_stats >= 0 ? static_cast<float*>(buf_ptr(op.out_stats, s)) : nullptr;
    a.col_sum = prm_ptr(op.colsum_off);
    return a;
  }

  // Device time of the captured forward at every batch size 1..max_batch (EngineOptions::
  // efficient_batch): slot 0's MAIN graph of the batch's bucket with the live count set to B, one
  // warm-up and three timed back-to-back replays (the serving loop runs graphs back to back), or
  // (EngineOptions::batch_curve_median) the median of three such groups.
  void measure_batch_curve() {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    Slot& sl = slots_[0];
    long long* lv = sl.h_lens + live_index();
    batch_ms_.assign(static_cast<size_t>(max_batch_) + 1, 0.0);
    for (int b = 1; b <= max_batch_; ++b) {
      hipGraphExec_t g = graphs_[bucket_index(b) * static_cast<size_t>(depth_)];
      *lv = use_live_ ? b : max_batch_;
      HIP_CHECK(hipMemcpyAsync(sl.d_lens + live_index(), lv, sizeof(long long), hipMemcpyHostToDevice, s_compute_));
      HIP_CHECK(hipGraphLaunch(g, s_compute_));
      if (opt_.batch_curve_median) {  // median of three groups of three replays
        float grp[3];
        for (float& ms : grp) {
          HIP_CHECK(hipEventRecord(e0, s_compute_));
          for (int r = 0; r < 3; ++r) HIP_CHECK(hipGraphLaunch(g, s_compute_));
          HIP_CHECK(hipEventRecord(e1, s_compute_));
          HIP_CHECK(hipEventSynchronize(e1));
          HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        }
        std::sort(grp, grp + 3);
        batch_ms_[static_cast<size_t>(b)] = grp[1] / 3.0;
      } else {  // the mean of three replays right behind the warm-up (round 5)
        float ms = 0.f;
        HIP_CHECK(hipEventRecord(e0, s_compute_));
        for (int r = 0; r < 3; ++r) HIP_CHECK(hipGraphLaunch(g, s_compute_));
        HIP_CHECK(hipEventRecord(e1, s_compute_));
        HIP_CHECK(hipEventSynchronize(e1));
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        batch_ms_[static_cast<size_t>(b)] = ms / 3.0;
      }
    }
    *lv = max_batch_;
    HIP_CHECK(hipMemcpyAsync(sl.d_lens + live_index(), lv, sizeof(long long), hipMemcpyHostToDevice, s_compute_));
    HIP_CHECK(hipStreamSynchronize(s_compute_));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }

  size_t bucket_index(int B) const {
    size_t bi = 0;
    while (bi + 1 < buckets_.size() && buckets_[bi] < B) ++bi;
    return bi;
  }

  Tune tune_for(int B, size_t op_index) const {
    const size_t bi = bucket_index(B);
    if (bi < tune_.size() && op_index < tune_[bi].size() && tune_[bi][op_index].tile >= 0) return tune_[bi][op_index];
    const PlanOp& op = plan_.ops[op_index];
    const int M = B * op.conv.Ho * op.conv.Wo;
    Tune t;
    t.tile = kern::choose_tile(M, op.conv.N, op.conv.K);
    t.splits = kern::choose_splits(M, op.conv.N, op.conv.K, t.tile);
    t.fused = t.splits > 1 && !opt_.splitk_two_kernel;
    return t;
  }

  // Time every (tile, split-K) candidate of every conv at every bucket and keep the fastest.
  // Runs once at start-up on the real buffers (a full forward first, so inputs hold real data).
  // Autotune every conv/GEMM at every bucket.  Candidates are timed one launch at a time behind
  // an L2 scrub (EngineOptions::tune_cold = false: back-to-back launches instead): inside a forward a layer reads
  // its input just written by the previous layer and its weights from the Infinity Cache, never a
  // warm L2 -- warm back-to-back timing favoured shallow LDS rings whose load latency is exposed
  // once the operands come from further away (stage-3 3x3 convs: 17.5 us tuned, 27 us in the graph).
  // Tune-cache / memo key of a conv problem: the shape, its epilogue, and the tuning regime.
  std::string shape_key(const kern::ConvArgs& base, bool warm_input) const {
    char key[256];
    std::snprintf(key, sizeof(key), "o%s%s%s%s%s%s%s%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d", opt_.tune_streamk ? "k:" : "",
                  opt_.tune_tail ? "t:" : "",
                  opt_.tune_cold ? "c:" : "",
                  warm_input ? "w:" : "", sp_ ? "f32:" : "", base.stats_out || base.row_parts ? "ls:" : "",
                  opt_.splitk_two_kernel ? (opt_.splitk_fused_margin > 0.f ? "fm:" : "sk2:") : (opt_.tune_orders ? "" : "o0:"),
                  base.M, base.N, base.K, base.Cin, base.H, base.W, base.KH, base.KW, base.stride, base.pad_h, base.relu,
                  base.res != nullptr, base.out2 != nullptr, base.out_f32 != nullptr, base.out != nullptr);
    return key;
  }

  void autotune() {
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    const bool cold = opt_.tune_cold;
    constexpr size_t kScrubBytes = 96u << 20;
    void* scrub = nullptr;
    float* sink = nullptr;
    if (cold) {
      HIP_CHECK(hipMalloc(&scrub, kScrubBytes));
      HIP_CHECK(hipMemset(scrub, 0, kScrubBytes));
      HIP_CHECK(hipMalloc(&sink, sizeof(float)));
    }
    tune_.assign(buckets_.size(), std::vector<Tune>(plan_.ops.size(), Tune{-1, 1}));
    double total_best_us = 0;
    std::map<std::string, std::pair<Tune, double>> tuned_shapes;
    const std::string cache_path = tune_cache_path();
    const size_t loaded = load_tune_cache(cache_path, tuned_shapes);
    for (size_t bi = 0; bi < buckets_.size(); ++bi) {
      const int B = buckets_[bi];
      encode_forward(B, 0, s_compute_);
      HIP_CHECK(hipStreamSynchronize(s_compute_));
      for (size_t oi = 0; oi < plan_.ops.size(); ++oi) {
        const PlanOp& op = plan_.ops[oi];
        if (op.kind != PlanOp::CONV) continue;
        kern::ConvArgs base = conv_args(op, B, 0);
        base.ws = ws_;
        base.live = nullptr;  // tune the whole bucket
        // EngineOptions::tune_warm_input: the op that produced this conv's input runs right before
        // every timed launch (after the L2 scrub), so the candidate reads its input warm from the
        // producer and its weights cold -- as inside a forward
        int producer = -1;
        if (opt_.tune_warm_input)
          for (int j = static_cast<int>(oi) - 1; j >= 0 && producer < 0; --j) {
            const PlanOp& q = plan_.ops[static_cast<size_t>(j)];
            if ((q.out >= 0 && q.out == op.in) || (q.out2 >= 0 && q.out2 == op.in) || (q.out3 >= 0 && q.out3 == op.in))
              producer = j;
          }
        // identical problems (repeated blocks) share one measurement
        const std::string key = shape_key(base, producer >= 0);
        auto memo = tuned_shapes.find(key);
        // (a cached result without this run's candidate list is re-measured when the in-graph pass
        // needs the front runners -- unless that pass's own results are cached too)
        if (memo != tuned_shapes.end() && (!opt_.tune_in_graph || cands_.count(key) || in_graph_cached(tuned_shapes, B))) {
          tune_[bi][oi] = memo->second.first;
          if (B == max_batch_) total_best_us += memo->second.second;
          continue;
        }
        const int nk = base.Kpad / 64;
        float best = 1e30f, best_fused = 1e30f;
        Tune bt{kern::choose_tile(base.M, base.N, base.K), 1}, bt_fused = bt;
        std::vector<std::pair<float, Tune>> measured;  // every valid candidate (in-graph retune)
        for (int tile = 0; tile < kern::NUM_CFGS; ++tile) {
          for (int sp = 1; sp <= 16; sp *= 2) {
            if (sp > 1 && (base.N % 8 || sp > nk || kern::splitk_workspace_bytes(base.M, base.N, sp) > ws_bytes_)) break;
            // split-K candidates reduce in-kernel unless the two-kernel form is allowed
            for (int fused = sp > 1 && !opt_.splitk_two_kernel ? 1 : 0; fused < (sp > 1 ? 2 : 1); ++fused)
            // Tile order: the heuristic (ConvArgs::order 0; tuning N- vs M-fastest per shape picked
            // M-fastest for ~30 % of shapes behind a cold L2 but made the in-graph forwards 1-2 %
            // slower, profiles/r3_gemm_feed.md section 6), plus -- where the heuristic replicates the
            // weights on every XCD, there are >= 4 N-tiles and the activations are at most 3x the
            // weights (a panel order reads every activation row once per panel: ViT's MLP2, 8x,
            // won in isolation and lost 16 % in the graph) -- the 2- and 4-panel orders, whose
            // XCDs each read one panel of the weights (profiles/r5_xcd_panels.md)
            for (int order : {0, 3, 4})
            // Tail split-K (ConvArgs::tail = 256, one tile per CU per round): next to each fused
            // split-K candidate of an LDS-DMA config, heuristic order, when the tile grid spills a
            // few tiles (at most 160) past a whole number of 256-tile rounds -- the steps of the
            // per-batch-size forward time (profiles/r5_batch_curve.md)
            for (int tail : {0, 256}) {
              if (tail > 0) {
                int bm, bn;
                kern::tile_dims(tile, bm, bn);
                const int T = ((base.M + bm - 1) / bm) * ((base.N + bn - 1) / bn);
                const int v = tile / kern::NUM_TILES;
                if (!opt_.tune_tail || !fused || order != 0 || v == 0 || v >= 6 || T <= tail || T % tail == 0 ||
                    T % tail > 160)
                  continue;
              }
              if (order > 0 && !opt_.tune_orders) continue;
              if (order > 0) {
                int bm, bn;
                kern::tile_dims(tile, bm, bn);
                const long long wts = static_cast<long long>(base.N) * base.K;
                const long long acts = static_cast<long long>(base.B) * base.H * base.W * base.Cin;
                if (tile / kern::NUM_TILES >= 6 || wts > acts || acts > 3 * wts ||
                    (base.N + bn - 1) / bn < 4 * (order == 4 ? 2 : 1))
                  continue;
              }
              kern::ConvArgs a = base;
              a.splits = sp;
              a.order = order;
              a.tail = tail;
              if (!fused) a.counters = nullptr;
              if (kern::conv_igemm(a, tile, s_compute_) != hipSuccess) continue;  // warm-up / validity
              float ms = 0;
              if (cold) {
                // median of 3 (x3, to keep the 3-launch scale of the stored times): one slow
                // repetition (a clock or queue hiccup) no longer decides the winner -- the mean
                // did, and repeated tunings of one model picked different tiles run to run
                float rep[3];
                for (int r = 0; r < 3; ++r) {
                  HIP_CHECK(kern::l2_scrub(scrub, kScrubBytes, sink, s_compute_));
                  if (producer >= 0)
                    encode_forward(B, 0, s_compute_, nullptr, ALL, static_cast<size_t>(producer),
                                   static_cast<size_t>(producer) + 1);
                  HIP_CHECK(hipEventRecord(e0, s_compute_));
                  HIP_CHECK(kern::conv_igemm(a, tile, s_compute_));
                  HIP_CHECK(hipEventRecord(e1, s_compute_));
                  HIP_CHECK(hipEventSynchronize(e1));
                  HIP_CHECK(hipEventElapsedTime(&rep[r], e0, e1));
                }
                std::sort(rep, rep + 3);
                ms = 3.f * rep[1];
              } else {
                HIP_CHECK(hipEventRecord(e0, s_compute_));
                for (int r = 0; r < 3; ++r) HIP_CHECK(kern::conv_igemm(a, tile, s_compute_));
                HIP_CHECK(hipEventRecord(e1, s_compute_));
                HIP_CHECK(hipEventSynchronize(e1));
                HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
              }
              measured.push_back({ms, Tune{tile, sp, fused != 0, order, tail}});
              if (ms < best) {
                best = ms;
                bt = Tune{tile, sp, fused != 0, order, tail};
              }
              if (fused && ms < best_fused) {
                best_fused = ms;
                bt_fused = Tune{tile, sp, true, order, tail};
              }
            }
          }
        }
        // Stream-K candidates (EngineOptions::tune_streamk): the LDS-DMA loops with P = 256 / 512 /
        // 1024 blocks splitting the tiles x K-steps evenly (ConvArgs::sk) -- for grids whose tile
        // count lands just past a multiple of the CU count (ResNet50 stage-3 reduce at B = 24: 296
        // tiles = two tiles on 40 CUs, one on the rest)
        if (opt_.tune_streamk && base.N % 8 == 0 && !base.in_scale && !base.row_parts && !base.stats_out)
          for (int tile = 0; tile < kern::NUM_CFGS; ++tile) {
            const int v = tile / kern::NUM_TILES;
            if (v != 1 && v != 5) continue;  // 2-stage ring and 1-stage loop
            int bm, bn;
            kern::tile_dims(tile, bm, bn);
            const long long T = static_cast<long long>((base.M + bm - 1) / bm) * ((base.N + bn - 1) / bn);
            for (int P : {256, 512, 1024}) {
              if (T * nk < P || T > kCounters || kern::streamk_workspace_bytes(P, bm, bn) > ws_bytes_) continue;
              kern::ConvArgs a = base;
              a.splits = 1;
              a.sk = P;
              if (kern::conv_igemm(a, tile, s_compute_) != hipSuccess) continue;
              float ms = 0;
              if (cold) {
                float rep[3];
                for (int r = 0; r < 3; ++r) {
                  HIP_CHECK(kern::l2_scrub(scrub, kScrubBytes, sink, s_compute_));
                  if (producer >= 0)
                    encode_forward(B, 0, s_compute_, nullptr, ALL, static_cast<size_t>(producer),
                                   static_cast<size_t>(producer) + 1);
                  HIP_CHECK(hipEventRecord(e0, s_compute_));
                  HIP_CHECK(kern::conv_igemm(a, tile, s_compute_));
                  HIP_CHECK(hipEventRecord(e1, s_compute_));
                  HIP_CHECK(hipEventSynchronize(e1));
                  HIP_CHECK(hipEventElapsedTime(&rep[r], e0, e1));
                }
                std::sort(rep, rep + 3);
                ms = 3.f * rep[1];
              } else {
                HIP_CHECK(hipEventRecord(e0, s_compute_));
                for (int r = 0; r < 3; ++r) HIP_CHECK(kern::conv_igemm(a, tile, s_compute_));
                HIP_CHECK(hipEventRecord(e1, s_compute_));
                HIP_CHECK(hipEventSynchronize(e1));
                HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
              }
              Tune tk{tile, 1, true, 0, 0, P};
              measured.push_back({ms, tk});
              if (ms < best) {
                best = ms;
                bt = tk;
              }
            }
          }
        if (bt.splits > 1 && !bt.fused && best_fused <= best * (1.f + opt_.splitk_fused_margin)) {
          bt = bt_fused;  // EngineOptions::splitk_fused_margin: one graph node instead of two
          best = best_fused;
        }
        tune_[bi][oi] = bt;
        tuned_shapes[key] = {bt, best / 3 * 1000.0};
        if (opt_.tune_in_graph) {  // the isolated-launch front runners, for the in-graph pass
          std::sort(measured.begin(), measured.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
          auto& c = cands_[key];
          for (const auto& m : measured)
            if (c.size() < kInGraphCands && m.first <= best * kInGraphSlack) c.push_back(m.second);
        }
        if (B == max_batch_) total_best_us += best / 3 * 1000.0;
      }
    }
    tuned_conv_us_ = total_best_us;
    tune_cache_hits_ = static_cast<long long>(loaded);
    if (opt_.tune_in_graph) tune_in_graph(tuned_shapes);
    if (tuned_shapes.size() > loaded) save_tune_cache(cache_path, tuned_shapes);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(scrub);
    (void)hipFree(sink);
  }

  // In-graph retune (EngineOptions::tune_in_graph): the isolated launches above time each conv
  // behind an L2 scrub; inside a forward the conv reads its input just written by the previous op
  // and its weights from wherever the last forward left them.  For every conv with more than one
  // front runner (within kInGraphSlack of the isolated best, at most kInGraphCands), each candidate
  // is timed IN PLACE -- eager forwards with events around every op, the conv's own interval, median
  // of kInGraphReps -- and the fastest kept.  Ops are visited in order, so later ops are timed
  // behind the earlier ops' final choices.  Results go to the tune cache under the op's position.
  // the in-graph pass's results for bucket B are in the tune cache already
  bool in_graph_cached(const std::map<std::string, std::pair<Tune, double>>& shapes, int B) const {
    const std::string pre = "g" + std::to_string(plan_.ops.size()) + ":b" + std::to_string(B) + ":";
    for (const auto& kv : shapes)
      if (kv.first.compare(0, pre.size(), pre) == 0) return true;
    return false;
  }
  static constexpr size_t kInGraphCands = 4;
  static constexpr float kInGraphSlack = 1.25f;
  static constexpr int kInGraphReps = 5;
  void tune_in_graph(std::map<std::string, std::pair<Tune, double>>& tuned_shapes) {
    const size_t n = plan_.ops.size();
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    long long changed = 0, timed = 0;
    for (size_t bi = 0; bi < buckets_.size(); ++bi) {
      const int B = buckets_[bi];
      slots_[0].h_lens[live_index()] = B;  // the whole bucket is live
      encode_forward(B, 0, s_compute_);   // warm
      for (size_t oi = 0; oi < n; ++oi) {
        const PlanOp& op = plan_.ops[oi];
        if (op.kind != PlanOp::CONV) continue;
        kern::ConvArgs base = conv_args(op, B, 0);
        // keyed by position AND by the op's shape + tuning regime: another model with
        // the same op count and names, or another tuning regime, never loads this choice
        const std::string gkey = "g" + std::to_string(n) + ":b" + std::to_string(B) + ":o" + std::to_string(oi) + ":" +
                                 op.name.substr(0, 64) + ":" + std::to_string(sp_) + ":" + shape_key(base, false);
        auto memo = tuned_shapes.find(gkey);
        if (memo != tuned_shapes.end()) {
          tune_[bi][oi] = memo->second.first;
          continue;
        }
        const auto c = cands_.find(shape_key(base, false));  // the isolated-launch front runners
        if (c == cands_.end() || c->second.size() < 2) continue;
        float best = 1e30f;
        Tune bt = tune_[bi][oi];
        for (const Tune& t : c->second) {
          tune_[bi][oi] = t;
          std::vector<float> v;
          for (int r = 0; r < kInGraphReps; ++r) {
            encode_forward(B, 0, s_compute_, ev.data());
            HIP_CHECK(hipStreamSynchronize(s_compute_));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, ev[oi], ev[oi + 1]));
            v.push_back(ms);
          }
          std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
          ++timed;
          if (v[v.size() / 2] < best) {
            best = v[v.size() / 2];
            bt = t;
          }
        }
        const Tune& first = c->second.front();
        if (bt.tile != first.tile || bt.splits != first.splits || bt.fused != first.fused) ++changed;
        tune_[bi][oi] = bt;
        tuned_shapes[gkey] = {bt, best * 1000.0};
      }
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    in_graph_timed_ = timed;
    in_graph_changed_ = changed;
  }

  // Encode one forward pass for `B` samples using slot `s`'s input/output buffers.
  // op_events (profiling): if given, events[0] is recorded before the first op and events[i + 1]
  // after op i.
  enum Part { ALL = 0, PREP = 1, MAIN = 2 };
  // PREP = decode-table fetch + device decode + the leading input-prep ops (per-slot buffers only);
  // MAIN = the rest.  submit() runs PREP on the copy stream so it overlaps the previous batch's
  // MAIN on the compute stream.
  // range_begin/range_end (autotune): encode only ops [range_begin, range_end), nothing else.
  void encode_forward(int B, int s, hipStream_t st, hipEvent_t* op_events = nullptr, Part part = ALL,
                      size_t range_begin = SIZE_MAX, size_t range_end = 0) {
    auto buf = [&](int id) -> void* { return buf_ptr(id, s); };
    auto prm = [&](size_t off) -> const float* { return prm_ptr(off); };
    const bool ranged = range_begin != SIZE_MAX;
    if (ranged) part = MAIN;
    const size_t op_begin = ranged ? range_begin : part == MAIN ? n_prep_ops_ : 0;
    const size_t op_end = ranged ? range_end : part == PREP ? n_prep_ops_ : plan_.ops.size();
    if (part != MAIN) {  // the slot's table (live batch; decode lens/offsets) from host-coherent memory
      const hipError_t ec = kern::copy_i64(slots_[s].h_lens_dev, slots_[s].d_lens, static_cast<int>(table_len()), st);
      if (ec != hipSuccess) throw std::runtime_error("launch of table fetch failed: " + std::string(hipGetErrorString(ec)));
    }
    if (text_cap_ && part != MAIN) {
      Slot& sl = slots_[s];
      // packed samples (d_lens row 2 >= 0) are expanded in registers by the decode kernels
      const hipError_t e = kern::decode_json_numbers(d_text_, sl.d_lens + max_batch_, text_cap_, sl.d_lens, B, sl.d_in,
                                                     static_cast<long long>(in_numel_), sl.d_status,
                                                     sl.d_status + max_batch_, sl.d_scratch, st, d_packed_,
                                                     d_packed_ ? sl.d_lens + 2 * max_batch_ : nullptr);
      if (e != hipSuccess) throw std::runtime_error("launch of device decode failed: " + std::string(hipGetErrorString(e)));
    }
    if (op_events) HIP_CHECK(hipEventRecord(op_events[0], st));
    const hipStream_t main_st = st;
    const long long* live = use_live_ ? slots_[s].d_lens + live_index() : nullptr;
    int pending_join = -1;  // open side branch: the op that waits for it
    for (size_t op_index = op_begin; op_index < op_end; ++op_index) {
      const PlanOp& op = plan_.ops[op_index];
      hipError_t e = hipSuccess;
      if (static_cast<int>(op_index) == pending_join) {
        HIP_CHECK(hipStreamWaitEvent(main_st, ev_join_, 0));
        pending_join = -1;
      }
      // per-op profiling times ops one after another: no branches then
      const bool side = branches_ && !op_events && op.join >= 0 && pending_join < 0;
      st = main_st;
      if (side) {
        HIP_CHECK(hipEventRecord(ev_fork_, main_st));
        HIP_CHECK(hipStreamWaitEvent(s_side_, ev_fork_, 0));
        st = s_side_;
      }
      switch (op.kind) {
        case PlanOp::INPUT_PREP:
          if (op.Cp > 8)
            e = kern::input_prep_wide(static_cast<const float*>(buf(op.in)), prm(op.scale_off), prm(op.shift_off),
                                      static_cast<uint16_t*>(buf(op.out)), B, op.C, op.H, op.W, op.Cp, st, sp_);
          else
            e = kern::input_prep(static_cast<const float*>(buf(op.in)), prm(op.scale_off), prm(op.shift_off),
                                 static_cast<uint16_t*>(buf(op.out)), B, op.C, op.H, op.W, op.Cp, st, sp_);
          break;
        case PlanOp::ROWS_PREP:
          e = kern::rows_prep(static_cast<const float*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)),
                              op.rows_per_sample * B, op.C, op.Cp, st, sp_);
          break;
        case PlanOp::COPY_COLS: {
          const long long R = op.rows_per_sample * B;
          e = kern::copy_cols(static_cast<const uint16_t*>(buf(op.in)), R * op.ld[0], op.ld[0], op.col[0],
                              static_cast<uint16_t*>(buf(op.out)), R * op.ld[1], op.ld[1], op.col[1], R, op.C, st, sp_);
          break;
        }
        case PlanOp::BINARY:
          e = kern::binary_rows(static_cast<const uint16_t*>(buf(op.in)), static_cast<const uint16_t*>(buf(op.in2)),
                                static_cast<uint16_t*>(buf(op.out)), op.rows_per_sample * B, op.C, op.rows_per_sample,
                                op.S, op.gidx, op.act, op.clip_lo, op.clip_hi, st, live, sp_, op.Cp);
          break;
        case PlanOp::UNARY:
          e = kern::unary_rows(static_cast<const uint16_t*>(buf(op.in)), prm(op.scale_off), prm(op.shift_off),
                               static_cast<uint16_t*>(buf(op.out)), op.rows_per_sample * B, op.C, op.act, op.clip_lo,
                               op.clip_hi, st, live, op.rows_per_sample, sp_, op.Cp);
          break;
        case PlanOp::CONV: {
          kern::ConvArgs a = conv_args(op, B, s);
          if (!use_live_) a.live = nullptr;
          const Tune t = tune_for(B, op_index);
          a.splits = t.splits;
          a.tail = t.tail;
          a.sk = t.sk;
          a.order = opt_.conv_order > 0 ? opt_.conv_order : t.order;
          a.ws = side ? ws_side_ : wss_[s % n_exec_];
          if (side) a.counters = counters_side_;
          if (!t.fused) a.counters = nullptr;
          e = kern::conv_igemm(a, t.tile, st);
          break;
        }
        case PlanOp::CONV_PAIR: {
          kern::PairArgs a;
          a.x = static_cast<const uint16_t*>(buf(op.in));
          a.w1 = reinterpret_cast<const uint16_t*>(params_ + op.w_off);
          a.bias1 = prm(op.bias_off);
          a.res = static_cast<const uint16_t*>(buf(op.in2));
          a.xout = static_cast<uint16_t*>(buf(op.out));
          a.aout = static_cast<uint16_t*>(buf(op.out3));
          a.scale2 = prm(op.s2_off);
          a.shift2 = prm(op.b2_off);
          a.relu2 = op.conv.relu2;
          a.w2 = reinterpret_cast<const uint16_t*>(params_ + op.w2_off);
          a.bias2 = prm(op.bias2_off);
          a.relu = op.pair_relu;
          a.out = static_cast<uint16_t*>(buf(op.out2));
          a.M = B * op.conv.Ho * op.conv.Wo;
          a.K1 = op.conv.K;
          a.N1 = op.conv.N;
          a.N2 = op.n2;
          a.rows_per_sample = op.conv.Ho * op.conv.Wo;
          a.live = live;
          a.zeros = zeros_;
          a.split = sp_;
          a.wplane1 = op.conv.wplane;
          a.wplane2 = op.w2plane;
          e = kern::conv_pair(a, st);
          break;
        }
        case PlanOp::PAD:
          e = kern::pad_nhwc(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)), B, op.H, op.W,
                             op.C, op.Ho, op.Wo, op.ph, op.pw, st, sp_, op.sh, op.sw);
          break;
        case PlanOp::WHERE:
          e = kern::where_rows(static_cast<const uint16_t*>(buf(op.in)), op.in2 >= 0 ? static_cast<const uint16_t*>(buf(op.in2)) : nullptr,
                               op.in3 >= 0 ? static_cast<const uint16_t*>(buf(op.in3)) : nullptr, op.clip_lo, op.clip_hi,
                               static_cast<uint16_t*>(buf(op.out)), op.rows_per_sample * B, op.C, st, live,
                               op.rows_per_sample, sp_, op.Cp);
          break;
        case PlanOp::BMM:
          e = kern::bmm_rows(static_cast<const uint16_t*>(buf(op.in)), static_cast<const uint16_t*>(buf(op.in2)),
                             static_cast<uint16_t*>(buf(op.out)), B, op.S, op.Cp, op.gidx, op.ld[0], op.ld[1], op.C, st,
                             live, sp_);
          break;
        case PlanOp::RESIZE:
          e = kern::resize_nhwc(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)), B, op.H, op.W,
                                op.C, op.Ho, op.Wo, op.clip_lo, op.clip_hi, op.gidx, op.act, op.is_max, st, live, sp_);
          break;
        case PlanOp::POOL:
          e = kern::pool2d(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)), B, op.H, op.W,
                           op.C, op.Ho, op.Wo, op.kh, op.kw, op.sh, op.sw, op.ph, op.pw, op.is_max, op.cip, st, live,
                           prm(op.scale_off), prm(op.shift_off), op.act, sp_);
          break;
        case PlanOp::GAP:
          e = kern::global_avgpool(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)),
                                   nullptr, nullptr, nullptr, 0, B, op.H * op.W, op.C, st, live, sp_, op.gidx);
          break;
        case PlanOp::GAP_FC:
          e = kern::gap_fc(static_cast<const uint16_t*>(buf(op.in)), B, op.H * op.W, op.C, op.gidx,
                           reinterpret_cast<const uint16_t*>(params_ + op.w_off), op.conv.wplane, op.conv.Kpad,
                           prm(op.bias_off), op.Cp, op.act, static_cast<float*>(buf(op.out_f32)),
                           side ? ws_side_ : wss_[s % n_exec_], ws_bytes_, side ? counters_side_ : counterss_[s % n_exec_],
                           kCounters, st, live, sp_);
          break;
        case PlanOp::AFFINE:
          e = kern::affine_act(static_cast<const uint16_t*>(buf(op.in)), static_cast<const uint16_t*>(buf(op.in2)),
                               prm(op.scale_off), prm(op.shift_off), op.act, static_cast<uint16_t*>(buf(op.out)),
                               op.rows_per_sample * B, op.C, st, live, op.rows_per_sample, sp_, op.clip_lo, op.clip_hi);
          break;
        case PlanOp::TO_NCHW_F32:
          if (op.ld_store > 0)
            e = kern::nhwc_to_nchw_f32_strided(static_cast<const uint16_t*>(buf(op.in)), static_cast<float*>(buf(op.out_f32)),
                                               B, op.H, op.W, op.C, op.ld_store, st, sp_);
          else
            e = kern::nhwc_to_nchw_f32(static_cast<const uint16_t*>(buf(op.in)), static_cast<float*>(buf(op.out_f32)), B,
                                       op.H, op.W, op.C, st, sp_);
          break;
        case PlanOp::STEM:
          if (op.is_max) {  // + max pool (+ the pooled value's affine), input prep fused
            e = kern::conv_stem_pool_nchw(static_cast<const float*>(buf(op.in)), op.C, prm(op.scale_off), prm(op.shift_off),
                                          reinterpret_cast<const uint16_t*>(params_ + op.w_off), prm(op.bias_off),
                                          op.conv.relu, prm(op.s2_off), prm(op.b2_off), op.act,
                                          static_cast<uint16_t*>(buf(op.out)), B, op.conv.H, op.conv.W, op.conv.Ho,
                                          op.conv.Wo, op.Ho, op.Wo, st, live, sp_);
            break;
          }
          if (op.in == -2) {  // graph input, input prep fused
            e = kern::conv_stem7x7_nchw(static_cast<const float*>(buf(op.in)), op.C, prm(op.scale_off),
                                        prm(op.shift_off), reinterpret_cast<const uint16_t*>(params_ + op.w_off),
                                        prm(op.bias_off), static_cast<uint16_t*>(buf(op.out)), B, op.conv.H,
                                        op.conv.W, op.conv.Ho, op.conv.Wo, op.conv.relu, st, live, sp_);
            break;
          }
          e = kern::conv_stem7x7(static_cast<const uint16_t*>(buf(op.in)),
                                 reinterpret_cast<const uint16_t*>(params_ + op.w_off), prm(op.bias_off),
                                 static_cast<uint16_t*>(buf(op.out)), B, op.conv.H, op.conv.W, op.conv.Ho, op.conv.Wo,
                                 op.conv.relu, st, live, sp_);
          break;
        case PlanOp::LAYERNORM:
          if (op.stats_only)
            e = kern::layernorm_rows(static_cast<const uint16_t*>(buf(op.in)), nullptr, prm(op.scale_off),
                                     prm(op.shift_off), op.eps, op.rows_per_sample * B, op.C, st, sp_, op.Cp, 0,
                                     static_cast<float*>(buf(op.out)));
          else
            e = kern::layernorm_rows(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)),
                                     prm(op.scale_off), prm(op.shift_off), op.eps, op.rows_per_sample * B, op.C, st, sp_,
                                     op.Cp);
          break;
        case PlanOp::TOKENS:
          e = kern::tokens_assemble(static_cast<const uint16_t*>(buf(op.in)), prm(op.scale_off), prm(op.shift_off),
                                    static_cast<uint16_t*>(buf(op.out)), B, op.S, op.C, st, sp_,
                                    op.out_stats >= 0 ? static_cast<float*>(buf(op.out_stats)) : nullptr);
          break;
        case PlanOp::GATHER_ROWS:
          e = kern::gather_rows(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)), B, op.S,
                                op.gidx, op.C, st, sp_);
          break;
        case PlanOp::ATTENTION:
          e = kern::attention(static_cast<const uint16_t*>(buf(op.in)) + op.col[0],
                              static_cast<const uint16_t*>(buf(op.in2)) + op.col[1],
                              static_cast<const uint16_t*>(buf(op.in3)) + op.col[2], static_cast<uint16_t*>(buf(op.out)),
                              B, op.S, op.nh, op.hd, op.ld[0], op.ld[1], op.ld[2], op.C, op.fscale, st, sp_);
          break;
        case PlanOp::GCONV: {
          kern::GConvArgs g;
          g.x = static_cast<const uint16_t*>(buf(op.in));
          g.w = prm(op.w_off);
          g.bias = prm(op.bias_off);
          g.res = static_cast<const uint16_t*>(buf(op.in2));
          g.out = static_cast<uint16_t*>(buf(op.out));
          g.B = B;
          g.H = op.H;
          g.W = op.W;
          g.Cin = op.C;
          g.Ho = op.Ho;
          g.Wo = op.Wo;
          g.Cout = op.Cp;
          g.groups = op.groups;
          g.KH = op.kh;
          g.KW = op.kw;
          g.stride = op.sh;
          g.dil = op.sw;
          g.pad_h = op.ph;
          g.pad_w = op.pw;
          g.act = op.act;
          g.clip_lo = op.clip_lo;
          g.clip_hi = op.clip_hi;
          g.split = sp_;
          g.live = live;
          e = kern::grouped_conv(g, st);
          break;
        }
        case PlanOp::SOFTMAX:
          e = kern::softmax_rows(static_cast<const uint16_t*>(buf(op.in)), static_cast<uint16_t*>(buf(op.out)),
                                 static_cast<float*>(buf(op.out_f32)), op.rows_per_sample * B, op.C, st, sp_, op.ld_store);
          break;
        case PlanOp::BF16_TO_F32:
          if (op.ld_store > 0)
            e = kern::rows_to_f32(static_cast<const uint16_t*>(buf(op.in)), static_cast<float*>(buf(op.out_f32)),
                                  op.rows_per_sample * B, op.C, op.ld_store, st, sp_);
          else
            e = kern::bf16_to_f32(static_cast<const uint16_t*>(buf(op.in)), static_cast<float*>(buf(op.out_f32)),
                                  static_cast<long long>(B) * op.C, st, sp_);
          break;
      }
      if (e != hipSuccess)
        throw std::runtime_error("launch of " + op.name + " failed: " + std::string(hipGetErrorString(e)));
      if (side) {
        HIP_CHECK(hipEventRecord(ev_join_, s_side_));
        pending_join = op.join;
      }
      if (op_events) HIP_CHECK(hipEventRecord(op_events[op_index + 1], st));
    }
    if (pending_join >= 0) HIP_CHECK(hipStreamWaitEvent(main_st, ev_join_, 0));  // part ended before the join
  }

  // Per-op device time (eager launches bracketed by events), averaged over `iters` forwards.
  Json profile_ops(int B, int iters) override {
    std::lock_guard<std::mutex> submit_guard(submit_mu_);
    synchronize();
    B = std::max(1, std::min(B, max_batch_));
    const size_t n = plan_.ops.size();
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
    std::vector<double> us(n, 0.0);
    size_t bi = 0;
    while (buckets_[bi] < B) ++bi;
    const int Bk = buckets_[bi];
    slots_[0].h_lens[live_index()] = Bk;  // profile the whole bucket
    encode_forward(Bk, 0, s_compute_);  // warm
    for (int it = 0; it < iters; ++it) {
      encode_forward(Bk, 0, s_compute_, ev.data());
      HIP_CHECK(hipStreamSynchronize(s_compute_));
      for (size_t i = 0; i < n; ++i) {
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
        us[i] += ms * 1000.0 / iters;
      }
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    static const char* kinds[] = {"input_prep", "conv", "pool", "gap", "affine", "to_nchw_f32", "bf16_to_f32",
                                  "layernorm", "tokens", "gather_rows", "attention", "stem", "gconv", "softmax",
                                  "rows_prep", "copy_cols", "binary", "unary", "conv_pair", "pad", "where", "resize", "bmm", "gap_fc"};
    static_assert(sizeof(kinds) / sizeof(kinds[0]) == PlanOp::GAP_FC + 1, "one name per PlanOp kind");
    Json out = Json::object();
    Json ops = Json::array();
    double total = 0;
    for (size_t i = 0; i < n; ++i) {
      const PlanOp& op = plan_.ops[i];
      Json o = Json::object();
      o["name"] = op.name;
      o["kind"] = kinds[op.kind];
      o["us"] = us[i];
      o["gflop"] = op.flops_per_sample * Bk / 1e9;
      o["tflops"] = us[i] > 0 ? op.flops_per_sample * Bk / (us[i] * 1e6) : 0.0;
      if (op.kind == PlanOp::CONV) {
        const Tune t = tune_for(Bk, i);
        o["tile"] = t.tile;
        o["splits"] = t.splits;
        o["fused_splitk"] = t.fused;
        o["tile_order"] = t.order;
        o["tail_splitk"] = t.tail > 0;
        o["streamk_blocks"] = t.sk;
      }
      total += us[i];
      ops.push_back(o);
    }
    out["batch"] = Bk;
    out["total_us"] = total;
    out["tflops"] = total > 0 ? plan_.flops_per_sample * Bk / (total * 1e6) : 0.0;
    out["ops"] = ops;
    return out;
  }

 private:
  static constexpr int kStageStreams = 2;
  struct Slot {
    float* d_gather = nullptr;  // data parallel: [world][max_batch][out_numel]
    int* d_gstatus = nullptr;
    float* h_gather = nullptr;
    int* h_gstatus = nullptr;
    hipEvent_t ev_gather{};
    float* d_in = nullptr;
    float* d_out = nullptr;
    float* h_out = nullptr;
    void* d_scratch = nullptr;
    long long* d_lens = nullptr;      // [lens][text offsets into d_text_][packed offsets into d_packed_] x max_batch
    long long* h_lens = nullptr;      // pinned host-coherent, same layout
    long long* h_lens_dev = nullptr;  // its device-side address
    int* d_status = nullptr;          // [status x max_batch][ntok x max_batch]
    int* h_status = nullptr;          // pinned
    hipEvent_t ev_h2d[kStageStreams] = {};
    hipEvent_t ev_d2h{};
    hipEvent_t ev_main{};  // MAIN done on the compute stream: the result copies (s_out_) wait on it
    hipEvent_t ev_prep{};
    std::vector<void*> d_prep;  // per-slot outputs of the PREP part's input-prep ops
  };
  struct Job {
    int slot = 0;
    int B = 0;
    BatchDone done;
    std::chrono::steady_clock::time_point t0;
    std::string error;
    bool has_text = false;
    bool dp_gathered = false;  // failed, but the collectives ran with this rank's shard flag cleared
    int ev = 0;  // first of its kEvPerJob timing events in tev_
    int bi = 0;  // batch bucket
  };

  struct StageReq {
    int t;
    const char* text;
    size_t len;
    bool packed;  // 4-bit packed: (len + 1) / 2 bytes to d_packed_
  };
  static constexpr int kQueued = 0, kIssued = 1, kFailed = 2;

  // Block until the stager has issued (or failed) ticket t's copy; returns its state.
  int wait_staged(int t) {
    std::unique_lock<std::mutex> lk(stage_mu_);
    stage_done_cv_.wait(lk, [&] { return stage_state_[t] != kQueued; });
    return stage_state_[t];
  }

  void stager_loop() {
    (void)hipSetDevice(dev_);
    unsigned long long rr = 0;
    while (true) {
      StageReq rq;
      {
        std::unique_lock<std::mutex> lk(stage_mu_);
        stage_cv_.wait(lk, [&] { return stage_stop_ || !stage_q_.empty(); });
        if (stage_q_.empty()) return;
        rq = stage_q_.front();
        stage_q_.pop_front();
      }
      // round-robin over kStageStreams copy streams (one reaches ~36 GB/s for 1 MiB pinned copies,
      // two ~47 GB/s); per stream copies complete in issue order, which the sequence number records
      const int si = static_cast<int>(rr++ % n_copy_streams_);
      const auto ti0 = std::chrono::steady_clock::now();
      const bool ok = (rq.packed ? hipMemcpyAsync(d_packed_ + static_cast<size_t>(rq.t) * (text_cap_ / 2), rq.text,
                                                  (rq.len + 1) / 2, hipMemcpyHostToDevice, s_stage_[si])
                                 : hipMemcpyAsync(d_text_ + static_cast<size_t>(rq.t) * text_cap_, rq.text, rq.len,
                                                  hipMemcpyHostToDevice, s_stage_[si])) == hipSuccess &&
                      hipEventRecord(stage_ev_[rq.t], s_stage_[si]) == hipSuccess;
      diag_issue_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - ti0).count();
      if (ok) h2d_bytes_.fetch_add(static_cast<long long>(rq.packed ? (rq.len + 1) / 2 : rq.len), std::memory_order_relaxed);
      {
        std::lock_guard<std::mutex> g(stage_mu_);
        stage_stream_[rq.t] = si;
        stage_seq_[rq.t] = ++stage_counter_[si];
        stage_state_[rq.t] = ok ? kIssued : kFailed;
      }
      stage_done_cv_.notify_all();
    }
  }

  void completion_loop() {
    (void)hipSetDevice(dev_);
    while (true) {
      Job job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return;
        job = std::move(jobs_.front());
        jobs_.pop_front();
      }
      Slot& sl = slots_[job.slot];
      TraceRange tr_done("engine.completion(d2h wait+callback)");
      BatchResult r;
      if (job.error.empty()) {
        hipError_t e;
        if (completion_poll_us_ > 0) {
          // sleep-poll instead of the runtime wait, which was seen spinning a whole CPU even with a
          // blocking-sync event (gpurun_out/r2_46 threads_*.txt): that CPU serves HTTP/JSON instead
          while ((e = hipEventQuery(sl.ev_d2h)) == hipErrorNotReady)
            std::this_thread::sleep_for(std::chrono::microseconds(completion_poll_us_));
        } else {
          e = hipEventSynchronize(sl.ev_d2h);
        }
        if (e != hipSuccess) {
          r.ok = false;
          r.error = std::string("device error: ") + hipGetErrorString(e);
        } else {
          float ms = 0;
          if (hipEventElapsedTime(&ms, tev_[job.ev + 1], tev_[job.ev + 2]) == hipSuccess) r.device_us = ms * 1000.0;
          float wait_ms = 0, gap_ms = 0;
          if (hipEventElapsedTime(&wait_ms, tev_[job.ev], tev_[job.ev + (prep_on_compute_ ? 3 : 1)]) == hipSuccess) copy_wait_ms_total_ = copy_wait_ms_total_.load() + wait_ms;
          if (prev_ev_ >= 0 && hipEventElapsedTime(&gap_ms, tev_[prev_ev_ + 2], tev_[job.ev]) == hipSuccess && gap_ms > 0)
            gpu_gap_ms_total_ = gpu_gap_ms_total_.load() + gap_ms;
          prev_ev_ = job.ev;
          {
            // pacing model: device-time EMA per bucket, and lead = EMA of this batch's input path
            // (first copy issued -> PREP done, on the device) + a margin for the dispatch itself
            // that grows when MAIN had to wait for its input anyway (wait_ms: compute stream idle
            // behind the copies/prep) and shrinks slowly otherwise
            float in_ms = 0;
            // (PREP in line on the compute stream: the lead covers the copies only)
            const bool have_in =
                hipEventElapsedTime(&in_ms, tev_[job.ev + 5], tev_[job.ev + (prep_on_compute_ ? 6 : 4)]) == hipSuccess;
            std::lock_guard<std::mutex> g(pace_mu_);
            double& e = est_ms_[job.bi];
            e = e > 0.0 ? 0.8 * e + 0.2 * ms : ms;
            if (have_in) input_ms_ = input_ms_ > 0.0 ? 0.8 * input_ms_ + 0.2 * in_ms : in_ms;
            if (wait_ms > 0.02) margin_ms_ = std::min(margin_ms_ + 0.02, 1.0);
            else margin_ms_ = std::max(margin_ms_ - 0.004, 0.03);
            lead_ms_ = input_ms_ + margin_ms_;
            lead_ms_total_ += lead_ms_;
          }
          float prep_ms = 0;
          if (hipEventElapsedTime(&prep_ms, tev_[job.ev + 3], tev_[job.ev + 4]) == hipSuccess)
            prep_ms_total_ = prep_ms_total_.load() + prep_ms;
          r.outputs = sl.h_out;
          r.output_numel = out_numel_;
          if (job.has_text) {
            r.status = sl.h_status;
            r.ntok = sl.h_status + max_batch_;
          }
          if (comm_) {
            r.gathered = dp_world_;
            r.outputs = sl.h_gather;
            r.status = job.has_text ? sl.h_gstatus : nullptr;
            r.ntok = r.status ? sl.h_gstatus + max_batch_ : nullptr;
            r.status_stride = static_cast<int>(status_len());
            rank_ok_copy_.resize(static_cast<size_t>(dp_world_));
            for (int k = 0; k < dp_world_; ++k)
              rank_ok_copy_[static_cast<size_t>(k)] = sl.h_gstatus[static_cast<size_t>(k) * status_len() + rank_ok_index()];
            r.rank_ok = rank_ok_copy_.data();
          }
          batches_++;
          images_ += job.B;
          device_ms_total_ = device_ms_total_.load() + ms;
        }
      } else {
        r.ok = false;
        r.error = job.error;
        if (job.dp_gathered && comm_ && hipEventSynchronize(sl.ev_d2h) == hipSuccess) {
          // this rank's shard failed, the others' rows arrived: hand them over with the flags, so the
          // DP engine fails exactly this shard's items (the host backend's semantics, dp_layout.h)
          r.gathered = dp_world_;
          r.outputs = sl.h_gather;
          r.output_numel = out_numel_;
          r.status = job.has_text ? sl.h_gstatus : nullptr;
          r.ntok = r.status ? sl.h_gstatus + max_batch_ : nullptr;
          r.status_stride = static_cast<int>(status_len());
          rank_ok_copy_.resize(static_cast<size_t>(dp_world_));
          for (int k = 0; k < dp_world_; ++k)
            rank_ok_copy_[static_cast<size_t>(k)] = sl.h_gstatus[static_cast<size_t>(k) * status_len() + rank_ok_index()];
          r.rank_ok = rank_ok_copy_.data();
        }
      }
      r.wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - job.t0).count();
      // Take the results out of the slot's pinned buffers and free the slot BEFORE the callbacks
      // (cache inserts, response hand-off for B requests): the batcher can dispatch the next batch
      // into this slot while they run, so the GPU does not idle behind host bookkeeping.
      if (r.ok || r.rank_ok) {
        const size_t rows = static_cast<size_t>(job.B) * (comm_ ? dp_world_ : 1);
        if (r.outputs) {
          out_copy_.assign(r.outputs, r.outputs + rows * out_numel_);
          r.outputs = out_copy_.data();
        }
        if (r.status) {
          const size_t n = comm_ ? status_len() * dp_world_ : 2 * static_cast<size_t>(max_batch_);
          const int* base = r.status;
          status_copy_.assign(base, base + n);
          r.status = status_copy_.data();
          r.ntok = status_copy_.data() + max_batch_;
        }
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        --inflight_;
      }
      slot_cv_.notify_all();
      try {
        job.done(r);
      } catch (...) {
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        --callbacks_running_;
      }
      slot_cv_.notify_all();
    }
  }

  std::string path_;
  EngineOptions opt_;
  int dev_ = 0;
  std::string arch_;
  int max_batch_ = 32;
  int depth_ = 2;
  Plan plan_;
  int sp_ = 0;  // fp32 mode (split kernels)
  size_t in_numel_ = 0, out_numel_ = 0;
  size_t text_cap_ = 0;  // bytes of input text per sample for device decode (0 = off)
  unsigned char* d_text_ = nullptr;  // (n_stage_ + depth_ * max_batch_) x text_cap_
  unsigned char* d_packed_ = nullptr;  // depth_ * max_batch_ x text_cap_ / 2 (packed texts, copied at submit)
  static constexpr int kTableRows = 3;  // per-slot decode table: lens, text offsets, packed offsets
  // ... followed by one element: the live batch (samples of the bucket that are real)
  size_t table_len() const { return static_cast<size_t>(kTableRows) * max_batch_ + 1; }
  // per-slot status table: [status x max_batch][ntok x max_batch][shard ok flag, 3 x pad]; a
  // data-parallel rank all-gathers the whole table, so the flag rides with the rows
  size_t status_len() const { return 2 * static_cast<size_t>(max_batch_) + 4; }
  size_t rank_ok_index() const { return 2 * static_cast<size_t>(max_batch_); }

  // Data parallel: every rank contributes its B rows and its status table to every other rank over
  // xGMI (the same collectives in the same order on every rank, whatever its shard holds), then
  // copies all rows and tables to its host; a group of one copies straight from d_out.
  // The stream a batch's result copies / collectives go on: s_out_ behind an event after the work
  // queued on cs so far (EngineOptions::result_stream), else cs itself.
  hipStream_t result_stream(Slot& sl, hipStream_t cs) {
    if (!s_out_) return cs;
    HIP_CHECK(hipEventRecord(sl.ev_main, cs));
    HIP_CHECK(hipStreamWaitEvent(s_out_, sl.ev_main, 0));
    return s_out_;
  }
  void dp_collectives(Slot& sl, int B, hipStream_t cs) {
    dp_issued_ = true;
    if (dp_world_ > 1) {  // one grouped operation: logits + status table (shard flag included)
      comm_->group_begin();
      comm_->all_gather(sl.d_out, sl.d_gather, sizeof(float) * out_numel_ * B, cs);
      comm_->all_gather(sl.d_status, sl.d_gstatus, sizeof(int) * status_len(), cs);
      comm_->group_end();
      dp_collective_ops_.fetch_add(1, std::memory_order_relaxed);
    }
    HIP_CHECK(hipEventRecord(sl.ev_gather, cs));
    HIP_CHECK(hipMemcpyAsync(sl.h_gather, dp_world_ > 1 ? sl.d_gather : sl.d_out, sizeof(float) * out_numel_ * B * dp_world_,
                             hipMemcpyDeviceToHost, cs));
    HIP_CHECK(hipMemcpyAsync(sl.h_gstatus, dp_world_ > 1 ? sl.d_gstatus : sl.d_status, sizeof(int) * status_len() * dp_world_,
                             hipMemcpyDeviceToHost, cs));
    d2h_bytes_.fetch_add(static_cast<long long>((sizeof(float) * out_numel_ * B + sizeof(int) * status_len()) * dp_world_),
                         std::memory_order_relaxed);
    HIP_CHECK(hipEventRecord(sl.ev_d2h, cs));
  }
  size_t live_index() const { return static_cast<size_t>(kTableRows) * max_batch_; }
  int n_stage_ = 0;                  // early-upload slots (stage_text)
  hipStream_t s_out_ = nullptr;      // result copies / data-parallel collectives (behind Slot::ev_main)
  hipStream_t s_stage_[kStageStreams] = {};
  int n_copy_streams_ = kStageStreams;  // copy streams in use (EngineOptions::copy_streams, 1..kStageStreams)
  unsigned long long stage_counter_[kStageStreams] = {};
  std::vector<hipEvent_t> stage_ev_;
  std::vector<unsigned long long> stage_seq_;  // guarded by stage_mu_ (like the three below)
  std::vector<int> stage_stream_;
  std::vector<char> stage_packed_;  // the ticket's text is 4-bit packed
  std::vector<int> stage_state_;
  std::vector<int> stage_free_;
  std::deque<StageReq> stage_q_;
  bool stage_stop_ = false;
  std::mutex stage_mu_;
  std::condition_variable stage_cv_, stage_done_cv_;
  std::thread stager_;
  std::atomic<long long> staged_total_{0}, staged_used_{0};
  std::atomic<long long> diag_issue_ns_{0}, diag_submit_wait_ns_{0}, diag_not_ready_{0}, diag_submit_ns_{0};
  long long tune_cache_hits_ = 0;
  static constexpr int kCounters = 1 << 16;
  std::map<std::string, std::vector<Tune>> cands_;  // isolated-launch front runners per shape (tune_in_graph)
  long long in_graph_timed_ = 0, in_graph_changed_ = 0;
  static constexpr int kMaxExec = 2;
  int n_exec_ = 1;
  bool branches_ = false;  // side-branch stream in use (PlanOp::join)
  int completion_poll_us_ = 0;     // EngineOptions::completion_poll_us: > 0 = sleep-poll the D2H event (0 = hipEventSynchronize)
  bool prep_on_compute_ = false;  // PREP runs on the compute stream before MAIN (EngineOptions)
  bool use_live_ = true;          // skip the bucket's padding samples (EngineOptions::live_batch)
  double lead_scale_ = 1.0;       // EngineOptions::pace_lead_scale (< 1: dispatch later, trading GPU idle for batch size)
  hipStream_t s_side_{};
  hipStream_t s_prep_{};  // PREP stream (early upload), else PREP shares copy stream 0
  hipEvent_t ev_fork_{}, ev_join_{};
  float* ws_side_ = nullptr;
  int* counters_side_ = nullptr;
  hipStream_t s_exec_[kMaxExec] = {};
  uint8_t* arenas_[kMaxExec] = {};
  float* wss_[kMaxExec] = {};
  int* counterss_[kMaxExec] = {};
  size_t arena_bytes_ = 0;
  Communicator* comm_ = nullptr;  // data parallel (not owned)
  int dp_world_ = 1;
  double weight_bcast_ms_ = 0;                 // RCCL weight broadcast at start-up (stats)
  std::atomic<long long> dp_collective_ops_{0};  // grouped per-batch gathers issued
  std::vector<void*> registered_;
  uint8_t* params_ = nullptr;
  float* ws_ = nullptr;  // executor 0's (autotune)
  size_t ws_bytes_ = 0;
  uint16_t* zeros_ = nullptr;
  std::vector<std::vector<Tune>> tune_;  // [bucket][op]
  double tuned_conv_us_ = 0;
  hipStream_t s_compute_{};
  std::vector<Slot> slots_;
  std::vector<int> buckets_;
  std::vector<hipGraphExec_t> graphs_;       // MAIN part per (bucket, slot)
  std::vector<hipGraphExec_t> prep_graphs_;  // PREP part per (bucket, slot)
  size_t n_prep_ops_ = 0;                    // leading INPUT_PREP ops (PREP part)
  std::vector<int> prep_out_ids_;            // their outputs live in per-slot buffers
  std::unique_ptr<SamplePool> pool_;
  std::thread completion_;
  std::mutex mu_, submit_mu_;
  std::condition_variable cv_, slot_cv_;
  std::deque<Job> jobs_;
  int inflight_ = 0;
  // per job: [0] compute stream reaches the job, [1] MAIN start, [2] MAIN end, [3] PREP start,
  // [4] PREP end, [5] first input copy issued, [6] input copies done
  static constexpr int kTimingJobs = 16, kEvPerJob = 7;
  hipEvent_t tev_[kEvPerJob * kTimingJobs] = {};
  unsigned long long job_seq_ = 0;  // guarded by submit_mu_
  int prev_ev_ = -1;                // completion thread
  std::atomic<double> copy_wait_ms_total_{0.0}, gpu_gap_ms_total_{0.0}, prep_ms_total_{0.0};
  int callbacks_running_ = 0;           // submitted batches whose callback has not returned yet
  std::vector<float> out_copy_;         // completion thread: results of the batch being called back
  std::vector<int> status_copy_;
  std::vector<int> rank_ok_copy_;       // data parallel: gathered shard flags of the batch being called back
  bool dp_issued_ = false;              // submit(): this batch's collectives are issued (guarded by submit_mu_)
  long long nth_batch_ = 0;             // submit(): batches seen (fault injection; guarded by submit_mu_)
  int next_slot_ = 0;
  int last_ev_ = -1, last_bi_ = 0;  // most recent submitted job (guarded by mu_)
  mutable std::mutex pace_mu_;
  std::vector<double> est_ms_;      // EMA device ms per bucket (pace_mu_)
  std::vector<double> batch_ms_;    // start-up device ms per batch size (efficient_batch; empty = off)
  double lead_ms_ = 0.3, lead_ms_total_ = 0.0, input_ms_ = 0.0, margin_ms_ = 0.08;
  std::chrono::steady_clock::time_point pace_drain_{};  // predicted drain of the batch in flight
  bool pace_armed_ = false;
  std::atomic<long long> paced_batches_{0};
  bool stop_ = false;
  std::atomic<long long> batches_{0}, images_{0};
  std::atomic<long long> h2d_bytes_{0}, d2h_bytes_{0}, graph_replays_{0};
  std::atomic<double> device_ms_total_{0.0};
};

}  // namespace

std::unique_ptr<Engine> create_hip_engine(const std::string& model_path, const EngineOptions& opt, std::string* why) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    if (why) *why = "no HIP device visible";
    return nullptr;
  }
  if (opt.device_id >= n) {
    if (why) *why = "device " + std::to_string(opt.device_id) + " not present (" + std::to_string(n) + " visible)";
    return nullptr;
  }
  return std::make_unique<HipEngine>(model_path, opt);
}

std::unique_ptr<Engine> create_hip_engine_model(const std::string& label, onnx::Model model, const EngineOptions& opt,
                                                std::string* why) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || opt.device_id >= n) {
    if (why) *why = "no HIP device visible";
    return nullptr;
  }
  return std::make_unique<HipEngine>(label, std::move(model), opt);
}

}  // namespace die
