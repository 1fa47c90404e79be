#include <pthread.h>
#include "engine.h"
#include "hip_plan.h"

#include "../core/log.h"

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <iostream>
#include <stdexcept>
#include <thread>

#include "cpu_exec.h"

namespace die {

// ---- SamplePool --------------------------------------------------------------------------------

SamplePool::SamplePool(size_t floats_per_sample, AllocFn a, FreeFn f, size_t chunk)
    : floats_(floats_per_sample), alloc_(std::move(a)), free_(std::move(f)), chunk_(chunk) {
  // round each sample up to 256 bytes so DMA sources stay aligned
  floats_ = (floats_ + 63) / 64 * 64;
}

SamplePool::~SamplePool() {
  for (void* c : chunks_) {
    if (free_) free_(c);
    else std::free(c);
  }
}

SampleBuffer SamplePool::acquire() {
  std::lock_guard<std::mutex> g(mu_);
  if (free_list_.empty()) {
    const size_t bytes = floats_ * sizeof(float) * chunk_ + 256;
    void* mem = alloc_ ? alloc_(bytes) : std::aligned_alloc(256, (bytes + 255) / 256 * 256);
    if (!mem) throw std::bad_alloc();
    chunks_.push_back(mem);
    float* base = static_cast<float*>(mem);
    for (size_t k = 0; k < chunk_; ++k) free_list_.push_back(base + k * floats_);
    allocated_ += chunk_;
  }
  float* p = free_list_.back();
  free_list_.pop_back();
  return SampleBuffer{p, floats_};
}

void SamplePool::release(SampleBuffer b) {
  if (!b.data) return;
  std::lock_guard<std::mutex> g(mu_);
  free_list_.push_back(b.data);
}

// ---- Engine helpers ----------------------------------------------------------------------------

size_t Engine::input_numel() const {
  size_t n = 1;
  for (auto d : getInputShape()) n *= static_cast<size_t>(d);
  return n;
}
size_t Engine::output_numel() const {
  size_t n = 1;
  for (auto d : getOutputShape()) n *= static_cast<size_t>(d);
  return n;
}

namespace {

std::vector<std::vector<float>> run_sync(Engine& e, std::vector<BatchItem> items) {
  std::promise<std::vector<std::vector<float>>> pr;
  auto fut = pr.get_future();
  const size_t B = items.size();
  e.submit(std::move(items), [&pr, B](BatchResult& r) {
    if (!r.ok) {
      pr.set_exception(std::make_exception_ptr(std::runtime_error(r.error)));
      return;
    }
    std::vector<std::vector<float>> out(B);
    for (size_t i = 0; i < B; ++i) out[i].assign(r.outputs + i * r.output_numel, r.outputs + (i + 1) * r.output_numel);
    pr.set_value(std::move(out));
  });
  return fut.get();
}

}  // namespace

std::vector<float> Engine::predict(const std::vector<float>& input) {
  const size_t n = std::min(input.size(), input_numel());  // truncate like resize() in the reference
  std::vector<BatchItem> items{BatchItem{input.data(), n}};
  return run_sync(*this, std::move(items)).at(0);
}

std::vector<std::vector<float>> Engine::batchPredict(const std::vector<std::vector<float>>& inputs) {
  if (inputs.empty()) return {};
  const size_t numel = input_numel();
  std::vector<std::vector<float>> all;
  for (size_t b0 = 0; b0 < inputs.size(); b0 += static_cast<size_t>(max_batch())) {
    std::vector<BatchItem> items;
    for (size_t i = b0; i < std::min(inputs.size(), b0 + static_cast<size_t>(max_batch())); ++i) {
      if (inputs[i].size() > numel)
        throw std::runtime_error("input has " + std::to_string(inputs[i].size()) + " values; model expects at most " +
                                 std::to_string(numel));
      items.push_back(BatchItem{inputs[i].data(), inputs[i].size()});
    }
    auto part = run_sync(*this, std::move(items));
    for (auto& p : part) all.push_back(std::move(p));
  }
  return all;
}

// ---- CPU engine ----------------------------------------------------------------------------------

namespace {

std::vector<int64_t> static_shape(const onnx::ValueInfo& vi) {
  std::vector<int64_t> s = vi.dims;
  for (auto& d : s)
    if (d <= 0) d = 1;
  if (!s.empty()) s[0] = 1;
  return s;
}

class CpuEngine : public Engine {
 public:
  CpuEngine(const std::string& path, const EngineOptions& opt)
      : path_(path), opt_(opt), exec_(onnx::load_onnx(path)) {
    shard_id_ = opt.shard_id;
    const auto& m = exec_.model();
    if (m.inputs.empty() || m.outputs.empty()) throw std::runtime_error("model needs at least one input and output");
    in_shape_ = static_shape(m.inputs[0]);
    out_shape_ = static_shape(m.outputs[0]);
    bool dyn = false;
    for (size_t k = 1; k < m.outputs[0].dims.size(); ++k) dyn |= m.outputs[0].dims[k] <= 0;
    if (dyn || m.outputs[0].dims.empty()) {  // infer with a dry run
      auto x = std::make_shared<CpuValue>();
      x->shape = in_shape_;
      x->f.assign(static_cast<size_t>(x->numel()), 0.f);
      out_shape_ = exec_.run(x)->shape;
      out_shape_[0] = 1;
    }
    pool_ = std::make_unique<SamplePool>(input_numel());
    worker_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "die-cpu-exec");
      loop();
    });
  }
  ~CpuEngine() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }

  std::string name() const override { return "cpu"; }
  const std::string& getModelPath() const override { return path_; }
  std::vector<int64_t> getInputShape() const override { return in_shape_; }
  std::vector<int64_t> getOutputShape() const override { return out_shape_; }
  int max_batch() const override { return opt_.max_batch; }
  SamplePool& sample_pool() override { return *pool_; }

  void wait_for_slot() override {
    std::unique_lock<std::mutex> lk(mu_);
    space_cv_.wait(lk, [&] { return q_.size() < 1 || stop_; });
  }

  void submit(std::vector<BatchItem> items, BatchDone done) override {
    std::unique_lock<std::mutex> lk(mu_);
    space_cv_.wait(lk, [&] { return q_.size() < 1 || stop_; });
    q_.push_back(Job{std::move(items), std::move(done), std::chrono::steady_clock::now()});
    ++inflight_;
    cv_.notify_all();
  }

  void synchronize() override {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [&] { return inflight_ == 0; });
  }

  Json stats() const override {
    Json j = Json::object();
    j["device"] = "cpu";
    j["batches"] = static_cast<long long>(batches_.load());
    j["images"] = static_cast<long long>(images_.load());
    j["options"] = engine_options_json(opt_);
    return j;
  }

 private:
  struct Job {
    std::vector<BatchItem> items;
    BatchDone done;
    std::chrono::steady_clock::time_point t0;
  };

  void loop() {
    while (true) {
      Job job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      space_cv_.notify_all();
      BatchResult r;
      std::vector<float> outbuf;
      try {
        if (opt_.fail_batch_every > 0 && ++nth_batch_ % opt_.fail_batch_every == 0)
          throw std::runtime_error("injected batch failure (fail_batch_every)");
        const size_t B = job.items.size(), numel = input_numel();
        auto x = std::make_shared<CpuValue>();
        x->shape = in_shape_;
        x->shape[0] = static_cast<int64_t>(B);
        x->f.assign(B * numel, 0.f);
        for (size_t i = 0; i < B; ++i) {
          const size_t n = std::min(job.items[i].len, numel);
          if (n) std::memcpy(x->f.data() + i * numel, job.items[i].input, n * sizeof(float));
        }
        auto y = exec_.run(x);
        outbuf = std::move(y->f);
        r.outputs = outbuf.data();
        r.output_numel = B ? outbuf.size() / B : 0;
        batches_++;
        images_ += B;
      } catch (const std::exception& e) {
        r.ok = false;
        r.error = e.what();
      }
      r.wall_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - job.t0).count();
      job.done(r);
      {
        std::lock_guard<std::mutex> g(mu_);
        --inflight_;
      }
      idle_cv_.notify_all();
    }
  }

  std::string path_;
  EngineOptions opt_;
  CpuExecutor exec_;
  std::vector<int64_t> in_shape_, out_shape_;
  std::unique_ptr<SamplePool> pool_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_, space_cv_, idle_cv_;
  std::deque<Job> q_;
  int inflight_ = 0;
  bool stop_ = false;
  long long nth_batch_ = 0;  // executor thread only (fault injection)
  std::atomic<long long> batches_{0}, images_{0};
};

}  // namespace

Json engine_options_json(const EngineOptions& o) {
  Json j = Json::object();
  j["device"] = o.device;
  j["device_id"] = o.device_id;
  j["max_batch"] = o.max_batch;
  j["precision"] = o.precision;
  j["pipeline_depth"] = o.pipeline_depth;
  j["exec_streams"] = o.exec_streams;
  j["use_graphs"] = o.use_graphs;
  j["autotune"] = o.autotune;
  j["device_decode"] = o.device_decode;
  j["stage_slots"] = o.stage_slots;
  j["pace"] = o.pace;
  j["pack_text"] = o.pack_text;
  j["branch_streams"] = o.branch_streams;
  j["prep_on_compute"] = o.prep_on_compute;
  j["live_batch"] = o.live_batch;
  j["tune_cache"] = o.tune_cache;
  j["cpu_threads"] = o.cpu_threads;
  j["dp_world"] = o.dp_world;
  j["dp_rank"] = o.dp_rank;
  j["dp_backend"] = o.dp_backend;
  j["dp_force_merge"] = o.dp_force_merge;
  j["copy_streams"] = o.copy_streams;
  j["bucket_div"] = o.bucket_div;
  j["coarse_buckets"] = o.coarse_buckets;
  j["pace_lead_scale"] = o.pace_lead_scale;
  j["completion_poll_us"] = o.completion_poll_us;
  j["bn_on_load"] = o.bn_on_load;
  j["fuse_pairs"] = o.fuse_pairs;
  j["fuse_stem_pool"] = o.fuse_stem_pool;
  j["fuse_gap_fc"] = o.fuse_gap_fc;
  j["fold_layernorm"] = o.fold_layernorm;
  j["ln_stats_epilogue"] = o.ln_stats_epilogue;
  j["tune_in_graph"] = o.tune_in_graph;
  j["tune_orders"] = o.tune_orders;
  j["tune_tail"] = o.tune_tail;
  j["tune_streamk"] = o.tune_streamk;
  j["efficient_batch"] = o.efficient_batch;
  j["efficient_batch_tol"] = o.efficient_batch_tol;
  j["efficient_batch_margin"] = o.efficient_batch_margin;
  j["batch_curve_median"] = o.batch_curve_median;
  j["efficient_batch_ends"] = o.efficient_batch_ends;
  j["tune_cold"] = o.tune_cold;
  j["tune_warm_input"] = o.tune_warm_input;
  j["splitk_fused_margin"] = o.splitk_fused_margin;
  j["splitk_two_kernel"] = o.splitk_two_kernel;
  j["result_stream"] = o.result_stream;
  j["conv_order"] = o.conv_order;
  j["fail_batch_every"] = o.fail_batch_every;
  return j;
}

int pick_efficient_batch(const double* ms, int max_b, int queued, double tol, double margin, const int* ends,
                         int n_ends) {
  const int q = std::min(queued, max_b);
  if (!ms || q <= 1) return std::max(1, q);
  if (ends && n_ends > 0) {  // bucket ends only: the cheapest per image, the largest within tol of it
    double best = 1e30;
    for (int i = 0; i < n_ends && ends[i] <= q; ++i) best = std::min(best, ms[ends[i]] / ends[i]);
    if (best >= 1e30) return q;
    const double lim = best * (1.0 + std::max(0.0, tol));
    int pick = 1;
    for (int i = 0; i < n_ends && ends[i] <= q; ++i)
      if (ms[ends[i]] / ends[i] <= lim) pick = ends[i];
    return pick;
  }
  double best = 1e30;
  for (int b = 1; b <= q; ++b) best = std::min(best, ms[b] / b);
  // the whole queue unless a smaller batch is clearly cheaper per image
  if (ms[q] / q * (1.0 - std::max(0.0, margin)) <= best) return q;
  const double lim = best * (1.0 + std::max(0.0, tol));
  for (int b = q - 1; b > 1; --b)
    if (ms[b] / b <= lim) return b;
  return 1;
}

std::unique_ptr<Engine> create_cpu_engine(const std::string& model_path, const EngineOptions& opt) {
  return std::make_unique<CpuEngine>(model_path, opt);
}

std::unique_ptr<Engine> create_engine(const std::string& model_path, const EngineOptions& opt) {
  if (opt.precision != "bf16" && opt.precision != "fp32")
    throw std::runtime_error("unknown precision '" + opt.precision + "' (bf16 | fp32)");
  // fp32 (default, the reference's ORT numerics): on the HIP engine every GEMM runs on split hi/lo
  // bf16 operands with fp32 accumulation (kernels/common.h); bf16 is the opt-in fast mode.
  if (opt.dp_world >= 1 && !opt.dp_group.empty() && opt.dp_comm == nullptr) return create_dp_engine(model_path, opt);
  if (opt.device != "cpu") {
    std::string why;
    std::unique_ptr<Engine> e;
    bool unlowerable = false;
    try {
      e = create_hip_engine(model_path, opt, &why);
    } catch (const PlanUnsupported& ex) {
      why = ex.what();
      unlowerable = true;
    } catch (const std::exception& ex) {
      why = ex.what();
      if (opt.device == "hip") throw;
    }
    if (e) return e;
    if (unlowerable) {
      // the reference's per-node EP fallback (src/inference_engine.cpp:21-31): the nodes the HIP
      // planner cannot lower run on the CPU executor, every other piece stays on the GPU
      std::string why2;
      try {
        e = create_hybrid_engine(model_path, opt, &why2);
      } catch (const std::exception& ex) {
        why2 = ex.what();
      }
      if (e) {
        // device "hip" asked for GPU execution: say loudly that part of the graph runs on the CPU
        if (opt.device == "hip")
          DIE_LOG(WARN, "device=hip: the graph has nodes the HIP planner cannot lower; serving it as " << e->name()
                                                                                                      << " (CPU islands)");
        return e;
      }
      DIE_LOG(WARN, "hybrid HIP + CPU partition unavailable: " << why2);
      if (opt.device == "hip") throw std::runtime_error(why);
    }
    if (opt.device == "hip") throw std::runtime_error("HIP engine unavailable: " + why);
    DIE_LOG(WARN, "HIP engine unavailable (" << why << "); falling back to the CPU executor");
  }
  return create_cpu_engine(model_path, opt);
}

}  // namespace die
