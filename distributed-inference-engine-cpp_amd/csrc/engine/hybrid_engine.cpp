// Hybrid HIP + CPU execution: the reference's per-node execution-provider fallback.
//
// The reference appends ORT's CUDA EP, then the CPU EP, and creates the session on any model
// (/root/reference/src/inference_engine.cpp:21-31): ORT places each node the CUDA EP cannot run on
// the CPU and keeps the rest on the GPU, copying tensors across at the boundaries.  Here the HIP
// planner lowers whole graphs, so the same effect is built one level up:
//   1. cut points: positions in the topological order where exactly ONE non-constant tensor is live
//      (ResNet unit boundaries, transformer layer boundaries, ...).  Every piece between two cuts is
//      a single-input, single-output graph of its own;
//   2. a piece runs on the HIP engine when the planner lowers it and it holds GEMM work (Conv,
//      Gemm, MatMul), else on the CPU executor; neighbours on the same device merge;
//   3. at run time a batch flows through the segments in order, each HIP segment being a full HIP
//      engine (hipGraphs, autotuned kernels) fed from and read back to host memory: the H2D / D2H
//      at every boundary are the copies ORT's EP partitioning inserts.
// A graph whose every piece lowers keeps the plain HIP engine (no segment boundaries at all).
#include <pthread.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <future>
#include <mutex>
#include <set>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "../core/log.h"
#include "cpu_exec.h"
#include "engine.h"
#include "hip_plan.h"

namespace die {

namespace {

bool gemm_op(const std::string& op) { return op == "Conv" || op == "Gemm" || op == "MatMul" || op == "ConvTranspose"; }

// Sub-model of nodes [first, last] reading tensor `in` (per-sample shape in_shape, batch dynamic)
// and producing `out`.
onnx::Model sub_model(const onnx::Model& m, int first, int last, const std::string& in, const std::vector<int64_t>& in_shape,
                      const std::string& out, const std::vector<int64_t>& out_shape) {
  onnx::Model s;
  s.ir_version = m.ir_version;
  s.opsets = m.opsets;
  s.producer_name = m.producer_name;
  s.graph_name = m.graph_name + "[" + std::to_string(first) + ":" + std::to_string(last) + "]";
  for (int k = first; k <= last; ++k) {
    const onnx::Node& n = m.nodes[static_cast<size_t>(k)];
    s.nodes.push_back(n);
    for (const auto& x : n.inputs) {
      auto it = m.initializers.find(x);
      if (it != m.initializers.end()) s.initializers.emplace(x, it->second);
    }
  }
  auto vi = [](const std::string& name, const std::vector<int64_t>& shape) {
    onnx::ValueInfo v;
    v.name = name;
    v.dims = shape;
    if (!v.dims.empty()) v.dims[0] = -1;
    v.dim_params.assign(v.dims.size(), "");
    if (!v.dim_params.empty()) v.dim_params[0] = "N";
    return v;
  };
  s.inputs.push_back(vi(in, in_shape));
  s.outputs.push_back(vi(out, out_shape));
  return s;
}

struct Cut {
  int after;           // node index the cut follows (-1: before the first node)
  std::string tensor;  // the one live tensor
};

std::vector<Cut> cut_points(const onnx::Model& m) {
  const int N = static_cast<int>(m.nodes.size());
  std::unordered_map<std::string, int> last_use;
  for (int k = 0; k < N; ++k)
    for (const auto& x : m.nodes[static_cast<size_t>(k)].inputs)
      if (!x.empty() && !m.initializers.count(x)) last_use[x] = k;
  for (const auto& o : m.outputs) last_use[o.name] = N;
  // every graph input that is read (not only input 0): a second input live across a candidate cut
  // makes it a two-tensor point, so it is no cut; initializers listed as graph inputs
  // (IR v3 models) are weights, not live state
  std::unordered_set<std::string> live;
  for (const auto& in : m.inputs)
    if (!m.initializers.count(in.name) && last_use.count(in.name)) live.insert(in.name);
  std::vector<Cut> cuts;
  if (live.size() == 1) cuts.push_back(Cut{-1, *live.begin()});
  for (int k = 0; k < N; ++k) {
    const onnx::Node& n = m.nodes[static_cast<size_t>(k)];
    for (const auto& x : n.inputs) {
      auto it = last_use.find(x);
      if (it != last_use.end() && it->second == k) live.erase(x);
    }
    for (const auto& y : n.outputs) {
      auto it = last_use.find(y);
      if (!y.empty() && it != last_use.end() && it->second > k) live.insert(y);
    }
    if (live.size() == 1) cuts.push_back(Cut{k, *live.begin()});
  }
  return cuts;
}

std::vector<int64_t> per_sample(std::vector<int64_t> s) {
  if (!s.empty()) s[0] = 1;
  return s;
}

}  // namespace

std::vector<HybridSegment> hybrid_partition(const onnx::Model& m, int max_batch, bool split) {
  if (m.inputs.empty() || m.outputs.empty()) throw std::runtime_error("model needs an input and an output");
  // shapes of every value: one batch-1 pass of the CPU executor
  std::vector<int64_t> in_shape = m.inputs[0].dims;
  for (auto& d : in_shape)
    if (d <= 0) d = 1;
  in_shape[0] = 1;
  CpuExecutor ex(m);
  auto x = std::make_shared<CpuValue>();
  x->shape = in_shape;
  x->f.assign(static_cast<size_t>(x->numel()), 0.f);
  std::unordered_map<std::string, CpuValuePtr> trace;
  ex.run(x, &trace);
  trace[m.inputs[0].name] = x;
  auto shape_of = [&](const std::string& t) {
    auto it = trace.find(t);
    if (it == trace.end()) throw std::runtime_error("hybrid partition: no shape for " + t);
    return per_sample(it->second->shape);
  };

  const std::vector<Cut> cuts = cut_points(m);
  const int N = static_cast<int>(m.nodes.size());
  if (cuts.empty() || cuts.front().after != -1 || cuts.back().after != N - 1)
    throw std::runtime_error("hybrid partition: the graph has no single-tensor cut at its input and output");
  // pieces between consecutive cuts
  std::vector<HybridSegment> pieces;
  std::vector<int> piece_of(static_cast<size_t>(N), -1);
  for (size_t c = 0; c + 1 < cuts.size(); ++c) {
    HybridSegment s;
    s.first = cuts[c].after + 1;
    s.last = cuts[c + 1].after;
    if (s.first > s.last) continue;
    s.input = cuts[c].tensor;
    s.output = cuts[c + 1].tensor;
    s.in_shape = shape_of(s.input);
    for (int k = s.first; k <= s.last; ++k) {
      s.convs += gemm_op(m.nodes[static_cast<size_t>(k)].op_type);
      piece_of[static_cast<size_t>(k)] = static_cast<int>(pieces.size());
    }
    pieces.push_back(std::move(s));
  }
  std::unordered_map<std::string, int> node_index;
  for (int k = 0; k < N; ++k) node_index[m.nodes[static_cast<size_t>(k)].name] = k;
  // A piece is CPU ("bad") if it holds a node the planner cannot lower.  Start from the whole
  // model's report (nodes downstream of an unsupported one are only "blocked" there), then plan
  // every maximal run of good pieces on its own and mark the pieces of any node it still rejects,
  // until every HIP run plans.  A run whose failure names no node is split off piece by piece.
  std::vector<bool> bad(pieces.size(), false);
  auto mark = [&](const PlanReport& r) {
    bool any = false;
    for (const auto& it : r.unsupported) {
      auto k = node_index.find(it.node);
      if (k != node_index.end() && piece_of[static_cast<size_t>(k->second)] >= 0 &&
          !bad[static_cast<size_t>(piece_of[static_cast<size_t>(k->second)])]) {
        bad[static_cast<size_t>(piece_of[static_cast<size_t>(k->second)])] = true;
        any = true;
      }
    }
    return any;
  };
  mark(plan_report(m, max_batch, split));
  auto runs = [&]() {  // maximal runs of equal `bad`: [begin, end)
    std::vector<std::pair<size_t, size_t>> out;
    for (size_t i = 0; i < pieces.size();) {
      size_t j = i;
      while (j < pieces.size() && bad[j] == bad[i]) ++j;
      out.emplace_back(i, j);
      i = j;
    }
    return out;
  };
  auto run_model = [&](size_t b, size_t e) {
    return sub_model(m, pieces[b].first, pieces[e - 1].last, pieces[b].input, pieces[b].in_shape, pieces[e - 1].output,
                     shape_of(pieces[e - 1].output));
  };
  for (bool changed = true; changed;) {
    changed = false;
    for (const auto& r : runs()) {
      if (bad[r.first]) continue;
      const PlanReport rep = plan_report(run_model(r.first, r.second), max_batch, split);
      if (rep.supported) continue;
      DIE_LOG(DEBUG, "hybrid partition: nodes " << pieces[r.first].first << ".." << pieces[r.second - 1].last
                                                << " do not plan:\n" << rep.text());
      if (!mark(rep)) bad[r.first] = true;  // nothing named: give up the run's first piece
      changed = true;
      break;
    }
  }
  // a HIP run without GEMM work is not worth two host round trips: CPU
  for (const auto& r : runs()) {
    if (bad[r.first]) continue;
    int g = 0;
    for (size_t i = r.first; i < r.second; ++i) g += pieces[i].convs;
    if (g == 0)
      for (size_t i = r.first; i < r.second; ++i) bad[i] = true;
  }
  std::vector<HybridSegment> segs;
  for (const auto& r : runs()) {
    HybridSegment s = pieces[r.first];
    s.hip = !bad[r.first];
    s.last = pieces[r.second - 1].last;
    s.output = pieces[r.second - 1].output;
    s.convs = 0;
    for (size_t i = r.first; i < r.second; ++i) s.convs += pieces[i].convs;
    segs.push_back(std::move(s));
  }
  return segs;
}

namespace {

class HybridEngine : public Engine {
 public:
  HybridEngine(const std::string& path, const EngineOptions& opt, onnx::Model m, std::vector<HybridSegment> segs)
      : path_(path), opt_(opt), model_(std::move(m)), segs_(std::move(segs)) {
    shard_id_ = opt.shard_id;
    in_shape_ = segs_.front().in_shape;
    // shapes again for the outputs (per sample)
    EngineOptions so = opt;
    so.device = "hip";
    so.device_decode = false;  // segment inputs are host floats
    so.pack_text = false;
    so.dp_world = 0;
    so.dp_group.clear();
    for (size_t i = 0; i < segs_.size(); ++i) {
      const HybridSegment& s = segs_[i];
      const std::vector<int64_t> out_shape =
          i + 1 < segs_.size() ? segs_[i + 1].in_shape : std::vector<int64_t>{};
      Stage st;
      onnx::Model sm = sub_model(model_, s.first, s.last, s.input, s.in_shape, s.output,
                                 out_shape.empty() ? model_.outputs[0].dims : out_shape);
      if (s.hip) {
        std::string why;
        st.hip = create_hip_engine_model(path + "#" + std::to_string(i), std::move(sm), so, &why);
        if (!st.hip) throw std::runtime_error("hybrid engine: HIP segment " + std::to_string(i) + ": " + why);
      } else {
        st.cpu = std::make_unique<CpuExecutor>(std::move(sm));
      }
      st.in_numel = 1;
      for (auto d : s.in_shape) st.in_numel *= static_cast<size_t>(d);
      stages_.push_back(std::move(st));
    }
    // output shape: a dry run of the whole chain on one zero sample
    std::vector<float> zero(input_numel(), 0.f);
    std::vector<float> y = run_chain(zero.data(), 1, nullptr);
    out_shape_ = {1, static_cast<int64_t>(y.size())};
    if (model_.outputs[0].dims.size() > 1) {
      std::vector<int64_t> d = model_.outputs[0].dims;
      size_t n = 1;
      for (size_t k = 1; k < d.size(); ++k) n *= static_cast<size_t>(std::max<int64_t>(1, d[k]));
      if (n == y.size()) {
        d[0] = 1;
        out_shape_ = d;
      }
    }
    pool_ = std::make_unique<SamplePool>(input_numel());
    worker_ = std::thread([this] {
      pthread_setname_np(pthread_self(), "die-hybrid");
      loop();
    });
    int hip = 0, cpu = 0;
    for (auto& s : segs_) (s.hip ? hip : cpu) += s.convs;
    DIE_LOG(INFO, "hybrid engine: " << segs_.size() << " segments, GEMM nodes " << hip << " on HIP / " << cpu
                                    << " on the CPU executor");
  }
  ~HybridEngine() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }

  std::string name() const override {
    std::string n = "hybrid(";
    for (size_t i = 0; i < segs_.size(); ++i) n += std::string(i ? "," : "") + (segs_[i].hip ? "hip" : "cpu");
    return n + ")";
  }
  const std::string& getModelPath() const override { return path_; }
  std::vector<int64_t> getInputShape() const override { return in_shape_; }
  std::vector<int64_t> getOutputShape() const override { return out_shape_; }
  int max_batch() const override { return std::max(1, opt_.max_batch); }
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
    j["device"] = "hip+cpu";
    j["name"] = name();
    j["batches"] = static_cast<long long>(batches_.load());
    j["images"] = static_cast<long long>(images_.load());
    Json segs = Json::array();
    int hip = 0, all = 0;
    for (size_t i = 0; i < segs_.size(); ++i) {
      const HybridSegment& s = segs_[i];
      Json e = Json::object();
      e["device"] = s.hip ? "hip" : "cpu";
      e["nodes"] = s.last - s.first + 1;
      e["gemm_nodes"] = s.convs;
      e["first_node"] = model_.nodes[static_cast<size_t>(s.first)].name;
      e["last_node"] = model_.nodes[static_cast<size_t>(s.last)].name;
      e["input"] = s.input;
      e["output"] = s.output;
      e["ms_total"] = seg_ms_[i].load() / 1e3;
      segs.push_back(e);
      all += s.convs;
      if (s.hip) hip += s.convs;
    }
    j["segments"] = segs;
    j["gemm_nodes_on_hip"] = hip;
    j["gemm_nodes_total"] = all;
    j["options"] = engine_options_json(opt_);
    return j;
  }

 private:
  struct Stage {
    std::unique_ptr<Engine> hip;
    std::unique_ptr<CpuExecutor> cpu;
    size_t in_numel = 0;
  };
  struct Job {
    std::vector<BatchItem> items;
    BatchDone done;
    std::chrono::steady_clock::time_point t0;
  };

  // B samples of the first segment's input (dense rows) through every segment; returns B rows.
  std::vector<float> run_chain(const float* x0, size_t B, std::atomic<long long>* seg_us) {
    std::vector<float> cur(x0, x0 + B * stages_.front().in_numel), next;
    for (size_t i = 0; i < stages_.size(); ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      Stage& st = stages_[i];
      const size_t n_in = st.in_numel;
      if (st.hip) {
        // the HIP engine batches up to its max; feed it in chunks and wait for each
        const size_t mb = static_cast<size_t>(st.hip->max_batch());
        next.clear();
        for (size_t b0 = 0; b0 < B; b0 += mb) {
          const size_t nb = std::min(mb, B - b0);
          std::vector<BatchItem> items;
          for (size_t b = 0; b < nb; ++b) items.push_back(BatchItem{cur.data() + (b0 + b) * n_in, n_in});
          std::promise<std::vector<float>> pr;
          auto fut = pr.get_future();
          st.hip->submit(std::move(items), [&pr, nb](BatchResult& r) {
            if (!r.ok) {
              pr.set_exception(std::make_exception_ptr(std::runtime_error(r.error)));
              return;
            }
            pr.set_value(std::vector<float>(r.outputs, r.outputs + nb * r.output_numel));
          });
          std::vector<float> part = fut.get();
          next.insert(next.end(), part.begin(), part.end());
        }
      } else {
        auto v = std::make_shared<CpuValue>();
        v->shape = segs_[i].in_shape;
        v->shape[0] = static_cast<int64_t>(B);
        v->f = std::move(cur);
        next = std::move(st.cpu->run(v)->f);
      }
      cur.swap(next);
      if (seg_us)
        seg_us[i].fetch_add(
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count());
    }
    return cur;
  }

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
      std::vector<float> out;
      try {
        const size_t B = job.items.size(), numel = input_numel();
        std::vector<float> x(B * numel, 0.f);
        for (size_t i = 0; i < B; ++i) {
          const size_t n = std::min(job.items[i].len, numel);
          if (n) std::memcpy(x.data() + i * numel, job.items[i].input, n * sizeof(float));
        }
        out = run_chain(x.data(), B, seg_ms_);
        r.outputs = out.data();
        r.output_numel = B ? out.size() / B : 0;
        batches_++;
        images_ += static_cast<long long>(B);
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
  onnx::Model model_;
  std::vector<HybridSegment> segs_;
  std::vector<Stage> stages_;
  std::vector<int64_t> in_shape_, out_shape_;
  std::unique_ptr<SamplePool> pool_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_, space_cv_, idle_cv_;
  std::deque<Job> q_;
  int inflight_ = 0;
  bool stop_ = false;
  std::atomic<long long> batches_{0}, images_{0};
  std::atomic<long long> seg_ms_[64] = {};  // microseconds per segment (name kept for the stats key)
};

}  // namespace

std::unique_ptr<Engine> create_hybrid_engine(const std::string& model_path, const EngineOptions& opt, std::string* why) {
  onnx::Model m = onnx::load_onnx(model_path);
  std::vector<HybridSegment> segs = hybrid_partition(m, std::max(1, opt.max_batch), opt.precision == "fp32");
  bool any_hip = false, any_cpu = false;
  for (auto& s : segs) (s.hip ? any_hip : any_cpu) = true;
  if (!any_hip || !any_cpu || segs.size() > 64) {
    if (why) *why = !any_hip ? "no segment lowers for the HIP engine" : !any_cpu ? "no CPU island needed" : "too many segments";
    return nullptr;
  }
  return std::make_unique<HybridEngine>(model_path, opt, std::move(m), std::move(segs));
}

}  // namespace die
