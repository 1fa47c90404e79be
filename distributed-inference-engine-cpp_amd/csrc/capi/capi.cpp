// C ABI over the native runtime, loaded from Python with ctypes (die_amd/native.py).
// Options travel as JSON strings; returned strings are malloc'ed and released with die_free().
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <string>
#include <thread>
#include <mutex>
#include <atomic>

#include "../core/json.h"
#include "../core/textpack.h"
#include "../engine/cpu_exec.h"
#include "../engine/engine.h"
#include "../serve/circuit_breaker.h"
#include "../serve/consistent_hash.h"
#include "../serve/gateway.h"
#include "../serve/loadgen.h"
#include "../parallel/dp_layout.h"
#include "../serve/lru_cache.h"
#include "../serve/worker.h"

using namespace die;

namespace {

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}

void set_err(char** err, const std::string& m) {
  if (err) *err = dup(m);
}

template <typename T>
T jget(const Json& j, const char* k, T d);
template <>
int jget(const Json& j, const char* k, int d) {
  auto* v = j.find(k);
  return v ? static_cast<int>(v->as_int()) : d;
}
template <>
long jget(const Json& j, const char* k, long d) {
  auto* v = j.find(k);
  return v ? static_cast<long>(v->as_int()) : d;
}
template <>
double jget(const Json& j, const char* k, double d) {
  auto* v = j.find(k);
  return v ? v->as_double() : d;
}
template <>
bool jget(const Json& j, const char* k, bool d) {
  auto* v = j.find(k);
  return v ? v->as_bool() : d;
}
template <>
std::string jget(const Json& j, const char* k, std::string d) {
  auto* v = j.find(k);
  return v ? v->as_string() : d;
}

EngineOptions engine_opts(const Json& j) {
  EngineOptions e;
  e.device = jget<std::string>(j, "device", e.device);
  e.device_id = jget<int>(j, "device_id", e.device_id);
  e.max_batch = jget<int>(j, "max_batch", e.max_batch);
  e.pipeline_depth = jget<int>(j, "pipeline_depth", e.pipeline_depth);
  e.use_graphs = jget<bool>(j, "use_graphs", e.use_graphs);
  e.autotune = jget<bool>(j, "autotune", e.autotune);
  e.device_decode = jget<bool>(j, "device_decode", e.device_decode);
  e.stage_slots = jget<int>(j, "stage_slots", e.stage_slots);
  e.pace = jget<bool>(j, "pace", e.pace);
  e.pack_text = jget<bool>(j, "pack_text", e.pack_text);
  e.branch_streams = jget<bool>(j, "branch_streams", e.branch_streams);
  e.prep_on_compute = jget<bool>(j, "prep_on_compute", e.prep_on_compute);
  e.live_batch = jget<bool>(j, "live_batch", e.live_batch);
  e.exec_streams = jget<int>(j, "exec_streams", e.exec_streams);
  e.tune_cache = jget<std::string>(j, "tune_cache", e.tune_cache);
  e.precision = jget<std::string>(j, "precision", e.precision);
  e.shard_id = jget<int>(j, "shard_id", e.shard_id);
  e.dp_world = jget<int>(j, "dp_world", e.dp_world);
  e.dp_rank = jget<int>(j, "dp_rank", e.dp_rank);
  e.dp_group = jget<std::string>(j, "dp_group", e.dp_group);
  e.dp_arena_mb = static_cast<size_t>(jget<long>(j, "dp_arena_mb", 0));
  e.dp_backend = jget<std::string>(j, "dp_backend", e.dp_backend);
  e.dp_force_merge = jget<bool>(j, "dp_force_merge", e.dp_force_merge);
  e.cpu_threads = jget<int>(j, "cpu_threads", e.cpu_threads);
  e.copy_streams = jget<int>(j, "copy_streams", e.copy_streams);
  e.bucket_div = jget<int>(j, "bucket_div", e.bucket_div);
  e.coarse_buckets = jget<bool>(j, "coarse_buckets", e.coarse_buckets);
  e.pace_lead_scale = jget<double>(j, "pace_lead_scale", e.pace_lead_scale);
  e.completion_poll_us = jget<int>(j, "completion_poll_us", e.completion_poll_us);
  e.bn_on_load = jget<bool>(j, "bn_on_load", e.bn_on_load);
  e.fuse_pairs = jget<bool>(j, "fuse_pairs", e.fuse_pairs);
  e.fuse_stem_pool = jget<bool>(j, "fuse_stem_pool", e.fuse_stem_pool);
  e.fuse_gap_fc = jget<bool>(j, "fuse_gap_fc", e.fuse_gap_fc);
  e.fold_layernorm = jget<bool>(j, "fold_layernorm", e.fold_layernorm);
  e.ln_stats_epilogue = jget<bool>(j, "ln_stats_epilogue", e.ln_stats_epilogue);
  e.tune_in_graph = jget<bool>(j, "tune_in_graph", e.tune_in_graph);
  e.tune_orders = jget<bool>(j, "tune_orders", e.tune_orders);
  e.tune_tail = jget<bool>(j, "tune_tail", e.tune_tail);
  e.tune_streamk = jget<bool>(j, "tune_streamk", e.tune_streamk);
  e.efficient_batch = jget<bool>(j, "efficient_batch", e.efficient_batch);
  e.efficient_batch_tol = jget<double>(j, "efficient_batch_tol", e.efficient_batch_tol);
  e.efficient_batch_margin = jget<double>(j, "efficient_batch_margin", e.efficient_batch_margin);
  e.batch_curve_median = jget<bool>(j, "batch_curve_median", e.batch_curve_median);
  e.efficient_batch_ends = jget<bool>(j, "efficient_batch_ends", e.efficient_batch_ends);
  e.tune_cold = jget<bool>(j, "tune_cold", e.tune_cold);
  e.tune_warm_input = jget<bool>(j, "tune_warm_input", e.tune_warm_input);
  e.splitk_fused_margin = static_cast<float>(jget<double>(j, "splitk_fused_margin", e.splitk_fused_margin));
  e.splitk_two_kernel = jget<bool>(j, "splitk_two_kernel", e.splitk_two_kernel);
  e.result_stream = jget<bool>(j, "result_stream", e.result_stream);
  e.conv_order = jget<int>(j, "conv_order", e.conv_order);
  e.fail_batch_every = jget<int>(j, "fail_batch_every", e.fail_batch_every);
  return e;
}

}  // namespace

extern "C" {

void die_free(void* p) { std::free(p); }

const char* die_version() { return "die_amd 0.1.0"; }

// ---- JSON ----
char* die_json_roundtrip(const char* text, char** err) {
  try {
    return dup(Json::parse(text).dump());
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

// Parses an /infer body: writes up to `cap` floats, returns count (-1 on error, message in err).
long die_parse_infer(const char* body, long n, float* out, long cap, char** id_out, char** err) {
  struct S : InferBodySink {
    float* o;
    size_t c;
    size_t n = 0;
    std::string id;
    void on_request_id(std::string_view s) override { id = s; }
    float* input_buffer() override { return o; }
    size_t input_capacity() const override { return c; }
    void on_input_count(size_t k) override { n = k; }
  } s;
  s.o = out;
  s.c = static_cast<size_t>(cap);
  try {
    std::string b(body, static_cast<size_t>(n));
    b.reserve(b.size() + 64);
    parse_infer_body(b, s);
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return -1;
  }
  if (id_out) *id_out = dup(s.id);
  return static_cast<long>(s.n);
}

char* die_format_floats(const float* v, long n) {
  std::string s;
  append_float_array(s, v, static_cast<size_t>(n));
  return dup(s);
}

// ---- ring / breaker / cache (unit tests) ----
uint32_t die_fnv1a(const char* s) { return ConsistentHash::fnv1a(s); }

void* die_ring_create(int vnodes) { return new ConsistentHash(vnodes); }
void die_ring_destroy(void* r) { delete static_cast<ConsistentHash*>(r); }
void die_ring_add(void* r, const char* n) { static_cast<ConsistentHash*>(r)->addNode(n); }
void die_ring_remove(void* r, const char* n) { static_cast<ConsistentHash*>(r)->removeNode(n); }
char* die_ring_get(void* r, const char* k) { return dup(static_cast<ConsistentHash*>(r)->getNode(k)); }
char* die_ring_nodes(void* r) {
  Json a = Json::array();
  for (auto& n : static_cast<ConsistentHash*>(r)->getAllNodes()) a.push_back(n);
  return dup(a.dump());
}
long die_ring_size(void* r) { return static_cast<long>(static_cast<ConsistentHash*>(r)->ringSize()); }

struct FakeClockBreaker {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::time_point{} + std::chrono::hours(1);
  std::unique_ptr<CircuitBreaker> b;
};
void* die_breaker_create(int fail_thr, int succ_thr, long timeout_ms) {
  auto* f = new FakeClockBreaker();
  f->b = std::make_unique<CircuitBreaker>(fail_thr, succ_thr, std::chrono::milliseconds(timeout_ms),
                                          [f] { return f->t; });
  return f;
}
void die_breaker_destroy(void* p) { delete static_cast<FakeClockBreaker*>(p); }
void die_breaker_advance(void* p, long ms) { static_cast<FakeClockBreaker*>(p)->t += std::chrono::milliseconds(ms); }
int die_breaker_allow(void* p) { return static_cast<FakeClockBreaker*>(p)->b->allowRequest() ? 1 : 0; }
void die_breaker_success(void* p) { static_cast<FakeClockBreaker*>(p)->b->recordSuccess(); }
void die_breaker_failure(void* p) { static_cast<FakeClockBreaker*>(p)->b->recordFailure(); }
char* die_breaker_state(void* p) {
  auto* b = static_cast<FakeClockBreaker*>(p)->b.get();
  Json j = Json::object();
  j["state"] = b->getStateString();
  j["failures"] = b->getFailureCount();
  j["successes"] = b->getSuccessCount();
  return dup(j.dump());
}

using FCache = LRUCache<InputKey, std::vector<float>, InputKeyHash>;
void* die_cache_create(long cap) { return new FCache(static_cast<size_t>(cap)); }
void die_cache_destroy(void* c) { delete static_cast<FCache*>(c); }
void die_cache_put(void* c, const float* k, long kn, const float* v, long vn) {
  static_cast<FCache*>(c)->put(hash_floats(k, static_cast<size_t>(kn)), std::vector<float>(v, v + vn));
}
// Returns value length (copied into out up to cap), or -1 on miss.
long die_cache_get(void* c, const float* k, long kn, float* out, long cap) {
  auto r = static_cast<FCache*>(c)->get(hash_floats(k, static_cast<size_t>(kn)));
  if (!r) return -1;
  std::memcpy(out, r->data(), sizeof(float) * std::min<size_t>(r->size(), static_cast<size_t>(cap)));
  return static_cast<long>(r->size());
}
char* die_cache_stats(void* c) {
  auto* p = static_cast<FCache*>(c);
  Json j = Json::object();
  j["size"] = static_cast<long long>(p->size());
  j["hits"] = static_cast<long long>(p->getHits());
  j["misses"] = static_cast<long long>(p->getMisses());
  j["hit_rate"] = p->getHitRate();
  return dup(j.dump());
}

// ---- batcher (unit tests): echo batches, records batch sizes ----
struct TestBatcher {
  std::unique_ptr<BatchProcessor<int, int>> bp;
  std::mutex mu;
  std::vector<int> sizes;
  int delay_ms = 0;
};
// size_cap > 0: a batch-size function (Engine::preferred_batch's hook) that takes at most size_cap
// balance: WorkerOptions::batch_balance (BatchProcessor::set_balance)
void* die_batcher_create(int max_batch, int timeout_ms, int deadline_policy, int delay_ms, int size_cap, int balance) {
  auto* t = new TestBatcher();
  t->delay_ms = delay_ms;
  t->bp = std::make_unique<BatchProcessor<int, int>>(
      static_cast<size_t>(max_batch), std::chrono::milliseconds(timeout_ms),
      [t](const std::vector<int>& reqs) {
        {
          std::lock_guard<std::mutex> g(t->mu);
          t->sizes.push_back(static_cast<int>(reqs.size()));
        }
        if (t->delay_ms) std::this_thread::sleep_for(std::chrono::milliseconds(t->delay_ms));
        std::vector<int> out;
        for (int r : reqs) {
          if (r < 0) throw std::runtime_error("negative request");
          out.push_back(r * 2);
        }
        return out;
      },
      deadline_policy ? BatchPolicy::DEADLINE : BatchPolicy::GREEDY);
  if (size_cap > 0)
    t->bp->set_size_fn([cap = static_cast<size_t>(size_cap)](size_t q) { return q > cap ? cap : q; });
  t->bp->set_balance(balance != 0);
  t->bp->start();
  return t;
}
int die_batcher_process(void* p, int v, char** err) {
  try {
    return static_cast<TestBatcher*>(p)->bp->process(v);
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return -1;
  }
}
char* die_batcher_metrics(void* p) {
  auto* t = static_cast<TestBatcher*>(p);
  auto m = t->bp->getMetrics();
  Json j = Json::object();
  j["total_requests"] = static_cast<long long>(m.total_requests);
  j["total_batches"] = static_cast<long long>(m.total_batches);
  j["timeout_batches"] = static_cast<long long>(m.timeout_batches);
  j["full_batches"] = static_cast<long long>(m.full_batches);
  j["avg_batch_size"] = m.avg_batch_size;
  j["trimmed_batches"] = t->bp->trimmed_batches();
  j["trimmed_requests"] = t->bp->trimmed_requests();
  Json hist = Json::array();
  const auto sh = t->bp->size_histogram();
  for (size_t i = 1; i < sh.size(); ++i) hist.push_back(sh[i]);
  j["size_histogram"] = hist;
  Json s = Json::array();
  {
    std::lock_guard<std::mutex> g(t->mu);
    for (int v : t->sizes) s.push_back(v);
  }
  j["sizes"] = s;
  return dup(j.dump());
}
void die_batcher_stop(void* p) { static_cast<TestBatcher*>(p)->bp->stop(); }
void die_batcher_destroy(void* p) { delete static_cast<TestBatcher*>(p); }

// ---- engine ----
void* die_engine_create(const char* model_path, const char* opts_json, char** err) {
  try {
    Json j = opts_json && *opts_json ? Json::parse(opts_json) : Json::object();
    return create_engine(model_path, engine_opts(j)).release();
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}
void die_engine_destroy(void* e) { delete static_cast<Engine*>(e); }
char* die_engine_profile(void* p, int B, int iters) { return dup(static_cast<Engine*>(p)->profile_ops(B, iters).dump()); }
char* die_engine_info(void* p) {
  auto* e = static_cast<Engine*>(p);
  Json j = e->stats();
  j["name"] = e->name();
  Json in = Json::array(), out = Json::array();
  for (auto d : e->getInputShape()) in.push_back(static_cast<long long>(d));
  for (auto d : e->getOutputShape()) out.push_back(static_cast<long long>(d));
  j["input_shape"] = in;
  j["output_shape"] = out;
  j["max_batch"] = e->max_batch();
  return dup(j.dump());
}
// `in`: B samples of `len` floats each (len <= input numel; zero-padded).  `out`: B * output numel.
int die_engine_run(void* p, const float* in, long B, long len, float* out, char** err) {
  auto* e = static_cast<Engine*>(p);
  try {
    std::vector<std::vector<float>> xs(static_cast<size_t>(B));
    for (long b = 0; b < B; ++b) xs[b].assign(in + b * len, in + (b + 1) * len);
    auto ys = e->batchPredict(xs);
    const size_t on = e->output_numel();
    for (long b = 0; b < B; ++b) std::memcpy(out + b * on, ys[b].data(), on * sizeof(float));
    return 0;
  } catch (const std::exception& ex) {
    set_err(err, ex.what());
    return -1;
  }
}

// 4-bit text packing (core/textpack.h): returns 1 if packed, 0 if a byte is outside the alphabet.
int die_pack_nibbles(const char* src, long long n, unsigned char* dst) { return pack_nibbles(src, static_cast<size_t>(n), dst) ? 1 : 0; }
void die_unpack_nibbles(const unsigned char* src, long long n, char* dst) { unpack_nibbles(src, static_cast<size_t>(n), dst); }
int die_engine_preferred_batch(void* p, int queued) { return static_cast<Engine*>(p)->preferred_batch(queued); }
int die_pick_efficient_batch(const double* ms, int max_b, int queued, double tol, double margin, const int* ends,
                             int n_ends) {
  return pick_efficient_batch(ms, max_b, queued, tol, margin, ends, n_ends);
}
int die_engine_text_packing(void* p) { return static_cast<Engine*>(p)->text_packing() ? 1 : 0; }

// Device-decode path: B texts (concatenated, lens[b] bytes each) -> outputs [B][out] and status[b]
// (0 ok, bit 0 = needs host parse, 2 = too many values; outputs of such samples are undefined).
int die_engine_run_text(void* p, const char* texts, const long long* lens, long B, float* out, int* status, int pack,
                        char** err) {
  auto* e = static_cast<Engine*>(p);
  try {
    if (e->text_capacity() == 0) throw std::runtime_error("engine has no device decode");
    SamplePool& pool = e->sample_pool();
    std::vector<SampleBuffer> bufs;
    std::vector<BatchItem> items;
    size_t off = 0;
    for (long b = 0; b < B; ++b) {
      if (static_cast<size_t>(lens[b]) > e->text_capacity()) throw std::runtime_error("text too long");
      SampleBuffer sb = pool.acquire();
      BatchItem it;
      const size_t n = static_cast<size_t>(lens[b]);
      // pack = 1: 4-bit packed upload when the engine takes it and the text fits the alphabet
      it.packed = pack && e->text_packing() && pack_nibbles(texts + off, n, reinterpret_cast<uint8_t*>(sb.data));
      if (!it.packed) std::memcpy(sb.data, texts + off, n);
      off += n;
      bufs.push_back(sb);
      it.text = reinterpret_cast<const char*>(sb.data);
      it.text_len = n;
      items.push_back(it);
    }
    std::promise<std::string> done;
    auto fut = done.get_future();
    const size_t on = e->output_numel();
    e->submit(std::move(items), [&](BatchResult& r) {
      if (!r.ok) {
        done.set_value(r.error.empty() ? "batch failed" : r.error);
        return;
      }
      std::memcpy(out, r.outputs, sizeof(float) * on * static_cast<size_t>(B));
      for (long b = 0; b < B; ++b) status[b] = r.status ? r.status[b] : 0;
      done.set_value("");
    });
    const std::string msg = fut.get();
    for (auto& sb : bufs) pool.release(sb);
    if (!msg.empty()) throw std::runtime_error(msg);
    return 0;
  } catch (const std::exception& ex) {
    set_err(err, ex.what());
    return -1;
  }
}

// ---- CPU executor oracle: full input tensor, returns output (malloc'ed) ----
float* die_cpu_run(const char* model_path, const float* in, const int64_t* shape, int rank, int64_t* out_shape,
                   int* out_rank, char** err) {
  try {
    CpuExecutor ex(onnx::load_onnx(model_path));
    auto x = std::make_shared<CpuValue>();
    x->shape.assign(shape, shape + rank);
    x->f.assign(in, in + x->numel());
    auto y = ex.run(x);
    *out_rank = static_cast<int>(y->shape.size());
    for (size_t k = 0; k < y->shape.size(); ++k) out_shape[k] = y->shape[k];
    float* o = static_cast<float*>(std::malloc(sizeof(float) * y->f.size()));
    std::memcpy(o, y->f.data(), sizeof(float) * y->f.size());
    return o;
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

// Debug probe: run the CPU executor and return intermediate value `name` (f32; ints converted).
float* die_cpu_run_value(const char* model_path, const float* in, const int64_t* shape, int rank, const char* name,
                         int64_t* out_shape, int* out_rank, char** err) {
  try {
    CpuExecutor ex(onnx::load_onnx(model_path));
    auto x = std::make_shared<CpuValue>();
    x->shape.assign(shape, shape + rank);
    x->f.assign(in, in + x->numel());
    std::unordered_map<std::string, CpuValuePtr> trace;
    ex.run(x, &trace);
    auto it = trace.find(name);
    if (it == trace.end()) throw std::runtime_error(std::string("no value named ") + name);
    const CpuValue& v = *it->second;
    *out_rank = static_cast<int>(v.shape.size());
    for (size_t k = 0; k < v.shape.size(); ++k) out_shape[k] = v.shape[k];
    const size_t n = static_cast<size_t>(v.numel());
    float* o = static_cast<float*>(std::malloc(sizeof(float) * std::max<size_t>(n, 1)));
    for (size_t k = 0; k < n; ++k) o[k] = v.is_int ? static_cast<float>(v.i[k]) : v.f[k];
    return o;
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

char* die_onnx_summary(const char* model_path, char** err) {
  try {
    auto m = onnx::load_onnx(model_path);
    Json j = Json::object();
    j["ir_version"] = static_cast<long long>(m.ir_version);
    j["opset"] = static_cast<long long>(m.opset());
    j["nodes"] = static_cast<long long>(m.nodes.size());
    j["initializers"] = static_cast<long long>(m.initializers.size());
    j["param_bytes"] = static_cast<long long>(m.param_bytes_f32());
    Json ops = Json::object();
    for (auto& n : m.nodes) ops[n.op_type] = ops[n.op_type].is_null() ? Json(1) : Json(ops[n.op_type].as_int() + 1);
    j["ops"] = ops;
    Json ins = Json::array();
    for (auto& vi : m.inputs) {
      Json v = Json::object();
      v["name"] = vi.name;
      Json d = Json::array();
      for (auto x : vi.dims) d.push_back(static_cast<long long>(x));
      v["dims"] = d;
      ins.push_back(v);
    }
    j["inputs"] = ins;
    Json outs = Json::array();
    for (auto& vi : m.outputs) {
      Json v = Json::object();
      v["name"] = vi.name;
      Json d = Json::array();
      for (auto x : vi.dims) d.push_back(static_cast<long long>(x));
      v["dims"] = d;
      outs.push_back(v);
    }
    j["outputs"] = outs;
    return dup(j.dump());
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

// ---- worker / gateway / loadgen ----
void* die_worker_create(const char* opts_json, char** err) {
  try {
    Json j = Json::parse(opts_json);
    WorkerOptions o;
    o.node_id = jget<std::string>(j, "node_id", o.node_id);
    o.host = jget<std::string>(j, "host", "127.0.0.1");
    o.port = jget<int>(j, "port", 0);
    o.model_path = jget<std::string>(j, "model_path", "");
    o.cache_capacity = static_cast<size_t>(jget<long>(j, "cache_capacity", 1000));
    o.max_batch = jget<int>(j, "max_batch", 32);
    o.batch_timeout = std::chrono::milliseconds(jget<long>(j, "batch_timeout_ms", 20));
    o.policy = jget<std::string>(j, "policy", "greedy") == "deadline" ? BatchPolicy::DEADLINE : BatchPolicy::GREEDY;
    o.http_threads = jget<int>(j, "http_threads", 0);
    o.parse_threads = jget<int>(j, "parse_threads", -1);
    o.parse_spin_us = jget<int>(j, "parse_spin_us", 0);
    o.batch_balance = jget<bool>(j, "batch_balance", true);
    o.engine = engine_opts(j.contains("engine") ? j.at("engine") : Json::object());
    o.fault_fail_rate = jget<double>(j, "fault_fail_rate", 0.0);
    o.fault_latency_ms = jget<int>(j, "fault_latency_ms", 0);
    o.accept_shm = jget<bool>(j, "accept_shm", true);
    o.reuse_port = jget<bool>(j, "reuse_port", false);
    auto* w = new WorkerNode(o);
    if (w->start() < 0) {
      delete w;
      set_err(err, "cannot bind worker port");
      return nullptr;
    }
    return w;
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}
int die_worker_port(void* w) { return static_cast<WorkerNode*>(w)->port(); }

// ---- data-parallel follower (rank >= 1): serves shards on a background thread ----
struct DpFollowerHandle {
  std::thread th;
  std::atomic<bool> stop{false};
  std::atomic<bool> running{true};
  std::atomic<long> served{0};
  std::mutex mu;
  std::string error;
};
void* die_dp_follower_start(const char* opts_json, char** err) {
  try {
    Json j = Json::parse(opts_json);
    const std::string model = jget<std::string>(j, "model_path", "");
    EngineOptions eo = engine_opts(j.contains("engine") ? j.at("engine") : Json::object());
    eo.max_batch = jget<int>(j, "max_batch", eo.max_batch);
    auto* h = new DpFollowerHandle();
    h->th = std::thread([h, model, eo] {
      try {
        h->served = run_dp_follower(model, eo, &h->stop);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(h->mu);
        h->error = e.what();
      }
      h->running = false;
    });
    return h;
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}
char* die_dp_follower_status(void* p) {
  auto* h = static_cast<DpFollowerHandle*>(p);
  Json j = Json::object();
  j["running"] = h->running.load();
  j["served"] = static_cast<long long>(h->served.load());
  std::lock_guard<std::mutex> g(h->mu);
  j["error"] = h->error;
  return dup(j.dump());
}
// Stop (if still running) and join; returns batches served.
long die_dp_follower_join(void* p, int stop) {
  auto* h = static_cast<DpFollowerHandle*>(p);
  if (stop) h->stop = true;
  if (h->th.joinable()) h->th.join();
  const long n = h->served.load();
  delete h;
  return n;
}
char* die_worker_health(void* w) { return dup(static_cast<WorkerNode*>(w)->getHealth().dump()); }
void die_worker_stop(void* w) { static_cast<WorkerNode*>(w)->stop(); }
void die_worker_destroy(void* w) { delete static_cast<WorkerNode*>(w); }

void* die_gateway_create(const char* opts_json, char** err) {
  try {
    Json j = Json::parse(opts_json);
    GatewayOptions o;
    for (auto& w : j.at("workers").as_array()) o.workers.push_back(w.as_string());
    o.host = jget<std::string>(j, "host", "127.0.0.1");
    o.port = jget<int>(j, "port", 0);
    o.failure_threshold = jget<int>(j, "failure_threshold", 5);
    o.success_threshold = jget<int>(j, "success_threshold", 2);
    o.breaker_timeout = std::chrono::milliseconds(static_cast<long>(jget<double>(j, "breaker_timeout_s", 30.0) * 1000));
    o.vnodes = jget<int>(j, "vnodes", 150);
    o.connect_timeout = std::chrono::milliseconds(jget<long>(j, "connect_timeout_ms", 5000));
    o.read_timeout = std::chrono::milliseconds(jget<long>(j, "read_timeout_ms", 5000));
    o.client_threads = jget<int>(j, "client_threads", 0);
    o.http_threads = jget<int>(j, "http_threads", 0);
    o.local_shm = jget<bool>(j, "local_shm", true);
    o.shm_mb = static_cast<size_t>(jget<long>(j, "shm_mb", 512));
    auto* g = new Gateway(o);
    if (g->start() < 0) {
      delete g;
      set_err(err, "cannot bind gateway port");
      return nullptr;
    }
    return g;
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}
int die_gateway_port(void* g) { return static_cast<Gateway*>(g)->port(); }
char* die_gateway_stats(void* g) { return dup(static_cast<Gateway*>(g)->getStats().dump()); }
void die_gateway_stop(void* g) { static_cast<Gateway*>(g)->stop(); }
void die_gateway_destroy(void* g) { delete static_cast<Gateway*>(g); }

static LoadgenOptions loadgen_opts(const Json& j) {
  LoadgenOptions o;
  o.host = jget<std::string>(j, "host", o.host);
  o.port = jget<int>(j, "port", o.port);
  o.path = jget<std::string>(j, "path", o.path);
  o.connections = jget<int>(j, "connections", o.connections);
  o.requests = jget<long>(j, "requests", o.requests);
  o.warmup = jget<long>(j, "warmup", o.warmup);
  o.payload = jget<std::string>(j, "payload", o.payload);
  o.input_numel = static_cast<size_t>(jget<long>(j, "input_numel", static_cast<long>(o.input_numel)));
  o.decimals = jget<int>(j, "decimals", o.decimals);
  o.distinct = jget<long>(j, "distinct", o.distinct);
  o.timeout_ms = jget<int>(j, "timeout_ms", o.timeout_ms);
  o.seed = static_cast<uint64_t>(jget<long>(j, "seed", static_cast<long>(o.seed)));
  o.id_prefix = jget<std::string>(j, "id_prefix", o.id_prefix);
  o.verify_tol = jget<double>(j, "verify_tol", o.verify_tol);
  o.verify_every = jget<long>(j, "verify_every", o.verify_every);
  o.scramble_ids = jget<bool>(j, "scramble_ids", o.scramble_ids);
  o.io_threads = jget<int>(j, "io_threads", o.io_threads);
  return o;
}

// ---- data-parallel row bookkeeping (parallel/dp_layout.h), for the CPU unit tests ----
// per <= 0: ceil(B / world).  Returns rank r's shard size and its first item in *begin.
int die_dp_shard(int B, int world, int per, int r, int* begin) {
  const DpLayout L = per > 0 ? DpLayout::with_per(B, world, per) : DpLayout::make(B, world);
  *begin = L.shard_begin(r);
  return L.shard_count(r);
}
int die_dp_per(int B, int world) { return DpLayout::make(B, world).per; }
// Shared input arena of a DP group for `world` ranks (engine_json = EngineOptions, max_batch = the
// whole DP batch): writes item bytes, items and total bytes.
int die_dp_arena_plan(long long input_numel, const char* engine_json, int world, long long* out3) {
  try {
    const DpArenaPlan a = dp_arena_plan(static_cast<size_t>(input_numel), engine_opts(Json::parse(engine_json)), world);
    out3[0] = static_cast<long long>(a.item_bytes);
    out3[1] = static_cast<long long>(a.items);
    out3[2] = static_cast<long long>(a.bytes);
    return 0;
  } catch (...) {
    return -1;
  }
}
void die_dp_items_from_gathered(int B, int world, int per, const int* gathered, long stride, int* out) {
  dp_items_from_gathered(DpLayout::with_per(B, world, per), gathered, static_cast<size_t>(stride), out);
}
void die_dp_rows_from_gathered(int B, int world, int per, const float* gathered, long rows_per_rank, long row_len,
                               float* out) {
  dp_rows_from_gathered(DpLayout::with_per(B, world, per), gathered, static_cast<size_t>(rows_per_rank),
                        static_cast<size_t>(row_len), out);
}
void die_dp_item_ok(int B, int world, int per, const int* rank_ok, unsigned char* out) {
  const auto ok = dp_item_ok(DpLayout::with_per(B, world, per), rank_ok);
  std::copy(ok.begin(), ok.end(), out);
}

char* die_loadgen_run(const char* opts_json, char** err) {
  try {
    return dup(run_loadgen(loadgen_opts(Json::parse(opts_json))).dump());
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

// Verify mode: k distinct inputs (k x input_numel floats) cycled over the requests, every answer
// compared with `expected` (k x out_numel floats).
char* die_loadgen_run_verify(const char* opts_json, const float* inputs, long k, const float* expected, long out_numel,
                             char** err) {
  try {
    LoadgenOptions o = loadgen_opts(Json::parse(opts_json));
    if (o.verify_every <= 0) o.payload = "verify";  // else: "full" with every verify_every-th request verified
    o.verify_inputs = inputs;
    o.verify_expected = expected;
    o.verify_count = static_cast<size_t>(k);
    o.output_numel = static_cast<size_t>(out_numel);
    return dup(run_loadgen(o).dump());
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

// Either form above (inputs == nullptr: no verification), with `on_ready` called on this thread
// right before the timed phase starts (LoadgenOptions::on_ready).
char* die_loadgen_run_cb(const char* opts_json, const float* inputs, long k, const float* expected, long out_numel,
                         void (*on_ready)(void*), char** err) {
  try {
    LoadgenOptions o = loadgen_opts(Json::parse(opts_json));
    if (inputs) {
      if (o.verify_every <= 0) o.payload = "verify";
      o.verify_inputs = inputs;
      o.verify_expected = expected;
      o.verify_count = static_cast<size_t>(k);
      o.output_numel = static_cast<size_t>(out_numel);
    }
    o.on_ready = on_ready;
    return dup(run_loadgen(o).dump());
  } catch (const std::exception& e) {
    set_err(err, e.what());
    return nullptr;
  }
}

}  // extern "C"

extern "C" {
// Parse `iters` times a ResNet-shaped body; returns average microseconds per parse.
double die_parse_bench(const char* body, long n, int iters, int simd) {
  struct S : InferBodySink {
    std::vector<float> buf = std::vector<float>(1 << 20);
    void on_request_id(std::string_view) override {}
    float* input_buffer() override { return buf.data(); }
    size_t input_capacity() const override { return buf.size(); }
    void on_input_count(size_t) override {}
  } s;
  std::string b(body, static_cast<size_t>(n));
  b.reserve(b.size() + 64);
  set_json_simd(simd != 0);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) parse_infer_body(b, s);
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
  set_json_simd(true);
  return us;
}
}
