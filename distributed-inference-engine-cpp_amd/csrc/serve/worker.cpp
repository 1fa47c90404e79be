#include <pthread.h>
#include "worker.h"

#include "../core/http_util.h"
#include "../core/log.h"
#include "../core/metrics.h"
#include "../core/textpack.h"
#include "../core/sysinfo.h"
#include "../core/trace.h"

#include <algorithm>
#include <cstring>
#include <iostream>
#include <random>
#include <thread>

namespace die {

namespace {

struct SampleSink : InferBodySink {
  SampleBuffer buf;
  size_t float_cap = 0;
  std::string id;
  size_t n = 0;
  bool defer = false;
  const char* text = nullptr;
  size_t text_n = 0;
  void on_request_id(std::string_view s) override { id.assign(s); }
  float* input_buffer() override { return buf.data; }
  size_t input_capacity() const override { return float_cap; }
  void on_input_count(size_t k) override { n = k; }
  bool defer_input_text() const override { return defer; }
  void on_input_text(const char* b, size_t k) override {
    text = b;
    text_n = k;
  }
};

thread_local std::mt19937_64 tl_rng{std::random_device{}()};

std::string build_response(const std::string& id, const float* out, size_t n, const std::string& node, bool cached,
                           int64_t us) {
  std::string s;
  s.reserve(n * 12 + 160 + id.size());
  s += "{\"request_id\":";
  append_json_string(s, id);
  s += ",\"output_data\":";
  append_float_array(s, out, n);
  s += ",\"node_id\":";
  append_json_string(s, node);
  s += cached ? ",\"cached\":true" : ",\"cached\":false";
  s += ",\"inference_time_us\":";
  s += std::to_string(us);
  s += '}';
  return s;
}

}  // namespace

WorkerNode::WorkerNode(WorkerOptions opt, std::unique_ptr<Engine> engine)
    : opt_(std::move(opt)), engine_(std::move(engine)), cache_(opt_.cache_capacity) {
  if (!engine_) {
    EngineOptions eo = opt_.engine;
    eo.max_batch = opt_.max_batch;
    engine_ = create_engine(opt_.model_path, eo);
  }
  fault_fail_rate_ = opt_.fault_fail_rate;
  fault_latency_ms_ = opt_.fault_latency_ms;
  Engine* eng = engine_.get();
  auto batch_fn = [eng](std::vector<Pending>&& reqs,
                        std::function<void(std::vector<Result>&&, std::exception_ptr)> finish) {
    std::vector<BatchItem> items;
    items.reserve(reqs.size());
    for (auto& r : reqs) {
      BatchItem it{r.buf.data, r.len};
      if (r.text_len) {
        it.input = nullptr;
        it.len = 0;
        it.text = reinterpret_cast<const char*>(r.buf.data);
        it.text_len = r.text_len;
        it.packed = r.packed;
        it.staged = r.staged;
      }
      items.push_back(it);
    }
    const size_t B = reqs.size();
    TraceRange tr_dispatch("worker.batch_dispatch");
    const auto t_dispatch = std::chrono::steady_clock::now();
    eng->submit(std::move(items), [B, finish, t_dispatch](BatchResult& br) {
      const auto t_done = std::chrono::steady_clock::now();
      if (!br.ok) {
        finish({}, std::make_exception_ptr(std::runtime_error(br.error)));
        return;
      }
      std::vector<Result> out(B);
      const int64_t per = B ? static_cast<int64_t>(br.wall_us) / static_cast<int64_t>(B) : 0;
      for (size_t i = 0; i < B; ++i) {
        out[i].inference_time_us = per;
        out[i].t_dispatch = t_dispatch;
        out[i].t_done = t_done;
        if (br.status && br.status[i]) {
          out[i].decode_status = br.status[i];
          out[i].ntok = br.ntok[i];
          continue;
        }
        out[i].output.assign(br.outputs + i * br.output_numel, br.outputs + (i + 1) * br.output_numel);
      }
      finish(std::move(out), nullptr);
    });
  };
  batcher_ = std::make_unique<BatchProcessor<Pending, Result>>(
      static_cast<size_t>(std::max(1, std::min(opt_.max_batch, engine_->max_batch()))), opt_.batch_timeout, batch_fn,
      [eng] { eng->wait_for_slot(); }, opt_.policy, [eng] { return eng->dispatch_not_before(); });
  batcher_->set_balance(opt_.batch_balance);
  if (opt_.policy == BatchPolicy::GREEDY)
    batcher_->set_size_fn([eng](size_t q) { return static_cast<size_t>(eng->preferred_batch(static_cast<int>(q))); });
  batcher_->start();

  int npt = opt_.parse_threads;
  if (npt < 0) npt = std::max(2, available_cpus() / 4);
  for (int i = 0; i < npt; ++i) parse_threads_.emplace_back([this] {
      pthread_setname_np(pthread_self(), "die-parse");
      parse_loop();
    });
  if (npt > 0) {
    server_.route("POST", "/infer", [this](HttpRequest& req, Responder res) {
      ParseJob j{std::make_shared<HttpRequest>(std::move(req)), std::move(res)};
      {
        std::lock_guard<std::mutex> g(parse_mu_);
        parse_q_.push_back(std::move(j));
        parse_pending_.fetch_add(1, std::memory_order_release);
      }
      parse_cv_.notify_one();
    });
  } else {
    server_.route("POST", "/infer", [this](HttpRequest& req, Responder res) { handle_infer(req, res); });
  }
  server_.route("GET", "/health", [this](HttpRequest&, Responder res) {
    HttpResponse r;
    r.body = getHealth().dump();
    res.send(std::move(r));
  });
  server_.route("GET", "/metrics", [this](HttpRequest&, Responder res) {
    HttpResponse r;
    r.content_type = "text/plain; version=0.0.4";
    r.body = prometheus_text(getHealth(), "die_worker", "node=\"" + opt_.node_id + "\"");
    res.send(std::move(r));
  });
  server_.route("POST", "/admin/fault", [this](HttpRequest& req, Responder res) { handle_admin_fault(req, res); });
  started_ = std::chrono::steady_clock::now();
}

WorkerNode::~WorkerNode() { stop(); }

int WorkerNode::start() { return server_.start(opt_.host, opt_.port, opt_.http_threads, opt_.reuse_port); }
void WorkerNode::wait() { server_.wait(); }

void WorkerNode::stop() {
  server_.stop();
  {
    std::lock_guard<std::mutex> g(parse_mu_);
    parse_stop_ = true;
  }
  parse_cv_.notify_all();
  for (auto& t : parse_threads_)
    if (t.joinable()) t.join();
  parse_threads_.clear();
  if (batcher_) batcher_->stop();
  if (engine_) engine_->synchronize();
}

void WorkerNode::parse_loop() {
  while (true) {
    ParseJob j;
    if (opt_.parse_spin_us > 0) {  // WorkerOptions::parse_spin_us: poll before sleeping
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(opt_.parse_spin_us);
      while (parse_pending_.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#else
        std::this_thread::yield();
#endif
    }
    {
      std::unique_lock<std::mutex> lk(parse_mu_);
      parse_cv_.wait(lk, [&] { return parse_stop_ || !parse_q_.empty(); });
      if (parse_q_.empty()) return;  // stopping and drained
      j = std::move(parse_q_.front());
      parse_q_.pop_front();
      parse_pending_.fetch_sub(1, std::memory_order_relaxed);
    }
    try {
      handle_infer(*j.req, j.res);
    } catch (const std::exception& e) {  // never let a request take the parse thread (and the process) down
      errors_++;
      j.res.send(error_response(500, e.what()));  // no-op when handle_infer already answered
    }
  }
}

HttpResponse WorkerNode::error_response(int status, const std::string& msg, bool client_error) const {
  HttpResponse r;
  r.status = status;
  // Same status and {"error": ...} body as the reference (500); the extra header tells the gateway
  // that the request, not this worker, is at fault (no failover, no breaker failure).
  if (client_error) r.headers.emplace_back("X-Die-Error", "client");
  Json j = Json::object();
  j["error"] = msg;
  r.body = j.dump();
  return r;
}

void WorkerNode::handle_admin_fault(HttpRequest& req, Responder res) {
  try {
    Json j = Json::parse(req.body);
    if (auto* v = j.find("fail_rate")) fault_fail_rate_ = v->as_double();
    if (auto* v = j.find("latency_ms")) fault_latency_ms_ = static_cast<int>(v->as_int());
    Json o = Json::object();
    o["fail_rate"] = fault_fail_rate_.load();
    o["latency_ms"] = fault_latency_ms_.load();
    HttpResponse r;
    r.body = o.dump();
    res.send(std::move(r));
  } catch (const std::exception& e) {
    res.send(error_response(500, e.what()));
  }
}

void WorkerNode::handle_infer(HttpRequest& req, Responder res) {
  total_requests_.fetch_add(1, std::memory_order_relaxed);
  const int lat = fault_latency_ms_.load(std::memory_order_relaxed);
  if (lat > 0) std::this_thread::sleep_for(std::chrono::milliseconds(lat));
  const double fr = fault_fail_rate_.load(std::memory_order_relaxed);
  if (fr > 0 && std::uniform_real_distribution<double>(0, 1)(tl_rng) < fr) {
    errors_++;
    res.send(error_response(500, "injected fault"));
    return;
  }

  Engine& eng = *engine_;
  SamplePool& pool = eng.sample_pool();
  SampleSink sink;
  try {
    sink.buf = pool.acquire();
  } catch (const std::exception&) {
    // staging exhausted (e.g. a data-parallel rank's share of the shared arena under a burst): a
    // retryable 503, not a dead parse thread
    errors_++;
    staging_exhausted_.fetch_add(1, std::memory_order_relaxed);
    res.send(error_response(503, "server busy: input staging exhausted"));
    return;
  }
  const size_t numel = eng.input_numel();
  sink.float_cap = std::min(sink.buf.capacity, numel);
  // device decode takes texts of up to text_capacity() characters; the staging item holds them
  // 4-bit packed (half the bytes) when the engine packs, raw otherwise
  const size_t item_bytes = sink.buf.capacity * sizeof(float);
  const size_t dev_cap = eng.text_capacity();
  const bool packing = eng.text_packing();
  const size_t text_cap = std::min(dev_cap, packing ? 2 * item_bytes : item_bytes);
  sink.defer = text_cap > 0;
  int seen = 0;
  TraceRange tr_parse("worker.parse");
  const auto t_parse = std::chrono::steady_clock::now();
  const auto t_start = t_parse;
  if (req.t_headers.time_since_epoch().count()) h_recv_.add(t_start - req.t_headers);
  InputKey key;
  size_t text_len = 0, text_off = 0;
  bool packed = false;
  std::string_view body = req.body_view();
  std::shared_ptr<const void> shm_keep;  // keeps the gateway arena's view mapped while we parse
  if (const std::string_view desc = req.header("x-die-shm"); !desc.empty()) {
    // co-located gateway: the body lies in its shared-memory arena (core/shm_arena.h).  Only a
    // loopback peer may send a descriptor, and the segment name carries the arena's random token.
    const char* p = nullptr;
    size_t n = 0;
    std::string err = "shared-memory bodies disabled";
    if (opt_.accept_shm && !req.peer_loopback) err = "shared-memory bodies are accepted from loopback peers only";
    if (!opt_.accept_shm || !req.peer_loopback || !shm_reader_.resolve(desc, &p, &n, &err, &shm_keep)) {
      pool.release(sink.buf);
      errors_++;
      HttpResponse r = error_response(500, err);
      r.headers.emplace_back("X-Die-Error", "shm");
      res.send(std::move(r));
      return;
    }
    body = std::string_view(p, n);
    shm_bodies_.fetch_add(1, std::memory_order_relaxed);
  }
  try {
    seen = parse_infer_body(body, sink);
    // too long for device decode, or not packable and too long to stage raw: parse on the host
    bool host = (seen & 4) && sink.text_n > text_cap;
    if ((seen & 4) && !host) {
      auto* dst = reinterpret_cast<uint8_t*>(sink.buf.data);
      if (packing && pack_nibbles(sink.text, sink.text_n, dst)) packed = true;  // half the bytes to copy
      else if (sink.text_n > item_bytes) host = true;
      else std::memcpy(dst, sink.text, sink.text_n);
    }
    if (host) {
      sink.defer = false;
      sink.text = nullptr;
      packed = false;
      seen = parse_infer_body(body, sink);
    }
    if (!(seen & 1)) throw JsonError("key 'request_id' not found");
    if (!(seen & 2)) throw JsonError("key 'input_data' not found");
    if (seen & 4) {
      text_len = sink.text_n;
      text_off = static_cast<size_t>(sink.text - body.data());
      const auto* dst = reinterpret_cast<const uint8_t*>(sink.buf.data);
      key = packed ? hash_bytes(dst, (text_len + 1) / 2, 2) : hash_text(sink.text, sink.text_n);
      // an empty list needs no conversion
      if (text_len == 0) {
        text_len = 0;
        sink.n = 0;
        key = hash_floats(sink.buf.data, 0);
      }
    } else {
      if (sink.n > numel)
        throw std::runtime_error("input_data has " + std::to_string(sink.n) + " values; model input holds " +
                                 std::to_string(numel));
      key = hash_floats(sink.buf.data, sink.n);
    }
    parse_ns_.fetch_add(static_cast<int64_t>(
                            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_parse)
                                .count()),
                        std::memory_order_relaxed);
    parse_bytes_.fetch_add(static_cast<int64_t>(body.size()), std::memory_order_relaxed);
    parsed_.fetch_add(1, std::memory_order_relaxed);
  } catch (const std::exception& e) {
    pool.release(sink.buf);
    errors_++;
    res.send(error_response(500, e.what(), true));
    return;
  }
  // Free the request body now: at ResNet size it is ~1 MB we no longer need.
  std::string().swap(req.body);

  if (auto hit = cache_.get(key)) {
    cache_hits_.fetch_add(1, std::memory_order_relaxed);
    pool.release(sink.buf);
    auto out = std::make_shared<std::vector<float>>(std::move(*hit));
    std::string id = std::move(sink.id);
    std::string node = opt_.node_id;
    res.defer([out, id = std::move(id), node = std::move(node)] {
      HttpResponse r;
      r.body = build_response(id, out->data(), out->size(), node, true, 50);
      return r;
    });
    return;
  }
  long staged = -1;
  if (text_len) {
    device_decoded_.fetch_add(1, std::memory_order_relaxed);
    // start the H2D of this request's text now: by the time its batch is dispatched the bytes are
    // on the device and the batch waits only for the GPU
    staged = eng.stage_text(reinterpret_cast<const char*>(sink.buf.data), text_len, packed);
  }
  const auto t_queued = std::chrono::steady_clock::now();
  h_parse_.add(t_queued - t_start);

  Pending p;
  p.t_start = t_start;
  p.t_queued = t_queued;
  p.request_id = std::move(sink.id);
  p.buf = sink.buf;
  p.len = sink.n;
  p.text_len = text_len;
  p.text_off = text_off;
  p.packed = packed;
  p.staged = staged;
  p.key = key;
  dispatch(std::move(p), std::move(res));
}

void WorkerNode::dispatch(Pending p, Responder res) {
  const SampleBuffer buf = p.buf;
  const size_t text_len = p.text_len, text_off = p.text_off;
  const bool packed = p.packed;
  const long staged = p.staged;
  const InputKey key = p.key;
  const auto t_start = p.t_start, t_queued = p.t_queued;
  std::string id_copy = p.request_id;
  batcher_->submit(std::move(p), [this, res, key, buf, text_len, packed, text_off, staged, t_start, t_queued,
                                  id = std::move(id_copy)](Result* r, std::exception_ptr err) mutable {
    // the batch is done (or the request never ran): its staged device copy is free again
    engine_->release_staged(staged, !err);
    if (err) {
      engine_->sample_pool().release(buf);
      errors_++;
      std::string msg = "inference failed";
      try {
        std::rethrow_exception(err);
      } catch (const std::exception& e) {
        msg = e.what();
      } catch (...) {
      }
      res.send(error_response(500, msg));
      return;
    }
    if (r->decode_status & kItemShardFailed) {
      engine_->sample_pool().release(buf);
      errors_++;
      res.send(error_response(500, "inference failed on a data-parallel rank"));
      return;
    }
    if (r->decode_status & kItemNeedsHostParse) {
      host_fallback(buf, text_len, packed, text_off, std::move(id), key, std::move(res));
      return;
    }
    engine_->sample_pool().release(buf);
    if (r->decode_status) {
      errors_++;
      res.send(error_response(500, "input_data has " + std::to_string(r->ntok) + " values; model input holds " +
                                       std::to_string(engine_->input_numel()), true));
      return;
    }
    h_queue_.add(r->t_dispatch - t_queued);
    h_engine_.add(r->t_done - r->t_dispatch);
    auto out = std::make_shared<std::vector<float>>(std::move(r->output));
    const int64_t us = r->inference_time_us;
    std::string node = opt_.node_id;
    const auto t_done = r->t_done;
    // This callback runs once per request, in a row, on the batch's completion thread: keep it to a
    // hand-off.  The JSON and the cache insert happen on the connection's reactor, in parallel
    // over the reactors, after the response is built.
    res.defer([this, out, key, id = std::move(id), node = std::move(node), us, t_start, t_done] {
      TraceRange tr_resp("worker.respond");
      HttpResponse resp;
      resp.body = build_response(id, out->data(), out->size(), node, false, us);
      const auto now = std::chrono::steady_clock::now();
      h_respond_.add(now - t_done);
      h_total_.add(now - t_start);
      cache_.put(key, *out);
      return resp;
    });
  });
}

void WorkerNode::host_fallback(SampleBuffer text_buf, size_t text_len, bool packed, size_t text_off, std::string id, InputKey key,
                               Responder res) {
  decode_fallbacks_.fetch_add(1, std::memory_order_relaxed);
  SamplePool& pool = engine_->sample_pool();
  const size_t numel = engine_->input_numel();
  std::string body;
  // Same byte offsets as the original body, so parse errors report the same position:
  // '{' + blanks + "input_data": '[' with the '[' at text_off - 1.
  static const char kKey[] = "\"input_data\":";
  const size_t pad = text_off >= sizeof(kKey) + 1 ? text_off - sizeof(kKey) - 1 : 0;
  body.reserve(text_len + pad + 32);
  body += '{';
  body.append(pad, ' ');
  body += kKey;
  body += '[';
  if (packed) {
    const size_t at = body.size();
    body.resize(at + text_len);
    unpack_nibbles(reinterpret_cast<const uint8_t*>(text_buf.data), text_len, &body[at]);
  } else {
    body.append(reinterpret_cast<const char*>(text_buf.data), text_len);
  }
  body += "]}";
  pool.release(text_buf);
  SampleSink sink;
  try {
    sink.buf = pool.acquire();
  } catch (const std::exception&) {
    errors_++;
    staging_exhausted_.fetch_add(1, std::memory_order_relaxed);
    res.send(error_response(503, "server busy: input staging exhausted"));
    return;
  }
  sink.float_cap = std::min(sink.buf.capacity, numel);
  try {
    parse_infer_body(body, sink);
    if (sink.n > numel)
      throw std::runtime_error("input_data has " + std::to_string(sink.n) + " values; model input holds " +
                               std::to_string(numel));
  } catch (const std::exception& e) {
    pool.release(sink.buf);
    errors_++;
    res.send(error_response(500, e.what(), true));
    return;
  }
  Pending p;
  p.request_id = std::move(id);
  p.buf = sink.buf;
  p.len = sink.n;
  p.key = key;
  p.t_start = p.t_queued = std::chrono::steady_clock::now();
  dispatch(std::move(p), std::move(res));
}

Json WorkerNode::getHealth() const {
  auto m = batcher_->getMetrics();
  Json h = Json::object();
  h["healthy"] = true;
  h["node_id"] = opt_.node_id;
  h["total_requests"] = static_cast<long long>(total_requests_.load());
  h["cache_hits"] = static_cast<long long>(cache_hits_.load());
  h["cache_size"] = static_cast<long long>(cache_.size());
  h["cache_hit_rate"] = cache_.getHitRate();
  Json b = Json::object();
  b["total_batches"] = static_cast<long long>(m.total_batches);
  b["avg_batch_size"] = m.avg_batch_size;
  b["timeout_batches"] = static_cast<long long>(m.timeout_batches);
  b["full_batches"] = static_cast<long long>(m.full_batches);
  b["total_requests"] = static_cast<long long>(m.total_requests);
  b["queue_depth"] = static_cast<long long>(batcher_->queue_depth());
  b["trimmed_batches"] = batcher_->trimmed_batches();    // batches cut below the queue (balance / preferred_batch)
  b["trimmed_requests"] = batcher_->trimmed_requests();  // requests those cuts left for the next batch
  {
    Json hist = Json::array();  // batches per size: [count at size 1, count at size 2, ...]
    const auto sh = batcher_->size_histogram();
    for (size_t i = 1; i < sh.size(); ++i) hist.push_back(sh[i]);
    b["size_histogram"] = hist;
  }
  h["batch_processor"] = b;
  // extras (superset of the reference keys)
  h["errors"] = static_cast<long long>(errors_.load());
  const int64_t np = parsed_.load();
  h["parse_us_avg"] = np ? parse_ns_.load() / 1e3 / np : 0.0;
  h["parse_gbps"] = parse_ns_.load() ? static_cast<double>(parse_bytes_.load()) / parse_ns_.load() : 0.0;
  h["device_decoded"] = static_cast<long long>(device_decoded_.load());
  h["shm_bodies"] = static_cast<long long>(shm_bodies_.load());
  h["shm_segments_mapped"] = static_cast<long long>(shm_reader_.mapped());
  h["shm_segments_unmapped"] = shm_reader_.unmapped();
  h["staging_exhausted"] = static_cast<long long>(staging_exhausted_.load());
  h["decode_fallbacks"] = static_cast<long long>(decode_fallbacks_.load());
  Json st = Json::object();
  st["recv"] = h_recv_.snapshot();
  st["parse"] = h_parse_.snapshot();
  st["queue"] = h_queue_.snapshot();
  st["engine"] = h_engine_.snapshot();
  st["respond"] = h_respond_.snapshot();
  st["total"] = h_total_.snapshot();
  h["stages_us"] = st;
  h["http_threads"] = opt_.http_threads;
  h["parse_threads"] = static_cast<int>(parse_threads_.size());
  h["engine"] = engine_->stats();
  h["engine"]["name"] = engine_->name();
  // per-GPU I/O counters, one schema for every engine (zeros where not applicable)
  Json io = Json::object();
  const Json& es = h["engine"];
  for (const char* k : {"h2d_bytes", "d2h_bytes", "graph_replays", "batches", "images"}) {
    const Json* v = es.find(k);
    io[k] = v ? v->as_int() : 0LL;
  }
  const Json* busy = es.find("device_busy_ms");
  io["device_busy_ms"] = busy ? busy->as_double() : 0.0;
  const Json* dev = es.find("device_id");
  io["device_id"] = dev ? dev->as_int() : -1LL;
  io["loopback_sock_buf_bytes"] = static_cast<long long>(http_detail::sock_buf_effective());
  h["io"] = io;
  Json lg = Json::object();
  lg["level"] = static_cast<long long>(log_level());
  lg["lines"] = static_cast<long long>(log_lines_emitted());
  lg["suppressed"] = static_cast<long long>(log_lines_suppressed());
  h["log"] = lg;
  Json ins = Json::array();
  for (auto d : engine_->getInputShape()) ins.push_back(static_cast<long long>(d));
  Json outs = Json::array();
  for (auto d : engine_->getOutputShape()) outs.push_back(static_cast<long long>(d));
  h["input_shape"] = ins;
  h["output_shape"] = outs;
  h["uptime_s"] = std::chrono::duration<double>(std::chrono::steady_clock::now() - started_).count();
  return h;
}

}  // namespace die
