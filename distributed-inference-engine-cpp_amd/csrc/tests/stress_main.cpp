// Concurrency stress for the host runtime, built under ThreadSanitizer and AddressSanitizer/UBSan
// (`make stress-tsan stress-asan`).  No GPU code is linked: HTTP server + client pool,
// gateway routing/failover/breakers, batcher, LRU cache, ring and JSON codec are hammered from many
// threads; any data race, leak, overflow or UB aborts with a sanitizer report.
//   die_stress [seconds_per_phase=2]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../core/http.h"
#include "../core/json.h"
#include "../serve/batcher.h"
#include "../serve/circuit_breaker.h"
#include "../serve/consistent_hash.h"
#include "../serve/gateway.h"
#include "../serve/lru_cache.h"

using namespace die;
using Clock = std::chrono::steady_clock;

static std::atomic<int> failures{0};
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

template <typename F>
void run_threads(int n, double seconds, F f) {
  std::vector<std::thread> th;
  std::atomic<bool> stop{false};
  for (int i = 0; i < n; ++i) th.emplace_back([&, i] {
      std::mt19937 rng(1234 + i);
      while (!stop.load(std::memory_order_relaxed)) f(i, rng);
    });
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop = true;
  for (auto& t : th) t.join();
}

static void stress_cache_ring_breaker(double secs) {
  LRUCache<InputKey, std::vector<float>, InputKeyHash> cache(64);
  ConsistentHash ring(150);
  for (int i = 0; i < 4; ++i) ring.addNode("node" + std::to_string(i));
  CircuitBreaker br(5, 2, std::chrono::milliseconds(5));
  std::atomic<long> ops{0};
  run_threads(32, secs, [&](int, std::mt19937& rng) {
    float v[4] = {static_cast<float>(rng() % 100), 1.f, 2.f, 3.f};
    const InputKey k = hash_floats(v, 4);
    if (rng() % 2) cache.put(k, std::vector<float>(v, v + 4));
    else if (auto hit = cache.get(k)) CHECK(hit->size() == 4 && (*hit)[0] == v[0]);
    const std::string node = ring.getNode("req_" + std::to_string(rng() % 1000));
    CHECK(!node.empty());
    if (br.allowRequest()) (rng() % 3 ? br.recordSuccess() : br.recordFailure());
    (void)br.getStateString();
    (void)cache.getHitRate();
    ops++;
  });
  CHECK(cache.size() <= 64);
  std::printf("cache/ring/breaker: %ld ops\n", ops.load());
}

static void stress_batcher(double secs) {
  std::atomic<long> done{0};
  BatchProcessor<int, int> bp(8, std::chrono::milliseconds(2), [](const std::vector<int>& reqs) {
    std::vector<int> out;
    for (int r : reqs) out.push_back(r * 2);
    return out;
  });
  bp.start();
  run_threads(48, secs, [&](int i, std::mt19937& rng) {
    const int x = static_cast<int>(rng() % 1000);
    if (i % 2) {
      CHECK(bp.process(x) == 2 * x);
      done++;
    } else {
      std::atomic<int> got{-1};
      std::atomic<bool> fin{false};
      bp.submit(x, [&](int* r, std::exception_ptr e) {
        got = e ? -2 : *r;
        fin = true;
      });
      while (!fin.load()) std::this_thread::yield();
      CHECK(got.load() == 2 * x);
      done++;
    }
  });
  auto m = bp.getMetrics();
  CHECK(m.total_requests >= done.load());
  bp.stop();
  std::printf("batcher: %ld requests, %lld batches\n", done.load(), static_cast<long long>(m.total_batches));
}

static void stress_json(double secs) {
  std::atomic<long> n{0};
  run_threads(8, secs, [&](int, std::mt19937& rng) {
    std::string body = "{\"request_id\":\"r" + std::to_string(rng()) + "\",\"input_data\":[";
    const int k = 1 + static_cast<int>(rng() % 300);
    for (int i = 0; i < k; ++i) {
      if (i) body += ',';
      body += std::to_string(static_cast<int>(rng() % 2000) - 1000) + "." + std::to_string(rng() % 10000);
    }
    body += "]}";
    // random corruption half of the time: must throw cleanly, never crash
    if (rng() % 2 && body.size() > 4) body[rng() % body.size()] = "x,[]{}\"-.e"[rng() % 10];
    struct Sink : InferBodySink {
      std::vector<float> buf = std::vector<float>(400);
      void on_request_id(std::string_view) override {}
      float* input_buffer() override { return buf.data(); }
      size_t input_capacity() const override { return buf.size(); }
      void on_input_count(size_t) override {}
    } s;
    body.reserve(body.size() + 64);
    try {
      parse_infer_body(body, s);
    } catch (const std::exception&) {
    }
    try {
      (void)Json::parse(body).dump();
    } catch (const std::exception&) {
    }
    n++;
  });
  std::printf("json: %ld bodies\n", n.load());
}

static void stress_http_gateway(double secs) {
  // three fake workers: echo request_id, one of them fails half of the time
  std::vector<std::unique_ptr<HttpServer>> workers;
  std::vector<std::string> names;
  for (int w = 0; w < 3; ++w) {
    auto s = std::make_unique<HttpServer>();
    s->route("POST", "/infer", [w](HttpRequest& req, Responder res) {
      std::string id;
      find_top_level_string(req.body, "request_id", id);
      HttpResponse r;
      if (w == 2 && (id.size() % 2)) {
        r.status = 500;
        r.body = "{\"error\":\"flaky\"}";
      } else {
        r.body = "{\"request_id\":\"" + id + "\",\"node_id\":\"w" + std::to_string(w) + "\"}";
      }
      if (id.size() % 3 == 0) {  // answer from another thread
        std::thread([res, r]() mutable { res.send(std::move(r)); }).detach();
      } else {
        res.send(std::move(r));
      }
    });
    const int port = s->start("127.0.0.1", 0, 2);
    CHECK(port > 0);
    names.push_back("127.0.0.1:" + std::to_string(port));
    workers.push_back(std::move(s));
  }
  GatewayOptions go;
  go.workers = names;
  go.host = "127.0.0.1";
  go.port = 0;
  go.breaker_timeout = std::chrono::milliseconds(50);
  go.client_threads = 2;
  go.http_threads = 2;
  Gateway gw(go);
  const int gport = gw.start();
  CHECK(gport > 0);
  std::atomic<long> ok{0}, bad{0};
  run_threads(24, secs, [&](int i, std::mt19937& rng) {
    thread_local std::unique_ptr<HttpClient> cl;
    if (!cl) cl = std::make_unique<HttpClient>("127.0.0.1", gport);
    const std::string id = "req_" + std::to_string(rng() % 100000);
    auto r = cl->post("/infer", "{\"request_id\":\"" + id + "\",\"input_data\":[1,2,3]}");
    if (r && r->status == 200 && r->body.find(id) != std::string::npos) ok++;
    else bad++;
    if (i == 0 && rng() % 50 == 0) (void)gw.getStats().dump();
  });
  gw.stop();
  for (auto& w : workers) w->stop();
  CHECK(bad.load() == 0);
  std::printf("http+gateway: %ld ok, %ld failed\n", ok.load(), bad.load());
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
  stress_cache_ring_breaker(secs);
  stress_batcher(secs);
  stress_json(secs);
  stress_http_gateway(secs);
  std::printf("stress done: %d check failures\n", failures.load());
  return failures ? 1 : 0;
}
