#include "gateway.h"

#include <unistd.h>

#include <iostream>

#include "../core/log.h"
#include "../core/metrics.h"
#include "../core/sysinfo.h"

namespace die {

namespace {

std::string error_body(const std::string& msg) {
  Json j = Json::object();
  j["error"] = msg;
  return j.dump();
}

HttpResponse error_response(const std::string& msg) {
  HttpResponse r;
  r.status = 500;
  r.body = error_body(msg);
  return r;
}

}  // namespace

// One request's failover walk: the primary, then the other nodes in ring order
// (src/gateway.cpp:46-59).
struct Gateway::Route {
  AsyncHttpClient::BodyRef body;
  long long shm_off = -1;
  std::function<void(HttpResponse&&)> done;
  std::string target;
  std::vector<std::string> order;
  size_t next = 0;
  std::chrono::steady_clock::time_point t_head, t_body, t_try;
};

Gateway::Gateway(GatewayOptions opt) : opt_(std::move(opt)), ring_(opt_.vnodes) {
  AsyncHttpClient::Options co;
  // Forwarding a ~1 MB body is a ~100 us kernel copy: with 2 loops the gateway capped at ~10.8k
  // req/s on a 16-CPU share (profiles/r2_gateway_threads.md), so it scales with the CPUs.
  co.threads = opt_.client_threads > 0 ? opt_.client_threads : std::max(2, available_cpus() / 2);
  co.connect_timeout = opt_.connect_timeout;
  co.read_timeout = opt_.read_timeout;
  client_ = std::make_unique<AsyncHttpClient>(co);
  for (const auto& w : opt_.workers) {
    ring_.addNode(w);
    breakers_[w] = std::make_unique<CircuitBreaker>(opt_.failure_threshold, opt_.success_threshold,
                                                    opt_.breaker_timeout);
    auto hp = parse_host_port(w);
    upstream_[w] = client_->add_upstream(hp.first, hp.second);
    node_shm_[w] = std::make_unique<NodeShm>();
    node_shm_[w]->local = hp.first == "127.0.0.1" || hp.first == "localhost";
    DIE_LOG(DEBUG, "Parsed URL: " << w << " -> host=" << hp.first << " port=" << hp.second);
  }
  bool any_local = false;
  for (auto& kv : node_shm_) any_local |= kv.second->local;
  if (opt_.local_shm && any_local) {
    static std::atomic<int> instance{0};
    std::string err;
    shm_ = ShmArena::create(shm_arena_name(std::to_string(getpid()) + "_" + std::to_string(instance++)),
                            opt_.shm_mb << 20, &err);
    if (!shm_) DIE_LOG(WARN, "gateway: no shared-memory body arena (" << err << "); forwarding bytes");
  }
  if (shm_) {
    // large bodies are received straight into the arena (the client's bytes are copied once, by the
    // kernel, into memory the co-located worker reads in place)
    std::weak_ptr<ShmArena> wa = shm_;
    server_.set_body_allocator(
        [wa](size_t n) -> BodyBuffer {
          auto a = wa.lock();
          if (!a) return {};
          const long long off = a->alloc(n);
          if (off < 0) return {};
          BodyBuffer b;
          b.data = a->base() + off;
          b.capacity = n;
          b.owner = std::shared_ptr<void>(b.data, [a, off](void*) { a->free(off); });
          return b;
        },
        64 << 10);
  }
  server_.route("POST", "/infer", [this](HttpRequest& req, Responder res) {
    const auto t_body = std::chrono::steady_clock::now();
    const auto t_head = req.t_headers.time_since_epoch().count() ? req.t_headers : t_body;
    h_recv_.add(t_body - t_head);
    AsyncHttpClient::BodyRef b;
    long long off = -1;
    if (req.ext_body) {
      b = AsyncHttpClient::BodyRef{req.ext_body, req.ext_len, req.ext_owner};
      off = req.ext_body - shm_->base();
    } else {
      auto body = std::make_shared<const std::string>(std::move(req.body));
      b = AsyncHttpClient::BodyRef{body->data(), body->size(), body};
    }
    routeRequest(std::move(b), off, [this, res, t_head, t_body](HttpResponse&& r) {
      const auto now = std::chrono::steady_clock::now();
      h_route_.add(now - t_body);
      h_total_.add(now - t_head);
      res.send(std::move(r));
    });
  });
  server_.route("GET", "/stats", [this](HttpRequest&, Responder res) {
    HttpResponse r;
    r.body = getStats().dump();
    res.send(std::move(r));
  });
  server_.route("GET", "/metrics", [this](HttpRequest&, Responder res) {
    HttpResponse r;
    r.content_type = "text/plain; version=0.0.4";
    r.body = prometheus_text(getStats(), "die_gateway", "");
    res.send(std::move(r));
  });
}

Gateway::~Gateway() { stop(); }

int Gateway::start() { return server_.start(opt_.host, opt_.port, opt_.http_threads); }
void Gateway::wait() { server_.wait(); }
void Gateway::stop() {
  server_.stop();
  if (client_) client_->stop();
}

void Gateway::routeRequest(AsyncHttpClient::BodyRef body, long long shm_off, std::function<void(HttpResponse&&)> done) {
  routed_++;
  std::string request_id;
  const std::string_view view(body.data ? body.data : "", body.size);
  if (!find_top_level_string(view, "request_id", request_id)) {
    // Slow path only to produce the same kind of error the reference returns.
    try {
      Json j = Json::parse(view);
      request_id = j.at("request_id").as_string();
    } catch (const std::exception& e) {
      failed_++;
      done(error_response(e.what()));
      return;
    }
  }
  auto r = std::make_shared<Route>();
  r->body = std::move(body);
  r->shm_off = shm_off;
  r->done = std::move(done);
  r->target = ring_.getNode(request_id);
  if (r->target.empty()) {
    failed_++;
    r->done(error_response("No workers available"));
    return;
  }
  r->order.push_back(r->target);
  for (const auto& node : ring_.getAllNodes())
    if (node != r->target) r->order.push_back(node);
  try_next(std::move(r));
}

void Gateway::try_next(std::shared_ptr<Route> r) {
  while (r->next < r->order.size()) {
    const std::string node = r->order[r->next++];
    CircuitBreaker& breaker = *breakers_.at(node);
    if (!breaker.allowRequest()) {
      DIE_LOG_EVERY_MS(DEBUG, 1000, "Circuit breaker OPEN for " << node << ", skipping");
      continue;
    }
    NodeShm& ns = *node_shm_.at(node);
    const bool via_shm = r->shm_off >= 0 && shm_ && ns.local && ns.ok.load(std::memory_order_relaxed);
    AsyncHttpClient::BodyRef send = r->body;
    std::string extra;
    if (via_shm) {  // descriptor only: the worker parses the body where it lies
      extra = "X-Die-Shm: " + shm_->name() + ":" + std::to_string(r->shm_off) + ":" + std::to_string(r->body.size) + "\r\n";
      send = AsyncHttpClient::BodyRef{nullptr, 0, r->body.owner};
      shm_forwards_++;
    } else {
      byte_forwards_++;
    }
    r->t_try = std::chrono::steady_clock::now();
    client_->post(upstream_.at(node), "/infer", std::move(send), "application/json", extra,
                  [this, r, node, via_shm](std::optional<HttpResponse> resp, const std::string& err) {
                    h_upstream_.add(std::chrono::steady_clock::now() - r->t_try);
                    CircuitBreaker& br = *breakers_.at(node);
                    if (via_shm && resp && resp->header("x-die-error") == "shm") {
                      // this worker cannot map the arena (other host / namespace): send it bytes
                      node_shm_.at(node)->ok.store(false);
                      DIE_LOG(WARN, "worker " << node << " cannot read the shared-memory arena (" << resp->body
                                              << "); forwarding bodies as bytes");
                      --r->next;
                      try_next(r);
                      return;
                    }
                    if (resp && resp->status == 200) {
                      br.recordSuccess();
                      if (node != r->target) failovers_++;
                      HttpResponse out;
                      out.body = std::move(resp->body);
                      r->done(std::move(out));
                      return;
                    }
                    if (resp && resp->header("x-die-error") == "client") {
                      // the worker is healthy; the request is bad: same answer from any node
                      br.recordSuccess();
                      client_errors_++;
                      HttpResponse out;
                      out.status = resp->status;
                      out.body = std::move(resp->body);
                      r->done(std::move(out));
                      return;
                    }
                    // the reference logs every failure (src/gateway.cpp:110-118); here at most one line
                    // per second per site, with a count of the ones it held back
                    if (resp) DIE_LOG_EVERY_MS(WARN, 1000, "Request to " << node << " failed with status: " << resp->status);
                    else DIE_LOG_EVERY_MS(WARN, 1000, "Request to " << node << " failed: " << err);
                    br.recordFailure();
                    try_next(r);
                  });
    return;
  }
  failed_++;
  r->done(error_response("All workers failed or circuit breakers open"));
}

Json Gateway::getStats() const {
  Json s = Json::object();
  s["total_workers"] = static_cast<long long>(ring_.getAllNodes().size());
  Json arr = Json::array();
  for (const auto& kv : breakers_) {  // std::map: lexicographic node order, like the reference
    Json b = Json::object();
    b["node"] = kv.first;
    b["state"] = kv.second->getStateString();
    b["failures"] = kv.second->getFailureCount();
    b["successes"] = kv.second->getSuccessCount();
    b["opened"] = kv.second->opened();
    b["half_opened"] = kv.second->half_opened();
    b["closed"] = kv.second->closed();
    arr.push_back(std::move(b));
  }
  s["circuit_breakers"] = arr;
  s["routed"] = static_cast<long long>(routed_.load());
  s["failovers"] = static_cast<long long>(failovers_.load());
  s["failed"] = static_cast<long long>(failed_.load());
  s["client_errors"] = static_cast<long long>(client_errors_.load());
  s["in_flight"] = client_->in_flight();
  s["upstream_connections_opened"] = client_->connections_opened();
  s["shm_forwards"] = static_cast<long long>(shm_forwards_.load());
  Json st = Json::object();
  st["recv"] = h_recv_.snapshot();
  st["upstream"] = h_upstream_.snapshot();
  st["route"] = h_route_.snapshot();
  st["total"] = h_total_.snapshot();
  s["stages_us"] = st;
  s["byte_forwards"] = static_cast<long long>(byte_forwards_.load());
  s["shm_arena_mib"] = shm_ ? static_cast<double>(shm_->size()) / (1 << 20) : 0.0;
  s["log_lines"] = static_cast<long long>(log_lines_emitted());
  s["log_lines_suppressed"] = static_cast<long long>(log_lines_suppressed());
  return s;
}

}  // namespace die
