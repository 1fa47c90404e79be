#include "gateway.h"

#include <iostream>

#include "../core/log.h"
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
  std::shared_ptr<const std::string> body;
  std::function<void(HttpResponse&&)> done;
  std::string target;
  std::vector<std::string> order;
  size_t next = 0;
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
    DIE_LOG(DEBUG, "Parsed URL: " << w << " -> host=" << hp.first << " port=" << hp.second);
  }
  server_.route("POST", "/infer", [this](HttpRequest& req, Responder res) {
    auto body = std::make_shared<const std::string>(std::move(req.body));
    routeRequest(std::move(body), [res](HttpResponse&& r) { res.send(std::move(r)); });
  });
  server_.route("GET", "/stats", [this](HttpRequest&, Responder res) {
    HttpResponse r;
    r.body = getStats().dump();
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

void Gateway::routeRequest(std::shared_ptr<const std::string> body, std::function<void(HttpResponse&&)> done) {
  routed_++;
  std::string request_id;
  if (!find_top_level_string(*body, "request_id", request_id)) {
    // Slow path only to produce the same kind of error the reference returns.
    try {
      Json j = Json::parse(*body);
      request_id = j.at("request_id").as_string();
    } catch (const std::exception& e) {
      failed_++;
      done(error_response(e.what()));
      return;
    }
  }
  auto r = std::make_shared<Route>();
  r->body = std::move(body);
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
    client_->post(upstream_.at(node), "/infer", r->body, "application/json",
                  [this, r, node](std::optional<HttpResponse> resp, const std::string& err) {
                    CircuitBreaker& br = *breakers_.at(node);
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
  s["log_lines"] = static_cast<long long>(log_lines_emitted());
  s["log_lines_suppressed"] = static_cast<long long>(log_lines_suppressed());
  return s;
}

}  // namespace die
