#include "gateway.h"

#include <iostream>

namespace die {

ThreadPool::ThreadPool(size_t n) {
  for (size_t i = 0; i < n; ++i)
    threads_.emplace_back([this] {
      while (true) {
        std::function<void()> fn;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
          if (q_.empty()) return;
          fn = std::move(q_.front());
          q_.pop_front();
        }
        fn();
      }
    });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void ThreadPool::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(fn));
  }
  cv_.notify_one();
}

namespace {

std::string error_body(const std::string& msg) {
  Json j = Json::object();
  j["error"] = msg;
  return j.dump();
}

}  // namespace

Gateway::Gateway(GatewayOptions opt) : opt_(std::move(opt)), ring_(opt_.vnodes) {
  for (const auto& w : opt_.workers) {
    ring_.addNode(w);
    breakers_[w] = std::make_unique<CircuitBreaker>(opt_.failure_threshold, opt_.success_threshold,
                                                    opt_.breaker_timeout);
    auto hp = parse_host_port(w);
    clients_[w] = std::make_unique<HttpClient>(hp.first, hp.second, opt_.connect_timeout, opt_.read_timeout);
    if (opt_.verbose) std::cout << "Parsed URL: " << w << " -> host=" << hp.first << " port=" << hp.second << std::endl;
  }
  pool_ = std::make_unique<ThreadPool>(static_cast<size_t>(std::max(1, opt_.forward_threads)));
  server_.route("POST", "/infer", [this](HttpRequest& req, Responder res) {
    auto body = std::make_shared<std::string>(std::move(req.body));
    pool_->post([this, body, res] {
      auto r = routeRequest(*body);
      HttpResponse resp;
      resp.status = r.first;
      resp.body = std::move(r.second);
      res.send(std::move(resp));
    });
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
void Gateway::stop() { server_.stop(); }

std::optional<std::string> Gateway::tryNode(const std::string& node, const std::string& body) {
  auto b = breakers_.find(node);
  if (b == breakers_.end()) return std::nullopt;
  CircuitBreaker& breaker = *b->second;
  if (!breaker.allowRequest()) {
    if (opt_.verbose) std::cout << "Circuit breaker OPEN for " << node << ", skipping" << std::endl;
    return std::nullopt;
  }
  auto c = clients_.find(node);
  if (c == clients_.end()) {
    breaker.recordFailure();
    return std::nullopt;
  }
  std::string err;
  auto resp = c->second->post("/infer", body, "application/json", &err);
  if (resp && resp->status == 200) {
    breaker.recordSuccess();
    return std::move(resp->body);
  }
  if (opt_.verbose) {
    if (resp) std::cerr << "Request to " << node << " failed with status: " << resp->status << std::endl;
    else std::cerr << "Request to " << node << " failed: " << err << std::endl;
  }
  breaker.recordFailure();
  return std::nullopt;
}

std::pair<int, std::string> Gateway::routeRequest(const std::string& body) {
  routed_++;
  std::string request_id;
  if (!find_top_level_string(body, "request_id", request_id)) {
    // Slow path only to produce the same kind of error the reference returns.
    try {
      Json j = Json::parse(body);
      request_id = j.at("request_id").as_string();
    } catch (const std::exception& e) {
      failed_++;
      return {500, error_body(e.what())};
    }
  }
  const std::string target = ring_.getNode(request_id);
  if (target.empty()) {
    failed_++;
    return {500, error_body("No workers available")};
  }
  if (auto r = tryNode(target, body)) return {200, std::move(*r)};
  for (const auto& node : ring_.getAllNodes()) {
    if (node == target) continue;
    if (auto r = tryNode(node, body)) {
      failovers_++;
      return {200, std::move(*r)};
    }
  }
  failed_++;
  return {500, error_body("All workers failed or circuit breakers open")};
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
  return s;
}

}  // namespace die
