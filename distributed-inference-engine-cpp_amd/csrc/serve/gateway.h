// Gateway: consistent-hash routing on request_id with a circuit breaker per worker and failover.
//
// Reference: Gateway (src/gateway.cpp:12-159) and main (:161-200).  Same routing key, ring,
// breaker thresholds, failover order (primary, then every other node in ring order), /stats
// document and error bodies.  Differences: the request body is forwarded verbatim (only
// `request_id` is extracted, no re-parse/re-dump), gateway->worker traffic uses a keep-alive
// connection pool per worker (the reference's single httplib::Client per worker serialises all
// forwards to that worker: SURVEY Q4), and per-request logging is off unless --verbose (Q11).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "../core/http.h"
#include "../core/json.h"
#include "circuit_breaker.h"
#include "consistent_hash.h"

namespace die {

class ThreadPool {
 public:
  explicit ThreadPool(size_t n);
  ~ThreadPool();
  void post(std::function<void()> fn);

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> threads_;
  bool stop_ = false;
};

struct GatewayOptions {
  std::vector<std::string> workers;
  std::string host = "0.0.0.0";
  int port = 8000;                                  // src/gateway.cpp:198
  int failure_threshold = 5;                        // :20
  int success_threshold = 2;                        // :21
  std::chrono::milliseconds breaker_timeout{30000};  // :22
  int vnodes = 150;                                 // include/consistent_hash.h:12
  std::chrono::milliseconds connect_timeout{5000};  // :32
  std::chrono::milliseconds read_timeout{5000};     // :33
  int http_threads = 0;
  int forward_threads = 256;
  bool verbose = false;
};

class Gateway {
 public:
  explicit Gateway(GatewayOptions opt);
  ~Gateway();
  int start();
  void wait();
  void stop();
  int port() const { return server_.port(); }

  Json getStats() const;
  // Synchronous routing (tests / reuse): returns (status, body).
  std::pair<int, std::string> routeRequest(const std::string& body);
  const ConsistentHash& ring() const { return ring_; }

 private:
  std::optional<std::string> tryNode(const std::string& node, const std::string& body);

  GatewayOptions opt_;
  ConsistentHash ring_;
  std::map<std::string, std::unique_ptr<CircuitBreaker>> breakers_;
  std::map<std::string, std::unique_ptr<HttpClient>> clients_;
  std::unique_ptr<ThreadPool> pool_;
  HttpServer server_;
  std::atomic<int64_t> routed_{0}, failovers_{0}, failed_{0};
};

}  // namespace die
