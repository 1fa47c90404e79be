// Gateway: consistent-hash routing on request_id with a circuit breaker per worker and failover.
//
// Reference: Gateway (src/gateway.cpp:12-159) and main (:161-200).  Same routing key, ring,
// breaker thresholds, failover order (primary, then every other node in ring order), /stats
// document and error bodies.  Differences: the request body is forwarded verbatim (only
// `request_id` is extracted, no re-parse/re-dump), gateway->worker traffic is event-driven over
// keep-alive connections (core/http_async.h: any number of forwards in flight per worker, no thread
// per request; the reference's single httplib::Client per worker serialises all forwards to that
// worker: SURVEY Q4), per-request logging is off unless --verbose (Q11), and a worker's answer
// marked as a client error (X-Die-Error: client, e.g. malformed JSON) is passed through without
// failover and without counting against the worker's breaker -- in the reference any non-200 is a
// breaker failure, so five malformed requests open every breaker (src/gateway.cpp:104-122).
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
#include "../core/http_async.h"
#include "../core/json.h"
#include "../core/shm_arena.h"
#include "circuit_breaker.h"
#include "stage_stats.h"
#include "consistent_hash.h"

namespace die {

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
  int client_threads = 0;  // event loops of the worker-side client (0 = half the usable CPUs, >= 2)
  bool verbose = false;  // --verbose = log level debug (core/log.h)
  // Co-located workers (loopback upstreams) get large bodies as a shared-memory descriptor instead
  // of the bytes (core/shm_arena.h); a worker that cannot map the arena answers X-Die-Error: shm
  // and is sent the bytes from then on.
  bool local_shm = true;
  size_t shm_mb = 512;
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
  // Route one /infer body (reference Gateway::routeRequest, src/gateway.cpp:38-61): primary by
  // request_id, then every other node in ring order; `done(status, response)` runs once, on a
  // client loop thread (or inline for requests that never reach a worker).
  // shm_off >= 0: the body lies in this gateway's arena at that offset.
  void routeRequest(AsyncHttpClient::BodyRef body, long long shm_off, std::function<void(HttpResponse&&)> done);
  const ConsistentHash& ring() const { return ring_; }

 private:
  struct Route;
  void try_next(std::shared_ptr<Route> r);

  GatewayOptions opt_;
  ConsistentHash ring_;
  std::map<std::string, std::unique_ptr<CircuitBreaker>> breakers_;
  std::map<std::string, int> upstream_;  // node -> AsyncHttpClient upstream id
  std::shared_ptr<ShmArena> shm_;
  struct NodeShm {
    bool local = false;
    std::atomic<bool> ok{true};
  };
  std::map<std::string, std::unique_ptr<NodeShm>> node_shm_;
  std::atomic<int64_t> shm_forwards_{0}, byte_forwards_{0};
  std::unique_ptr<AsyncHttpClient> client_;
  HttpServer server_;
  std::atomic<int64_t> routed_{0}, failovers_{0}, failed_{0}, client_errors_{0};
  // per-stage latency (tail analysis): request head parsed -> body received (recv); forward issued
  // -> worker answer received, per attempt (upstream); body received -> answer handed to the
  // reactor (route); head parsed -> answer handed over (total)
  StageHist h_recv_, h_upstream_, h_route_, h_total_;
};

}  // namespace die
