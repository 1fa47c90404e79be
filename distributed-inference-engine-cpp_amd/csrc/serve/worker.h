// Worker node: HTTP /infer + /health in front of an LRU cache, a dynamic batcher and an Engine.
//
// Reference: WorkerNode (src/worker_node.cpp:27-143) and its main (:145-204).  Same routes, JSON
// keys, status codes, cache-hit constants (`cached:true`, `inference_time_us:50`) and miss timing
// (batch wall time / batch size).  Differences: async request handling (no HTTP thread blocked per
// request), floats decoded straight into engine-owned (pinned) staging -- or, with a HIP engine,
// the raw input_data text copied there and converted on the GPU (device decode) -- full-input cache keys,
// oversized inputs rejected with 500 instead of corrupting the batch, optional fault
// injection for resilience tests.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../core/http.h"
#include "../core/json.h"
#include "../core/shm_arena.h"
#include "../engine/engine.h"
#include "batcher.h"
#include "lru_cache.h"
#include "stage_stats.h"

namespace die {

struct WorkerOptions {
  std::string node_id = "worker";
  std::string host = "0.0.0.0";
  int port = 8001;
  std::string model_path;
  size_t cache_capacity = 1000;                          // src/worker_node.cpp:33
  int max_batch = 32;                                    // :35
  std::chrono::milliseconds batch_timeout{20};           // :36
  BatchPolicy policy = BatchPolicy::GREEDY;
  // GREEDY: when the queue holds more than the previous batch carried, dispatch the mean of the two
  // (BatchProcessor::set_balance) instead of everything -- evens out closed-loop batch sizes
  bool batch_balance = true;
  int http_threads = 0;
  EngineOptions engine;
  // fault injection (tests / fault drills)
  double fault_fail_rate = 0.0;
  int fault_latency_ms = 0;
  bool verbose = false;
  // Accept X-Die-Shm body descriptors from a co-located gateway (core/shm_arena.h).
  bool accept_shm = true;
  // Share the listening port with other processes (the ranks of a data-parallel worker).
  bool reuse_port = false;
  // /infer bodies are parsed (JSON scan, 4-bit text packing, cache key) on this many pool threads
  // instead of the connection's reactor, so a reactor busy parsing a 1 MB body never holds a
  // finished response back.  0 = parse on the reactor; -1 = auto (a quarter of the CPUs, >= 2).
  int parse_threads = -1;
  // An idle parse thread polls the queue this long before it sleeps on the condition variable: a
  // request that arrives meanwhile is taken without a futex wake-up (0 = sleep at once).
  int parse_spin_us = 0;
};

class WorkerNode {
 public:
  // Takes ownership of an engine (tests inject custom engines); nullptr = create from options.
  explicit WorkerNode(WorkerOptions opt, std::unique_ptr<Engine> engine = nullptr);
  ~WorkerNode();

  int start();  // returns bound port (or -1)
  void wait();
  void stop();
  int port() const { return server_.port(); }

  Json getHealth() const;
  Engine& engine() { return *engine_; }
  const WorkerOptions& options() const { return opt_; }

  struct Pending {
    std::string request_id;
    SampleBuffer buf;
    size_t len = 0;       // parsed floats in buf
    size_t text_len = 0;  // > 0: buf holds input_data text for device decode instead
    size_t text_off = 0;  // offset of that text in the request body (host-fallback error offsets)
    bool packed = false;  // the text is 4-bit packed (core/textpack.h): (text_len + 1) / 2 bytes
    long staged = -1;     // Engine::stage_text ticket (text already uploading to the device)
    InputKey key;
    std::chrono::steady_clock::time_point t_start{}, t_queued{};
  };
  struct Result {
    std::vector<float> output;
    int64_t inference_time_us = 0;
    int decode_status = 0;  // device decode: bit 0 = needs host parse, 2 = too many values
    int ntok = 0;
    std::chrono::steady_clock::time_point t_dispatch{}, t_done{};
  };

 private:
  void handle_infer(HttpRequest& req, Responder res);
  void handle_admin_fault(HttpRequest& req, Responder res);
  // Queue a parsed (or text) request on the batcher and answer `res` when it completes.
  void dispatch(Pending p, Responder res);
  // Device decode flagged the text: convert it with the strict host parser and re-dispatch.
  void host_fallback(SampleBuffer text_buf, size_t text_len, bool packed, size_t text_off, std::string id, InputKey key,
                     Responder res);
  HttpResponse error_response(int status, const std::string& msg, bool client_error = false) const;

  WorkerOptions opt_;
  std::unique_ptr<Engine> engine_;
  LRUCache<InputKey, std::vector<float>, InputKeyHash> cache_;
  std::unique_ptr<BatchProcessor<Pending, Result>> batcher_;
  HttpServer server_;
  std::atomic<int64_t> total_requests_{0};
  std::atomic<int64_t> cache_hits_{0};
  std::atomic<int64_t> errors_{0};
  std::atomic<int64_t> parse_ns_{0}, parse_bytes_{0}, parsed_{0};
  std::atomic<int64_t> device_decoded_{0}, decode_fallbacks_{0}, shm_bodies_{0}, staging_exhausted_{0};
  ShmReader shm_reader_;
  // request stages: parse (body -> staging), queue (batcher wait), engine (submit -> outputs on
  // host), respond (outputs -> serialised response), total (handler entry -> response)
  StageHist h_recv_, h_parse_, h_queue_, h_engine_, h_respond_, h_total_;  // recv: head parsed -> body complete
  std::atomic<double> fault_fail_rate_{0.0};
  std::atomic<int> fault_latency_ms_{0};
  std::chrono::steady_clock::time_point started_;
  // parse pool (WorkerOptions::parse_threads)
  struct ParseJob {
    std::shared_ptr<HttpRequest> req;
    Responder res;
  };
  void parse_loop();
  std::mutex parse_mu_;
  std::condition_variable parse_cv_;
  std::deque<ParseJob> parse_q_;
  std::atomic<int> parse_pending_{0};  // parse_q_.size(), readable without the lock (parse_spin_us)
  bool parse_stop_ = false;
  std::vector<std::thread> parse_threads_;
};

}  // namespace die
