// Closed-loop HTTP load generator (C++): the reference's benchmark.py (benchmark.py:9-128) drives
// load from Python threads, which cannot produce 150,528-float ResNet payloads fast enough to
// measure an MI355X worker.  This generator keeps one keep-alive connection per client thread and
// patches a pre-serialised body per request (unique request_id and unique leading input values, so
// nothing is served from the result cache unless asked for).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../core/json.h"

namespace die {

struct LoadgenOptions {
  std::string host = "127.0.0.1";
  int port = 8000;
  std::string path = "/infer";
  int connections = 50;
  long requests = 10000;
  long warmup = 0;
  // "ref": reference payload [a, a+1, a+2], a = id % 10 (benchmark.py:21-24)
  // "full": `input_numel` values with `decimals` decimals, unique per request
  std::string payload = "ref";
  size_t input_numel = 3 * 224 * 224;
  int decimals = 4;
  uint64_t seed = 1234;
  int timeout_ms = 10000;
  std::string id_prefix = "req_";
  // Distinct payloads cycled (0 = every request unique).  With "ref" this is always 10.
  long distinct = 0;
  // Verify mode (payload "verify"): `verify_count` distinct inputs (verify_inputs: K x input_numel
  // floats, sent as shortest round-trip text) cycled over the requests, each with a unique
  // request_id; every 200 answer's output_data is compared with verify_expected (K x output_numel
  // floats) by relative L2 error <= verify_tol (0 = bit-exact) and its request_id echo is checked.
  // A shard / gather / batch-row mix-up shows up as `mismatched`, not as a slower run.
  const float* verify_inputs = nullptr;
  const float* verify_expected = nullptr;
  size_t verify_count = 0;
  size_t output_numel = 0;
  double verify_tol = 0.0;
  // Sampled verification in "full" mode (> 0): every verify_every-th request (id % verify_every ==
  // 0) carries verify input k = (id / verify_every) % verify_count instead of a unique image, its
  // answer is checked like verify mode, and its text is made unique by zero-padding the first two
  // values (0.5 -> 0.5000...: same floats, another cache key), so it is computed, never a cache hit.
  long verify_every = 0;
  // Print request numbers scrambled (a bijection of [0, 10^10), fixed width) instead of in order:
  // FNV-1a of consecutive decimal strings clusters on the gateway's ring (bench.py ring analysis).
  bool scramble_ids = false;
  // > 0: drive the connections from this many epoll threads instead of one blocking thread per
  // connection (same closed loop, one request in flight per connection), so the client takes less
  // of a CPU share it shares with the server under test.
  int io_threads = 0;
  // Called once, on the calling thread, after every connection is open, its payload template built
  // and the warm-up done, right before the timed phase starts (bench.py: the barrier that opens the
  // timed window runs here, so building payloads is never inside it).
  void (*on_ready)(void*) = nullptr;
  void* on_ready_arg = nullptr;
};

// Runs warmup then the timed phase; returns {"ok","failed","wall_s","rps","latency_ms":{...},
// "errors":{...}} (+ "verified","mismatched","max_rel_err","bad_request_id" in verify mode).
Json run_loadgen(const LoadgenOptions& opt);

}  // namespace die
