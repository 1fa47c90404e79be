// loadgen [--host H] [--port P] [--connections C] [--requests N] [--warmup W]
//         [--payload ref|full] [--input-numel K] [--decimals D] [--distinct M]
// Prints one JSON document with throughput and latency percentiles.
#include <iostream>

#include "../core/flags.h"
#include "../serve/loadgen.h"

int main(int argc, char** argv) {
  die::Flags f(argc, argv);
  die::LoadgenOptions o;
  o.host = f.str("host", "127.0.0.1");
  o.port = static_cast<int>(f.i("port", 8000));
  o.path = f.str("path", "/infer");
  o.connections = static_cast<int>(f.i("connections", 50));
  o.requests = f.i("requests", 10000);
  o.warmup = f.i("warmup", 0);
  o.payload = f.str("payload", "ref");
  o.input_numel = static_cast<size_t>(f.i("input-numel", 3 * 224 * 224));
  o.decimals = static_cast<int>(f.i("decimals", 4));
  o.distinct = f.i("distinct", 0);
  o.timeout_ms = static_cast<int>(f.i("timeout-ms", 10000));
  std::cout << die::run_loadgen(o).dump() << std::endl;
  return 0;
}
