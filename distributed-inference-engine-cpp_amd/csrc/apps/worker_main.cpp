// worker_node <port> <node_id> [model_path] [--flags]
// Same positional CLI and MODEL_PATH fallback as the reference (src/worker_node.cpp:145-168).
#include <pthread.h>
#include <csignal>
#include <iostream>

#include "../core/flags.h"
#include "../serve/worker.h"

int main(int argc, char** argv) {
  die::Flags f(argc, argv, {"verbose", "deadline", "no-graphs"});
  const auto& pos = f.positional();
  if (pos.size() < 2) {
    std::cerr << "Usage: " << argv[0] << " <port> <node_id> [model_path] [options]\n"
              << "  Or set MODEL_PATH environment variable\n"
              << "Options (defaults = reference constants):\n"
              << "  --cache-capacity N (1000)  --max-batch N (32)  --batch-timeout-ms N (20)\n"
              << "  --deadline (wait up to the timeout for full batches; default: greedy)\n"
              << "  --device auto|hip|cpu (auto)  --device-id N (0)  --precision bf16|fp32 (bf16)\n"
              << "  --pipeline-depth N (2)  --no-graphs  --http-threads N  --host ADDR (0.0.0.0)\n"
              << "  --fault-fail-rate P  --fault-latency-ms N  --verbose" << std::endl;
    return 1;
  }
  // Block SIGINT/SIGTERM in every thread; the main thread waits for them with sigwait() and then
  // shuts down cleanly (stop() is not async-signal-safe, so it never runs in a handler).
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGINT);
  sigaddset(&sigs, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  die::WorkerOptions o;
  try {
    o.port = std::stoi(pos[0]);
  } catch (...) {
    std::cerr << "invalid port: " << pos[0] << std::endl;
    return 1;
  }
  o.node_id = pos[1];
  if (pos.size() >= 3) {
    o.model_path = pos[2];
  } else if (const char* env = std::getenv("MODEL_PATH")) {
    o.model_path = env;
  } else {
    std::cerr << "Error: No model path provided!\n  Provide as: " << argv[0]
              << " <port> <node_id> <model_path>\n  Or set: export MODEL_PATH=/path/to/model.onnx" << std::endl;
    return 1;
  }
  o.host = f.str("host", "0.0.0.0");
  o.cache_capacity = static_cast<size_t>(f.i("cache-capacity", 1000));
  o.max_batch = static_cast<int>(f.i("max-batch", 32));
  o.batch_timeout = std::chrono::milliseconds(f.i("batch-timeout-ms", 20));
  o.policy = f.b("deadline") ? die::BatchPolicy::DEADLINE : die::BatchPolicy::GREEDY;
  o.http_threads = static_cast<int>(f.i("http-threads", 0));
  o.engine.device = f.str("device", "auto");
  o.engine.device_id = static_cast<int>(f.i("device-id", 0));
  o.engine.precision = f.str("precision", "bf16");
  o.engine.pipeline_depth = static_cast<int>(f.i("pipeline-depth", 2));
  o.engine.use_graphs = !f.b("no-graphs");
  o.engine.device_decode = !f.b("no-device-decode");
  o.engine.shard_id = o.port % 3;  // reference: InferenceEngine(model_path, port % 3) (unused there too)
  o.fault_fail_rate = f.f("fault-fail-rate", 0.0);
  o.fault_latency_ms = static_cast<int>(f.i("fault-latency-ms", 0));
  o.verbose = f.b("verbose");

  std::cout << "Using model: " << o.model_path << std::endl;
  std::unique_ptr<die::WorkerNode> worker;
  try {
    worker = std::make_unique<die::WorkerNode>(o);
  } catch (const std::exception& e) {
    std::cerr << "Failed to start worker: " << e.what() << std::endl;
    return 1;
  }
  auto& eng = worker->engine();
  auto shape_str = [](const std::vector<int64_t>& s) {
    std::string r = "[";
    for (size_t k = 0; k < s.size(); ++k) r += (k ? ", " : "") + std::to_string(s[k]);
    return r + "]";
  };
  if (worker->start() < 0) {
    std::cerr << "Failed to bind port " << o.port << std::endl;
    return 1;
  }
  std::cout << "━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━\n"
            << "Worker Node: " << o.node_id << "\n"
            << "━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━\n"
            << "   Port:              " << worker->port() << "\n"
            << "   Engine:            " << eng.name() << "\n"
            << "   Input shape:       " << shape_str(eng.getInputShape()) << "\n"
            << "   Output shape:      " << shape_str(eng.getOutputShape()) << "\n"
            << "   Cache Capacity:    " << o.cache_capacity << " entries\n"
            << "   Batch Size:        " << o.max_batch << " requests\n"
            << "   Batch Timeout:     " << o.batch_timeout.count() << "ms\n"
            << "━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━━\n"
            << "Ready to accept requests!\n"
            << std::endl;
  int sig = 0;
  sigwait(&sigs, &sig);
  std::cout << "signal " << sig << ": draining and shutting down" << std::endl;
  worker->stop();
  return 0;
}
