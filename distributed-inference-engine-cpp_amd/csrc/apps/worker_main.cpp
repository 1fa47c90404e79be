// worker_node <port> <node_id> [model_path] [--flags]
// Same positional CLI and MODEL_PATH fallback as the reference (src/worker_node.cpp:145-168).
// Data parallel: `--devices 0,1,...,7` makes this worker the DP leader on the first device and
// spawns one follower process per further device (`worker_node --dp-follower ...`, started with
// posix_spawn before this process touches the GPU).
#include <pthread.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <csignal>
#include <iostream>
#include <sstream>
#include <thread>

#include "../core/flags.h"
#include "../core/log.h"
#include "../core/sysinfo.h"
#include "../serve/worker.h"

extern char** environ;

namespace {

std::vector<int> parse_devices(const std::string& s) {
  std::vector<int> d;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ','))
    if (!tok.empty()) d.push_back(std::stoi(tok));
  return d;
}

// Engine options from the command line: the same flags for an ingesting worker, a DP rank it
// spawns and a compute-only follower, so every rank of a group plans the same program.
die::EngineOptions engine_options_from_flags(const die::Flags& f, const std::string& default_device) {
  die::EngineOptions eo;
  eo.device = f.str("device", default_device);
  eo.device_id = static_cast<int>(f.i("device-id", 0));
  eo.max_batch = static_cast<int>(f.i("max-batch", 32));
  eo.precision = f.str("precision", "fp32");
  eo.pipeline_depth = static_cast<int>(f.i("pipeline-depth", 3));
  eo.use_graphs = !f.b("no-graphs");
  eo.device_decode = !f.b("no-device-decode");
  eo.stage_slots = static_cast<int>(f.i("stage-slots", 0));
  eo.pace = !f.b("no-pace");
  eo.pack_text = !f.b("no-pack-text");
  eo.branch_streams = f.b("branch-streams");
  eo.exec_streams = static_cast<int>(f.i("exec-streams", 1));
  eo.tune_cache = f.str("tune-cache", "auto");
  eo.copy_streams = static_cast<int>(f.i("copy-streams", 0));
  eo.bucket_div = static_cast<int>(f.i("bucket-div", 8));
  eo.coarse_buckets = f.b("coarse-buckets");
  eo.pace_lead_scale = f.f("pace-lead-scale", 1.0);
  eo.splitk_fused_margin = static_cast<float>(f.f("splitk-fused-margin", 0.0));
  eo.splitk_two_kernel = f.b("splitk-two-kernel");
  eo.result_stream = !f.b("no-result-stream");
  eo.completion_poll_us = static_cast<int>(f.i("completion-poll-us", 0));
  eo.bn_on_load = f.b("bn-on-load");
  eo.fuse_pairs = !f.b("no-fuse-pairs");
  eo.fuse_stem_pool = !f.b("no-fuse-stem-pool");
  eo.fuse_gap_fc = f.b("fuse-gap-fc");
  eo.fold_layernorm = !f.b("no-fold-layernorm");
  eo.ln_stats_epilogue = !f.b("no-ln-stats-epilogue");
  eo.tune_in_graph = f.b("tune-in-graph");
  eo.tune_orders = !f.b("no-tune-orders");
  eo.tune_tail = f.b("tune-tail");
  if (f.has("tune-streamk")) eo.tune_streamk = f.b("tune-streamk");
  eo.tune_cold = !f.b("tune-warm");
  eo.efficient_batch = !f.b("no-efficient-batch");
  eo.efficient_batch_tol = f.f("efficient-batch-tol", 0.0);
  eo.efficient_batch_margin = f.f("efficient-batch-margin", eo.efficient_batch_margin);
  eo.dp_backend = f.str("dp-backend", "rccl");
  eo.dp_force_merge = f.b("dp-force-merge");
  eo.fail_batch_every = static_cast<int>(f.i("fail-batch-every", 0));
  return eo;
}

// worker_node --dp-follower <model> --dp-group G --dp-rank R --dp-world N --device-id D [engine flags]
int follower_main(die::Flags& f, sigset_t& sigs) {
  const auto& pos = f.positional();
  if (pos.empty()) {
    std::cerr << "--dp-follower needs the model path" << std::endl;
    return 1;
  }
  die::EngineOptions eo = engine_options_from_flags(f, "hip");
  eo.dp_group = f.str("dp-group", "");
  eo.dp_rank = static_cast<int>(f.i("dp-rank", 1));
  eo.dp_world = static_cast<int>(f.i("dp-world", 2));
  std::atomic<bool> stop{false};
  std::thread sig_thread([&] {
    int sig = 0;
    sigwait(&sigs, &sig);
    stop = true;
  });
  long served = 0;
  int rc = 0;
  try {
    served = die::run_dp_follower(pos[0], eo, &stop);
  } catch (const std::exception& e) {
    std::cerr << "dp follower " << eo.dp_rank << " failed: " << e.what() << std::endl;
    rc = 1;
  }
  std::cout << "dp follower " << eo.dp_rank << " served " << served << " batches" << std::endl;
  pthread_kill(sig_thread.native_handle(), SIGTERM);
  sig_thread.join();
  return rc;
}

const std::vector<std::string> kBoolFlags = {"verbose", "deadline", "no-graphs", "no-device-decode", "dp-follower",
                                             "no-shm", "reuse-port", "dp-no-ingest", "no-pace", "no-pack-text",
                                             "branch-streams", "coarse-buckets", "bn-on-load", "no-fuse-pairs", "no-fuse-stem-pool", "fuse-gap-fc", "no-fold-layernorm", "no-ln-stats-epilogue", "tune-in-graph", "no-tune-orders", "tune-tail", "tune-warm",
                                             "no-efficient-batch", "no-batch-balance",
                                             "dp-force-merge"};

}  // namespace

int main(int argc, char** argv) {
  die::configure_hip_runtime_env();  // before anything touches HIP (spawned DP ranks inherit it)
  die::Flags f(argc, argv, kBoolFlags);
  const auto& pos = f.positional();
  if (f.b("dp-follower")) {
    sigset_t fs;
    sigemptyset(&fs);
    sigaddset(&fs, SIGINT);
    sigaddset(&fs, SIGTERM);
    pthread_sigmask(SIG_BLOCK, &fs, nullptr);
    return follower_main(f, fs);
  }
  if (pos.size() < 2) {
    std::cerr << "Usage: " << argv[0] << " <port> <node_id> [model_path] [options]\n"
              << "  Or set MODEL_PATH environment variable\n"
              << "Options (defaults = reference constants):\n"
              << "  --cache-capacity N (1000)  --max-batch N (32)  --batch-timeout-ms N (20)\n"
              << "  --deadline (wait up to the timeout for full batches; default: greedy)\n"
              << "  --device auto|hip|cpu (auto)  --device-id N (0)  --precision fp32|bf16 (fp32)\n"
              << "  --pipeline-depth N (3)  --no-graphs  --no-device-decode  --stage-slots N (0 = off, -1 = auto)  --exec-streams N (1)\n"
              << "  --no-pace  --no-pack-text  --branch-streams  --copy-streams N (0 = auto)  --bucket-div N (8)  --coarse-buckets\n"
              << "  --pace-lead-scale X (1)  --splitk-fused-margin X (0)  --completion-poll-us N (0)  --bn-on-load  --no-fuse-pairs  --no-fuse-stem-pool  --fuse-gap-fc  --no-fold-layernorm  --no-ln-stats-epilogue  --tune-in-graph  --no-tune-orders  --tune-tail  --tune-warm  --no-efficient-batch  --efficient-batch-tol X (0)  --tune-cache PATH|auto|''\n"
              << "  --dp-backend rccl|host (rccl)  --dp-force-merge  --fail-batch-every N (fault injection, 0 = off)\n"
              << "  --http-threads N  --parse-threads N (-1 = auto, 0 = parse on the I/O threads)  --parse-spin-us N (0)  --no-batch-balance  --host ADDR (0.0.0.0)\n"
              << "  --devices 0,1,..  data parallel over these GPUs (one process each; --max-batch = whole batch);\n"
              << "      every rank serves HTTP on <port> (SO_REUSEPORT) unless --dp-no-ingest\n"
              << "  --fault-fail-rate P  --fault-latency-ms N  --verbose\n"
              << "  --log-level trace|debug|info|warn|error|off (info; env DIE_LOG_LEVEL)" << std::endl;
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
  o.parse_threads = static_cast<int>(f.i("parse-threads", -1));
  o.parse_spin_us = static_cast<int>(f.i("parse-spin-us", 0));
  o.batch_balance = !f.b("no-batch-balance");
  o.engine = engine_options_from_flags(f, "auto");
  o.engine.shard_id = o.port % 3;  // reference: InferenceEngine(model_path, port % 3) (unused there too)
  o.fault_fail_rate = f.f("fault-fail-rate", 0.0);
  o.fault_latency_ms = static_cast<int>(f.i("fault-latency-ms", 0));
  o.verbose = f.b("verbose");
  o.accept_shm = !f.b("no-shm");
  o.reuse_port = f.b("reuse-port");
  if (f.i("dp-rank", 0) > 0) {  // an ingesting rank of a data-parallel worker (spawned by rank 0)
    o.engine.dp_rank = static_cast<int>(f.i("dp-rank", 0));
    o.engine.dp_world = static_cast<int>(f.i("dp-world", 2));
    o.engine.dp_group = f.str("dp-group", "");
  }
  if (o.verbose) die::set_log_level(die::LogLevel::DEBUG);
  die::LogLevel lv;
  if (die::parse_log_level(f.str("log-level", ""), &lv)) die::set_log_level(lv);

  // data parallel: spawn the followers first (before this process initialises HIP)
  std::vector<pid_t> followers;
  const std::vector<int> devices = parse_devices(f.str("devices", ""));
  if (devices.size() > 1) {
    o.engine.dp_world = static_cast<int>(devices.size());
    o.engine.dp_group = "die_dp_" + std::to_string(getpid());
    o.engine.device_id = devices[0];
    if (o.engine.device == "auto") o.engine.device = "hip";
    // ingest on every rank: all ranks listen on the same port (needs a fixed port)
    const bool ingest = !f.b("dp-no-ingest") && o.port > 0;
    o.reuse_port = o.reuse_port || ingest;
    // Every rank gets this worker's own flags (engine AND serving: precision, depth, batch
    // timeout, cache, parse/http threads, shm, log level, ...), then its rank-specific ones, which
    // win (later flags override earlier ones): all ranks plan the same program.
    std::vector<std::string> shared;
    for (int k = 1; k < argc; ++k) {
      const std::string a = argv[k];
      if (a.rfind("--", 0) != 0) continue;  // positionals are rank-specific
      const std::string key = a.substr(2, a.find('=') == std::string::npos ? std::string::npos : a.find('=') - 2);
      const bool is_bool = std::find(kBoolFlags.begin(), kBoolFlags.end(), key) != kBoolFlags.end();
      const bool has_value = a.find('=') == std::string::npos && !is_bool && k + 1 < argc;
      if (key == "devices" || key == "dp-no-ingest" || key == "device-id" || key == "reuse-port") {
        if (has_value) ++k;
        continue;
      }
      shared.push_back(a);
      if (has_value) shared.push_back(argv[++k]);
    }
    for (size_t r = 1; r < devices.size(); ++r) {
      std::vector<std::string> args;
      if (ingest) {
        args = {argv[0], std::to_string(o.port), o.node_id + "-r" + std::to_string(r), o.model_path};
      } else {
        args = {argv[0], "--dp-follower", o.model_path};
      }
      args.insert(args.end(), shared.begin(), shared.end());
      if (ingest) args.push_back("--reuse-port");
      for (const std::string& a : {std::string("--dp-group"), o.engine.dp_group, std::string("--dp-rank"),
                                   std::to_string(r), std::string("--dp-world"), std::to_string(devices.size()),
                                   std::string("--device-id"), std::to_string(devices[r]), std::string("--device"),
                                   o.engine.device, std::string("--max-batch"), std::to_string(o.max_batch),
                                   std::string("--precision"), o.engine.precision})
        args.push_back(a);
      std::vector<char*> av;
      for (auto& a : args) av.push_back(const_cast<char*>(a.c_str()));
      av.push_back(nullptr);
      pid_t pid = 0;
      if (posix_spawn(&pid, "/proc/self/exe", nullptr, nullptr, av.data(), environ) != 0) {
        std::cerr << "failed to spawn dp follower " << r << std::endl;
        return 1;
      }
      followers.push_back(pid);
    }
  }

  std::cout << "Using model: " << o.model_path << std::endl;
  std::unique_ptr<die::WorkerNode> worker;
  try {
    worker = std::make_unique<die::WorkerNode>(o);
  } catch (const std::exception& e) {
    std::cerr << "Failed to start worker: " << e.what() << std::endl;
    for (pid_t p : followers) {
      kill(p, SIGTERM);
      int st = 0;
      waitpid(p, &st, 0);
    }
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
  worker.reset();  // a DP leader's engine stops the group here: followers drain and exit
  for (pid_t p : followers) {
    int st = 0;
    waitpid(p, &st, 0);
  }
  return 0;
}
