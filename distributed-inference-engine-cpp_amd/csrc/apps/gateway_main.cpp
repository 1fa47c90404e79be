// gateway <worker1:port> [worker2:port] ... [--flags]
// Same positional CLI as the reference (src/gateway.cpp:161-171); listens on :8000 by default.
#include <pthread.h>
#include <csignal>
#include <iostream>

#include "../core/flags.h"
#include "../core/log.h"
#include "../serve/gateway.h"

int main(int argc, char** argv) {
  die::Flags f(argc, argv, {"verbose", "no-local-shm"});
  const auto& pos = f.positional();
  if (pos.empty()) {
    std::cerr << "Usage: " << argv[0] << " <worker1:port> [worker2:port] ... [options]\n"
              << "Example: " << argv[0] << " localhost:8001 localhost:8002 localhost:8003\n"
              << "Options (defaults = reference constants):\n"
              << "  --port N (8000)  --failure-threshold N (5)  --success-threshold N (2)\n"
              << "  --breaker-timeout-s S (30)  --vnodes N (150)  --connect-timeout-ms N (5000)\n"
              << "  --read-timeout-ms N (5000)  --client-threads N (CPUs/2)  --http-threads N  --verbose\n"
              << "  --log-level trace|debug|info|warn|error|off (info; env DIE_LOG_LEVEL)\n"
              << "  --no-local-shm (send co-located workers the body bytes, not a shared-memory descriptor)"
              << "  --shm-mb N (512)"
              << std::endl;
    return 1;
  }
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGINT);
  sigaddset(&sigs, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  die::GatewayOptions o;
  o.workers = pos;
  o.host = f.str("host", "0.0.0.0");
  o.port = static_cast<int>(f.i("port", 8000));
  o.failure_threshold = static_cast<int>(f.i("failure-threshold", 5));
  o.success_threshold = static_cast<int>(f.i("success-threshold", 2));
  o.breaker_timeout = std::chrono::milliseconds(static_cast<long long>(f.f("breaker-timeout-s", 30.0) * 1000));
  o.vnodes = static_cast<int>(f.i("vnodes", 150));
  o.connect_timeout = std::chrono::milliseconds(f.i("connect-timeout-ms", 5000));
  o.read_timeout = std::chrono::milliseconds(f.i("read-timeout-ms", 5000));
  o.client_threads = static_cast<int>(f.i("client-threads", 0));
  o.local_shm = !f.b("no-local-shm");
  o.shm_mb = static_cast<size_t>(f.i("shm-mb", 512));
  o.http_threads = static_cast<int>(f.i("http-threads", 0));
  o.verbose = f.b("verbose");
  if (o.verbose) die::set_log_level(die::LogLevel::DEBUG);
  die::LogLevel lv;
  if (die::parse_log_level(f.str("log-level", ""), &lv)) die::set_log_level(lv);
  die::Gateway gw(o);
  if (gw.start() < 0) {
    std::cerr << "Failed to bind port " << o.port << std::endl;
    return 1;
  }
  std::cout << "Gateway listening on port " << gw.port() << "\n"
            << "Workers: " << o.workers.size() << "\n"
            << "Circuit breakers enabled\n"
            << "Ready!" << std::endl;
  int sig = 0;
  sigwait(&sigs, &sig);
  gw.stop();
  return 0;
}
