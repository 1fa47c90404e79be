// Event-driven HTTP/1.1 client for proxying (the gateway's worker side).
//
// The reference gateway forwards with one blocking httplib::Client per worker shared by all server
// threads (src/gateway.cpp:29-33,99-103; SURVEY Q4: effectively one in-flight request per worker).
// Here a few loop threads own non-blocking keep-alive connections per upstream and multiplex any
// number of in-flight requests: a forward costs no thread, requests are written with writev straight
// from the caller's body buffer (a ~1 MB ResNet body is never copied in user space), and the
// completion runs a callback on the loop thread.
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "http.h"

namespace die {

class AsyncHttpClient {
 public:
  struct Options {
    int threads = 2;
    std::chrono::milliseconds connect_timeout{5000};
    std::chrono::milliseconds read_timeout{5000};
    size_t max_idle_per_upstream = 512;  // per loop thread
  };
  // resp is nullopt on transport failure (connect/send/recv/timeout/malformed); `error` says why.
  using Callback = std::function<void(std::optional<HttpResponse> resp, const std::string& error)>;

  explicit AsyncHttpClient(Options opt);
  ~AsyncHttpClient();
  AsyncHttpClient(const AsyncHttpClient&) = delete;
  AsyncHttpClient& operator=(const AsyncHttpClient&) = delete;

  // Register an upstream before the first request; returns its id.
  int add_upstream(const std::string& host, int port);
  // Request body bytes that stay valid while `owner` is held (no copy is made).
  struct BodyRef {
    const char* data = nullptr;
    size_t size = 0;
    std::shared_ptr<const void> owner;
  };
  // Thread-safe; `cb` runs exactly once, on a loop thread.  `extra_headers` ("Name: value\r\n"
  // lines) are sent as given.
  void post(int upstream, const std::string& path, BodyRef body, const std::string& content_type,
            const std::string& extra_headers, Callback cb);
  void post(int upstream, const std::string& path, std::shared_ptr<const std::string> body,
            const std::string& content_type, Callback cb) {
    BodyRef b{body ? body->data() : nullptr, body ? body->size() : 0, body};
    post(upstream, path, std::move(b), content_type, std::string(), std::move(cb));
  }
  void stop();

  long long in_flight() const { return in_flight_.load(); }
  long long connections_opened() const { return opened_.load(); }

 private:
  struct Loop;
  struct Job;
  struct Conn;
  void run(Loop* L);

  Options opt_;
  struct Upstream {
    std::string host;
    int port = 0;
    std::string host_header;
  };
  std::vector<Upstream> ups_;
  std::vector<std::unique_ptr<Loop>> loops_;
  std::vector<std::thread> threads_;
  std::atomic<bool> running_{true};
  std::atomic<unsigned> rr_{0};
  std::atomic<long long> in_flight_{0}, opened_{0};
};

}  // namespace die
