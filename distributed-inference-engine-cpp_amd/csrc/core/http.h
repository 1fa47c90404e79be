// In-tree HTTP/1.1 server (epoll reactors) and pooled keep-alive client.
//
// Replaces cpp-httplib v0.14.3 (reference setup.sh:42; used at src/worker_node.cpp:172-202,
// src/gateway.cpp:29-33,99-103,174-198).  Differences that matter for throughput:
//  * handlers are asynchronous: a handler receives a Responder and may complete it later from any
//    thread, so a request waiting on the batcher never pins a server thread;
//  * the client keeps a pool of keep-alive connections per upstream instead of one mutex-guarded
//    connection, so concurrent gateway->worker requests are not serialised.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

namespace die {

// Memory a request body may be received into instead of HttpRequest::body (see
// HttpServer::set_body_allocator); `owner` releases it.
struct BodyBuffer {
  char* data = nullptr;
  size_t capacity = 0;
  std::shared_ptr<void> owner;
};

struct HttpRequest {
  std::string method;
  std::string path;    // without query string
  std::string query;   // raw query string (after '?'), may be empty
  std::vector<std::pair<std::string, std::string>> headers;  // names lower-cased
  std::string body;    // capacity always >= size + 64 (slack for SIMD parsers)
  // Body received into allocator memory (then `body` is empty): ext_len bytes at ext_body, followed by
  // 64 zero bytes of slack; ext_owner keeps the memory alive.
  char* ext_body = nullptr;
  size_t ext_len = 0;
  std::shared_ptr<void> ext_owner;
  bool keep_alive = true;
  bool peer_loopback = false;  // the connection comes from this host (127.0.0.0/8, ::1)
  std::chrono::steady_clock::time_point t_headers{};  // when the request head was parsed
  std::string_view header(std::string_view name) const;  // name must be lower-case
  std::string_view body_view() const { return ext_body ? std::string_view(ext_body, ext_len) : std::string_view(body); }
};

struct HttpResponse {
  int status = 200;
  std::string content_type = "application/json";
  std::string body;
  bool close = false;
  // extra headers (server: written as given; clients: every received header, names lower-cased)
  std::vector<std::pair<std::string, std::string>> headers;
  std::string_view header(std::string_view lower_name) const {
    for (auto& kv : headers)
      if (kv.first == lower_name) return kv.second;
    return {};
  }
};

const char* http_status_text(int status);

class HttpServer;

// One-shot completion handle for a request.  Copyable; only the first send() has an effect.
class Responder {
 public:
  Responder() = default;
  // Complete with a ready response (any thread).
  void send(HttpResponse resp) const;
  // Complete by running `build` on the connection's reactor thread (spreads serialisation work
  // over the reactors instead of the thread that finished the request).
  void defer(std::function<HttpResponse()> build) const;
  bool valid() const { return static_cast<bool>(state_); }

 private:
  friend class HttpServer;
  struct State;
  std::shared_ptr<State> state_;
};

class HttpServer {
 public:
  using Handler = std::function<void(HttpRequest& req, Responder res)>;

  HttpServer();
  ~HttpServer();
  HttpServer(const HttpServer&) = delete;
  HttpServer& operator=(const HttpServer&) = delete;

  void route(const std::string& method, const std::string& path, Handler h);
  // Receive Content-Length bodies of >= min_bytes straight into memory from `alloc(len + 64)`
  // (e.g. a shared-memory arena the next hop reads in place); an empty BodyBuffer declines.
  void set_body_allocator(std::function<BodyBuffer(size_t)> alloc, size_t min_bytes) {
    body_alloc_ = std::move(alloc);
    body_alloc_min_ = min_bytes;
  }
  // Bind and start `threads` reactor threads (0 = hardware concurrency, capped at 32).
  // port 0 picks an ephemeral port; returns the bound port, or -1 on failure.
  // reuse_port: SO_REUSEPORT, so several processes (the ranks of a data-parallel worker) can listen
  // on the same port and the kernel spreads incoming connections over them.
  int start(const std::string& host, int port, int threads = 0, bool reuse_port = false);
  // Block until stop() is called.
  void wait();
  void stop();
  int port() const { return port_; }
  bool running() const { return running_.load(); }
  uint64_t requests_served() const { return served_.load(); }
  size_t max_body_bytes = 512u << 20;

 private:
  struct Reactor;
  struct Conn;
  friend class Responder;
  void reactor_loop(Reactor* r);
  void dispatch(Reactor* r, Conn* c);

  std::vector<std::pair<std::pair<std::string, std::string>, Handler>> routes_;
  std::function<BodyBuffer(size_t)> body_alloc_;
  size_t body_alloc_min_ = 0;
  std::vector<std::unique_ptr<Reactor>> reactors_;
  std::vector<std::thread> threads_;
  int listen_fd_ = -1;
  int port_ = -1;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> served_{0};
  std::mutex wait_mu_, stop_mu_;
  std::condition_variable wait_cv_;
};

// Blocking HTTP/1.1 client with a keep-alive connection pool; safe for concurrent use.
class HttpClient {
 public:
  HttpClient(std::string host, int port, std::chrono::milliseconds connect_timeout = std::chrono::seconds(5),
             std::chrono::milliseconds read_timeout = std::chrono::seconds(5), size_t max_idle = 256);
  ~HttpClient();
  // Returns nullopt on transport failure (connect/send/recv/timeout/malformed response);
  // `error` then holds a description.
  std::optional<HttpResponse> request(const std::string& method, const std::string& path, std::string_view body,
                                      const std::string& content_type = "application/json",
                                      std::string* error = nullptr);
  std::optional<HttpResponse> post(const std::string& path, std::string_view body,
                                   const std::string& content_type = "application/json", std::string* error = nullptr) {
    return request("POST", path, body, content_type, error);
  }
  std::optional<HttpResponse> get(const std::string& path, std::string* error = nullptr) {
    return request("GET", path, {}, "", error);
  }
  const std::string& host() const { return host_; }
  int port() const { return port_; }

 private:
  int connect_new(std::string* error);
  void release(int fd);
  std::string host_;
  int port_;
  std::chrono::milliseconds connect_timeout_, read_timeout_;
  size_t max_idle_;
  std::mutex mu_;
  std::vector<int> idle_;
};

// Parse "host:port", "http://host:port/..." -> (host, port); default port 8080 like the
// reference's Gateway::parseUrl (src/gateway.cpp:130-154).
std::pair<std::string, int> parse_host_port(const std::string& url);

}  // namespace die
