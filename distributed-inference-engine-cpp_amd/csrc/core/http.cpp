#include <pthread.h>
#include "http.h"

#include <arpa/inet.h>

#include <atomic>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>

#include "http_util.h"
#include "json.h"
#include "sysinfo.h"

namespace die {

namespace http_detail {

struct IgnoreSigpipe {
  IgnoreSigpipe() { signal(SIGPIPE, SIG_IGN); }
} ignore_sigpipe;

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? static_cast<char>(c - 'A' + 'a') : c; }

std::string to_lower(std::string_view s) {
  std::string o(s);
  for (auto& c : o) c = lower(c);
  return o;
}

bool iequals(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (lower(a[i]) != lower(b[i])) return false;
  return true;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

namespace {
std::atomic<int> g_sock_buf_effective{-1};
}

int sock_buf_effective() { return g_sock_buf_effective.load(std::memory_order_relaxed); }

void set_nodelay(int fd, bool loopback_peer) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  // Loopback peers only: fixed 4 MiB socket buffers (DIE_SOCK_BUF_KB overrides, 0 = kernel
  // autotuning), so a ~1 MB request body crosses loopback in fewer send/recv rounds.  A/B on the
  // headline (profiles/r3_sock_buf_ab.md): gateway path 13.77k vs 13.32k req/s mean over 4
  // interleaved pairs, 11 % less sys time per request.  Remote peers keep TCP autotuning (a fixed
  // SO_RCVBUF turns it off).  The kernel caps the value at net.core.[rw]mem_max: the size it
  // actually granted is read back and reported (sock_buf_effective, worker /health "io").
  static const int buf = [] {
    const char* e = std::getenv("DIE_SOCK_BUF_KB");
    return (e && *e ? std::atoi(e) : 4096) * 1024;
  }();
  if (buf > 0 && loopback_peer) {
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
    if (g_sock_buf_effective.load(std::memory_order_relaxed) < 0) {
      int got = 0;
      socklen_t len = sizeof got;
      if (getsockopt(fd, SOL_SOCKET, SO_RCVBUF, &got, &len) == 0) g_sock_buf_effective.store(got, std::memory_order_relaxed);
    }
  }
}

// Parse a header block [b, e) (request line / status line excluded) into lower-cased pairs.
void parse_headers(std::string_view block, std::vector<std::pair<std::string, std::string>>& out) {
  size_t pos = 0;
  while (pos < block.size()) {
    size_t eol = block.find("\r\n", pos);
    if (eol == std::string_view::npos) eol = block.size();
    std::string_view line = block.substr(pos, eol - pos);
    pos = eol + 2;
    if (line.empty()) continue;
    size_t colon = line.find(':');
    if (colon == std::string_view::npos) continue;
    out.emplace_back(to_lower(trim(line.substr(0, colon))), std::string(trim(line.substr(colon + 1))));
  }
}

// Decode a complete chunked body starting at `data`; returns bytes consumed, 0 if incomplete,
// -1 if malformed, -2 if the decoded body would exceed `max_out` bytes.  Chunk sizes are checked
// without overflow (a size near 2^64 must not wrap the bounds test).
long dechunk(std::string_view data, std::string& out, size_t max_out) {
  size_t pos = 0;
  while (true) {
    size_t eol = data.find("\r\n", pos);
    if (eol == std::string_view::npos) return 0;
    std::string_view szs = data.substr(pos, eol - pos);
    size_t semi = szs.find(';');
    if (semi != std::string_view::npos) szs = szs.substr(0, semi);
    char* endp = nullptr;
    std::string tmp(trim(szs));
    if (tmp.empty() || tmp.size() > 16) return -1;
    unsigned long long sz = std::strtoull(tmp.c_str(), &endp, 16);
    if (endp && *endp) return -1;
    pos = eol + 2;
    if (sz == 0) {
      // trailers until blank line
      while (true) {
        size_t e2 = data.find("\r\n", pos);
        if (e2 == std::string_view::npos) return 0;
        bool blank = e2 == pos;
        pos = e2 + 2;
        if (blank) return static_cast<long>(pos);
      }
    }
    if (sz > max_out || out.size() > max_out - sz) return -2;
    if (pos > data.size() || data.size() - pos < 2 || sz > data.size() - pos - 2) return 0;
    out.append(data.data() + pos, static_cast<size_t>(sz));
    pos += sz + 2;
  }
}

}  // namespace http_detail

using namespace http_detail;

std::string_view HttpRequest::header(std::string_view name) const {
  for (auto& kv : headers)
    if (kv.first == name) return kv.second;
  return {};
}

const char* http_status_text(int s) {
  switch (s) {
    case 100: return "Continue";
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Unknown";
  }
}

// ------------------------------------------------------------------------------------------------
// Server
// ------------------------------------------------------------------------------------------------

struct Mailbox {
  struct Item {
    uint64_t conn_id;
    bool keep_alive;
    HttpResponse resp;
    std::function<HttpResponse()> build;
  };
  std::mutex mu;
  std::vector<Item> items;
  int efd = -1;
  bool open = true;
  std::atomic<bool> pending{false};  // items waiting: the reactor also checks between events

  void post(Item it) {
    // the wake-up write stays under the lock: HttpServer::stop() closes efd under it, so a
    // completion posted while the server stops never writes to a closed (or reused) descriptor
    std::lock_guard<std::mutex> g(mu);
    if (!open) return;
    items.push_back(std::move(it));
    pending.store(true, std::memory_order_release);
    uint64_t one = 1;
    ssize_t r = ::write(efd, &one, sizeof one);
    (void)r;
  }
};

struct Responder::State {
  std::shared_ptr<Mailbox> box;
  uint64_t conn_id = 0;
  bool keep_alive = true;
  std::atomic<bool> done{false};
};

void Responder::send(HttpResponse resp) const {
  if (!state_ || state_->done.exchange(true)) return;
  state_->box->post(Mailbox::Item{state_->conn_id, state_->keep_alive, std::move(resp), nullptr});
}

void Responder::defer(std::function<HttpResponse()> build) const {
  if (!state_ || state_->done.exchange(true)) return;
  state_->box->post(Mailbox::Item{state_->conn_id, state_->keep_alive, HttpResponse{}, std::move(build)});
}

namespace {
bool is_loopback(const sockaddr_storage& a) {
  if (a.ss_family == AF_INET)
    return (ntohl(reinterpret_cast<const sockaddr_in&>(a).sin_addr.s_addr) >> 24) == 127;
  if (a.ss_family == AF_INET6) {
    const in6_addr& v6 = reinterpret_cast<const sockaddr_in6&>(a).sin6_addr;
    if (IN6_IS_ADDR_LOOPBACK(&v6)) return true;
    return IN6_IS_ADDR_V4MAPPED(&v6) && v6.s6_addr[12] == 127;
  }
  return a.ss_family == AF_UNIX;
}
}  // namespace

struct HttpServer::Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;          // header bytes / pipelined leftovers
  bool headers_done = false;
  bool chunked = false;
  size_t body_len = 0;     // content-length
  size_t body_have = 0;
  BodyBuffer ext;          // allocator memory the current body is received into (if any)
  char* body_dst() { return ext.data ? ext.data : &req.body[0]; }
  HttpRequest req;
  bool busy = false;       // a request is being handled
  bool peer_eof = false;
  bool close_after = false;
  bool loopback = false;   // peer address is 127.0.0.0/8 or ::1
  // output
  std::string out_head, out_body;
  size_t out_off = 0;      // offset across head+body
  bool want_out = false;
};

struct HttpServer::Reactor {
  int ep = -1;
  std::shared_ptr<Mailbox> box = std::make_shared<Mailbox>();
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
  uint64_t next_id = 1;
};

HttpServer::HttpServer() = default;

HttpServer::~HttpServer() { stop(); }

void HttpServer::route(const std::string& method, const std::string& path, Handler h) {
  routes_.push_back({{method, path}, std::move(h)});
}

int HttpServer::start(const std::string& host, int port, int threads, bool reuse_port) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) return -1;
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (reuse_port) setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (host.empty() || host == "0.0.0.0") {
    addr.sin_addr.s_addr = INADDR_ANY;
  } else if (host == "localhost") {
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  } else if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    return -1;
  }
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0 || ::listen(listen_fd_, 4096) != 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    return -1;
  }
  socklen_t len = sizeof addr;
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  set_nonblock(listen_fd_);

  if (threads <= 0) threads = std::min(32, available_cpus());
  running_ = true;
  for (int i = 0; i < threads; ++i) {
    auto r = std::make_unique<Reactor>();
    r->ep = epoll_create1(EPOLL_CLOEXEC);
    r->box->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLEXCLUSIVE;
    ev.data.u64 = 0;  // listen
    epoll_ctl(r->ep, EPOLL_CTL_ADD, listen_fd_, &ev);
    ev.events = EPOLLIN;
    ev.data.u64 = 1;  // mailbox
    epoll_ctl(r->ep, EPOLL_CTL_ADD, r->box->efd, &ev);
    reactors_.push_back(std::move(r));
  }
  for (auto& r : reactors_) threads_.emplace_back([this, rp = r.get()] {
    pthread_setname_np(pthread_self(), "die-http");
    reactor_loop(rp);
  });
  return port_;
}

void HttpServer::wait() {
  std::unique_lock<std::mutex> lk(wait_mu_);
  wait_cv_.wait(lk, [&] { return !running_.load(); });
}

void HttpServer::stop() {
  std::lock_guard<std::mutex> stop_guard(stop_mu_);
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(wait_mu_);
  }
  wait_cv_.notify_all();
  for (auto& r : reactors_) {
    uint64_t one = 1;
    ssize_t w = ::write(r->box->efd, &one, sizeof one);
    (void)w;
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (auto& r : reactors_) {
    {
      std::lock_guard<std::mutex> g(r->box->mu);
      r->box->open = false;
      r->box->items.clear();
      ::close(r->box->efd);  // under the lock: see Mailbox::post
      r->box->efd = -1;
    }
    for (auto& kv : r->conns) ::close(kv.second->fd);
    r->conns.clear();
    ::close(r->ep);
  }
  reactors_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
}

namespace {

void update_events(int ep, int fd, uint64_t id, bool want_out) {
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | (want_out ? EPOLLOUT : 0);
  ev.data.u64 = id;
  epoll_ctl(ep, EPOLL_CTL_MOD, fd, &ev);
}

}  // namespace

void HttpServer::reactor_loop(Reactor* r) {
  std::vector<epoll_event> events(256);
  std::vector<Mailbox::Item> drained;

  auto close_conn = [&](Conn* c) {
    epoll_ctl(r->ep, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
    r->conns.erase(c->id);
  };

  // Returns false if the connection was closed.
  std::function<bool(Conn*)> try_parse;

  auto flush = [&](Conn* c) -> bool {
    while (true) {
      const size_t hs = c->out_head.size(), bs = c->out_body.size();
      const size_t total = hs + bs;
      if (c->out_off >= total) break;
      iovec iov[2];
      int n = 0;
      if (c->out_off < hs) {
        iov[n++] = {const_cast<char*>(c->out_head.data()) + c->out_off, hs - c->out_off};
        if (bs) iov[n++] = {const_cast<char*>(c->out_body.data()), bs};
      } else {
        iov[n++] = {const_cast<char*>(c->out_body.data()) + (c->out_off - hs), total - c->out_off};
      }
      ssize_t w = ::writev(c->fd, iov, n);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          if (!c->want_out) {
            c->want_out = true;
            update_events(r->ep, c->fd, c->id, true);
          }
          return true;
        }
        close_conn(c);
        return false;
      }
      c->out_off += static_cast<size_t>(w);
    }
    // fully written
    if (c->want_out) {
      c->want_out = false;
      update_events(r->ep, c->fd, c->id, false);
    }
    c->out_head.clear();
    c->out_body.clear();
    c->out_off = 0;
    if (c->busy) {
      c->busy = false;
      served_.fetch_add(1, std::memory_order_relaxed);
      if (c->close_after || c->peer_eof) {
        close_conn(c);
        return false;
      }
      return try_parse(c);
    }
    return true;
  };

  auto queue_response = [&](Conn* c, HttpResponse&& resp, bool keep_alive) -> bool {
    bool close = !keep_alive || resp.close || !running_.load(std::memory_order_relaxed);
    c->close_after = c->close_after || close;
    std::string& h = c->out_head;
    h.clear();
    h.reserve(160);
    h += "HTTP/1.1 ";
    h += std::to_string(resp.status);
    h += ' ';
    h += http_status_text(resp.status);
    h += "\r\nContent-Type: ";
    h += resp.content_type.empty() ? "text/plain" : resp.content_type;
    h += "\r\nContent-Length: ";
    h += std::to_string(resp.body.size());
    for (auto& kv : resp.headers) {
      h += "\r\n";
      h += kv.first;
      h += ": ";
      h += kv.second;
    }
    h += c->close_after ? "\r\nConnection: close\r\n\r\n" : "\r\nConnection: keep-alive\r\n\r\n";
    c->out_body = std::move(resp.body);
    c->out_off = 0;
    return flush(c);
  };

  auto respond_now = [&](Conn* c, int status, const std::string& msg) -> bool {
    HttpResponse resp;
    resp.status = status;
    Json j = Json::object();
    j["error"] = msg;
    resp.body = j.dump();
    c->busy = true;
    c->close_after = true;
    return queue_response(c, std::move(resp), false);
  };

  try_parse = [&](Conn* c) -> bool {
    while (!c->busy) {
      if (!c->headers_done) {
        size_t he = c->in.find("\r\n\r\n");
        if (he == std::string::npos) {
          if (c->in.size() > (64u << 10)) return respond_now(c, 400, "header too large");
          if (c->peer_eof) {
            close_conn(c);
            return false;
          }
          return true;
        }
        std::string_view all(c->in.data(), he);
        size_t le = all.find("\r\n");
        std::string_view line = all.substr(0, le == std::string_view::npos ? all.size() : le);
        size_t s1 = line.find(' ');
        size_t s2 = s1 == std::string_view::npos ? s1 : line.find(' ', s1 + 1);
        if (s1 == std::string_view::npos || s2 == std::string_view::npos) return respond_now(c, 400, "bad request line");
        c->req = HttpRequest{};
        c->req.method = std::string(line.substr(0, s1));
        std::string_view target = line.substr(s1 + 1, s2 - s1 - 1);
        std::string_view version = line.substr(s2 + 1);
        size_t q = target.find('?');
        c->req.path = std::string(target.substr(0, q));
        if (q != std::string_view::npos) c->req.query = std::string(target.substr(q + 1));
        if (le != std::string_view::npos) parse_headers(all.substr(le + 2), c->req.headers);
        std::string_view conn_h = c->req.header("connection");
        bool http10 = version == "HTTP/1.0";
        c->req.keep_alive = http10 ? iequals(conn_h, "keep-alive") : !iequals(conn_h, "close");
        std::string_view te = c->req.header("transfer-encoding");
        c->chunked = !te.empty() && te.find("chunked") != std::string_view::npos;
        std::string_view cl = c->req.header("content-length");
        c->body_len = cl.empty() ? 0 : std::strtoull(std::string(cl).c_str(), nullptr, 10);
        if (c->body_len > max_body_bytes) return respond_now(c, 413, "payload too large");
        if (iequals(c->req.header("expect"), "100-continue")) {
          static const char kContinue[] = "HTTP/1.1 100 Continue\r\n\r\n";
          ssize_t w = ::send(c->fd, kContinue, sizeof kContinue - 1, MSG_NOSIGNAL);
          (void)w;
        }
        c->in.erase(0, he + 4);
        c->headers_done = true;
        c->req.t_headers = std::chrono::steady_clock::now();
        c->req.peer_loopback = c->loopback;
        c->ext = BodyBuffer{};
        if (!c->chunked && body_alloc_ && c->body_len >= body_alloc_min_ && c->body_len > 0) {
          c->ext = body_alloc_(c->body_len + 64);
          if (c->ext.data && c->ext.capacity < c->body_len + 64) c->ext = BodyBuffer{};
        }
        if (!c->chunked) {
          if (!c->ext.data) {
            c->req.body.reserve(c->body_len + 64);
            c->req.body.resize(c->body_len);
          }
          size_t take = std::min(c->body_len, c->in.size());
          if (take) std::memcpy(c->body_dst(), c->in.data(), take);
          c->in.erase(0, take);
          c->body_have = take;
        }
      }
      if (c->chunked) {
        std::string decoded;
        long used = dechunk(c->in, decoded, max_body_bytes);
        if (used == -2) return respond_now(c, 413, "payload too large");
        if (used < 0) return respond_now(c, 400, "bad chunked body");
        if (used == 0 && c->in.size() > max_body_bytes + (64u << 10)) return respond_now(c, 413, "payload too large");
        if (used == 0) {
          if (c->peer_eof) {
            close_conn(c);
            return false;
          }
          return true;
        }
        c->in.erase(0, static_cast<size_t>(used));
        decoded.reserve(decoded.size() + 64);
        c->req.body = std::move(decoded);
      } else if (c->body_have < c->body_len) {
        if (c->peer_eof) {
          close_conn(c);
          return false;
        }
        return true;
      }
      // complete request
      if (c->ext.data) {
        std::memset(c->ext.data + c->body_len, 0, 64);  // parser slack
        c->req.ext_body = c->ext.data;
        c->req.ext_len = c->body_len;
        c->req.ext_owner = std::move(c->ext.owner);
        c->ext = BodyBuffer{};
      }
      c->headers_done = false;
      c->busy = true;
      dispatch(r, c);
      // dispatch may have completed synchronously through the mailbox; nothing else to do
      return r->conns.count(c->id) != 0;
    }
    return true;
  };

  auto on_readable = [&](Conn* c) {
    while (true) {
      ssize_t n;
      if (c->headers_done && !c->chunked && c->body_have < c->body_len) {
        n = ::recv(c->fd, c->body_dst() + c->body_have, c->body_len - c->body_have, 0);
        if (n > 0) {
          c->body_have += static_cast<size_t>(n);
          continue;
        }
      } else {
        size_t old = c->in.size();
        c->in.resize(old + 65536);
        n = ::recv(c->fd, &c->in[old], 65536, 0);
        c->in.resize(old + (n > 0 ? static_cast<size_t>(n) : 0));
        if (n > 0) {
          if (!c->busy && !c->headers_done && c->in.find("\r\n\r\n") != std::string::npos) {
            if (!try_parse(c)) return;
          }
          continue;
        }
      }
      if (n == 0) {
        c->peer_eof = true;
        break;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      close_conn(c);
      return;
    }
    if (!c->busy) {
      if (!try_parse(c)) return;
    }
    if (c->peer_eof && !c->busy && r->conns.count(c->id)) close_conn(c);
  };

  auto drain_mailbox = [&] {
    {
      std::lock_guard<std::mutex> g(r->box->mu);
      r->box->pending.store(false, std::memory_order_relaxed);
      drained.swap(r->box->items);
    }
    for (auto& it : drained) {
      auto f = r->conns.find(it.conn_id);
      if (f == r->conns.end()) continue;
      HttpResponse resp;
      if (it.build) {
        try {
          resp = it.build();
        } catch (const std::exception& e) {
          resp = HttpResponse{};
          resp.status = 500;
          Json j = Json::object();
          j["error"] = e.what();
          resp.body = j.dump();
        }
      } else {
        resp = std::move(it.resp);
      }
      queue_response(f->second.get(), std::move(resp), it.keep_alive);
    }
    drained.clear();
  };

  while (running_.load(std::memory_order_relaxed)) {
    int n = epoll_wait(r->ep, events.data(), static_cast<int>(events.size()), 200);
    if (n < 0) {
      if (errno == EINTR) continue;
      break;
    }
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = events[i].data.u64;
      if (tag == 0) {
        while (true) {
          sockaddr_storage peer{};
          socklen_t plen = sizeof peer;
          int fd = ::accept4(listen_fd_, reinterpret_cast<sockaddr*>(&peer), &plen, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (fd < 0) break;
          set_nodelay(fd, is_loopback(peer));
          auto c = std::make_unique<Conn>();
          c->fd = fd;
          c->loopback = is_loopback(peer);
          c->id = (r->next_id++) + 16;  // 0/1 reserved
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.u64 = c->id;
          epoll_ctl(r->ep, EPOLL_CTL_ADD, fd, &ev);
          r->conns.emplace(c->id, std::move(c));
        }
      } else if (tag == 1) {
        uint64_t v;
        ssize_t rd = ::read(r->box->efd, &v, sizeof v);
        (void)rd;
        drain_mailbox();
      } else {
        auto f = r->conns.find(tag);
        if (f == r->conns.end()) continue;
        Conn* c = f->second.get();
        const uint32_t ev = events[i].events;
        if (ev & EPOLLOUT) {
          if (!flush(c)) continue;
        }
        if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          // A malformed or hostile request must cost its connection, never the process.
          try {
            on_readable(c);
          } catch (const std::exception&) {
            if (r->conns.count(tag)) close_conn(c);
          }
        }
        // Completed responses are written between connection events, not after the whole batch of
        // events: a reactor busy receiving ~1 MB request bodies must not hold finished answers back
        // (head-of-line blocking of the respond stage).
        if (r->box->pending.load(std::memory_order_acquire)) drain_mailbox();
      }
    }
  }
}

void HttpServer::dispatch(Reactor* r, Conn* c) {
  Responder res;
  res.state_ = std::make_shared<Responder::State>();
  res.state_->box = r->box;
  res.state_->conn_id = c->id;
  res.state_->keep_alive = c->req.keep_alive;
  const Handler* h = nullptr;
  bool path_known = false;
  for (auto& rt : routes_) {
    if (rt.first.second == c->req.path) {
      path_known = true;
      if (rt.first.first == c->req.method) {
        h = &rt.second;
        break;
      }
    }
  }
  if (!h) {
    HttpResponse resp;
    resp.status = path_known ? 405 : 404;
    resp.content_type = "text/plain";
    resp.body = path_known ? "Method Not Allowed" : "Not Found";
    res.send(std::move(resp));
    return;
  }
  try {
    (*h)(c->req, res);
  } catch (const std::exception& e) {
    HttpResponse resp;
    resp.status = 500;
    Json j = Json::object();
    j["error"] = e.what();
    resp.body = j.dump();
    res.send(std::move(resp));
  }
}

// ------------------------------------------------------------------------------------------------
// Client
// ------------------------------------------------------------------------------------------------

std::pair<std::string, int> parse_host_port(const std::string& url) {
  std::string s = url;
  size_t proto = s.find("://");
  if (proto != std::string::npos) s = s.substr(proto + 3);
  size_t colon = s.find_last_of(':');
  if (colon == std::string::npos) {
    size_t slash = s.find('/');
    return {s.substr(0, slash), 8080};
  }
  std::string host = s.substr(0, colon);
  std::string port_str = s.substr(colon + 1);
  size_t slash = port_str.find('/');
  if (slash != std::string::npos) port_str = port_str.substr(0, slash);
  int port = 8080;
  try {
    port = std::stoi(port_str);
  } catch (...) {
    port = 8080;
  }
  return {host, port};
}

HttpClient::HttpClient(std::string host, int port, std::chrono::milliseconds ct, std::chrono::milliseconds rt,
                       size_t max_idle)
    : host_(std::move(host)), port_(port), connect_timeout_(ct), read_timeout_(rt), max_idle_(max_idle) {}

HttpClient::~HttpClient() {
  std::lock_guard<std::mutex> g(mu_);
  for (int fd : idle_) ::close(fd);
  idle_.clear();
}

int HttpClient::connect_new(std::string* error) {
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string h = host_ == "localhost" ? "127.0.0.1" : host_;
  if (getaddrinfo(h.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res) {
    if (error) *error = "cannot resolve host " + host_;
    return -1;
  }
  int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    freeaddrinfo(res);
    if (error) *error = "socket() failed";
    return -1;
  }
  set_nonblock(fd);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    ::close(fd);
    if (error) *error = std::string("connect failed: ") + strerror(errno);
    return -1;
  }
  if (rc != 0) {
    pollfd p{fd, POLLOUT, 0};
    int pr = ::poll(&p, 1, static_cast<int>(connect_timeout_.count()));
    int err = 0;
    socklen_t len = sizeof err;
    if (pr <= 0 || getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len) != 0 || err != 0) {
      ::close(fd);
      if (error) *error = pr == 0 ? "connection timeout" : std::string("connect failed: ") + strerror(err ? err : errno);
      return -1;
    }
  }
  sockaddr_storage peer{};
  socklen_t plen = sizeof peer;
  set_nodelay(fd, getpeername(fd, reinterpret_cast<sockaddr*>(&peer), &plen) == 0 && is_loopback(peer));
  return fd;
}

void HttpClient::release(int fd) {
  std::lock_guard<std::mutex> g(mu_);
  if (idle_.size() >= max_idle_) {
    ::close(fd);
    return;
  }
  idle_.push_back(fd);
}

namespace {

// Wait for fd readiness with a deadline; returns false on timeout/error.
bool wait_fd(int fd, short events, std::chrono::steady_clock::time_point deadline) {
  while (true) {
    auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() <= 0) return false;
    pollfd p{fd, events, 0};
    int r = ::poll(&p, 1, static_cast<int>(left.count()));
    if (r > 0) return true;
    if (r < 0 && errno == EINTR) continue;
    return false;
  }
}

}  // namespace

std::optional<HttpResponse> HttpClient::request(const std::string& method, const std::string& path,
                                                std::string_view body, const std::string& content_type,
                                                std::string* error) {
  std::string head;
  head.reserve(192);
  head += method;
  head += ' ';
  head += path;
  head += " HTTP/1.1\r\nHost: ";
  head += host_;
  head += ':';
  head += std::to_string(port_);
  if (!body.empty() || method == "POST") {
    head += "\r\nContent-Type: ";
    head += content_type;
    head += "\r\nContent-Length: ";
    head += std::to_string(body.size());
  }
  head += "\r\nConnection: keep-alive\r\n\r\n";

  for (int attempt = 0; attempt < 2; ++attempt) {
    int fd = -1;
    bool reused = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!idle_.empty()) {
        fd = idle_.back();
        idle_.pop_back();
        reused = true;
      }
    }
    if (fd < 0) fd = connect_new(error);
    if (fd < 0) return std::nullopt;
    auto deadline = std::chrono::steady_clock::now() + read_timeout_;
    // send
    size_t off = 0, total = head.size() + body.size();
    bool ok = true;
    while (off < total) {
      iovec iov[2];
      int n = 0;
      if (off < head.size()) {
        iov[n++] = {const_cast<char*>(head.data()) + off, head.size() - off};
        if (!body.empty()) iov[n++] = {const_cast<char*>(body.data()), body.size()};
      } else {
        iov[n++] = {const_cast<char*>(body.data()) + (off - head.size()), total - off};
      }
      msghdr mh{};
      mh.msg_iov = iov;
      mh.msg_iovlen = n;
      ssize_t w = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if ((errno == EAGAIN || errno == EWOULDBLOCK) && wait_fd(fd, POLLOUT, deadline)) continue;
        ok = false;
        if (error) *error = errno == EAGAIN ? "write timeout" : std::string("send failed: ") + strerror(errno);
        break;
      }
      off += static_cast<size_t>(w);
    }
    if (!ok) {
      ::close(fd);
      if (reused) continue;
      return std::nullopt;
    }
    // receive
    std::string buf;
    buf.reserve(16384);
    size_t header_end = std::string::npos;
    HttpResponse resp;
    std::vector<std::pair<std::string, std::string>> headers;
    size_t content_len = 0;
    bool has_len = false, chunked = false, server_close = false;
    bool got_any = false;
    std::string fail;
    while (true) {
      if (header_end == std::string::npos) {
        header_end = buf.find("\r\n\r\n");
        if (header_end != std::string::npos) {
          std::string_view all(buf.data(), header_end);
          size_t le = all.find("\r\n");
          std::string_view status_line = all.substr(0, le);
          size_t sp = status_line.find(' ');
          if (sp == std::string_view::npos) {
            fail = "malformed status line";
            break;
          }
          resp.status = std::atoi(std::string(status_line.substr(sp + 1, 3)).c_str());
          if (le != std::string_view::npos) parse_headers(all.substr(le + 2), headers);
          if (resp.status == 100) {  // skip interim response
            buf.erase(0, header_end + 4);
            header_end = std::string::npos;
            headers.clear();
            continue;
          }
          for (auto& kv : headers) {
            if (kv.first == "content-length") {
              content_len = std::strtoull(kv.second.c_str(), nullptr, 10);
              has_len = true;
            } else if (kv.first == "transfer-encoding" && kv.second.find("chunked") != std::string::npos) {
              chunked = true;
            } else if (kv.first == "connection" && iequals(kv.second, "close")) {
              server_close = true;
            } else if (kv.first == "content-type") {
              resp.content_type = kv.second;
            }
          }
          resp.headers = headers;
          if (has_len) buf.reserve(header_end + 4 + content_len + 64);
        }
      }
      if (header_end != std::string::npos) {
        const size_t body_start = header_end + 4;
        if (has_len && !chunked && buf.size() >= body_start + content_len) {
          resp.body.assign(buf.data() + body_start, content_len);
          break;
        }
        if (chunked) {
          std::string decoded;
          long used = dechunk(std::string_view(buf).substr(body_start), decoded, size_t{1} << 31);
          if (used < 0) {
            fail = "bad chunked response";
            break;
          }
          if (used > 0) {
            resp.body = std::move(decoded);
            break;
          }
        }
      }
      if (!wait_fd(fd, POLLIN, deadline)) {
        fail = "read timeout";
        break;
      }
      size_t old = buf.size();
      size_t want = 65536;
      if (header_end != std::string::npos && has_len && !chunked) {
        size_t need = header_end + 4 + content_len - old;
        want = std::max<size_t>(want, need);
      }
      buf.resize(old + want);
      ssize_t n = ::recv(fd, &buf[old], want, 0);
      if (n > 0) {
        buf.resize(old + static_cast<size_t>(n));
        got_any = true;
        continue;
      }
      buf.resize(old);
      if (n < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      if (n == 0 && header_end != std::string::npos && !has_len && !chunked) {
        resp.body.assign(buf.data() + header_end + 4, buf.size() - header_end - 4);
        server_close = true;
        break;
      }
      fail = n == 0 ? "connection closed by peer" : std::string("recv failed: ") + strerror(errno);
      break;
    }
    if (!fail.empty()) {
      ::close(fd);
      if (reused && !got_any && fail != "read timeout") continue;  // stale keep-alive socket
      if (error) *error = fail;
      return std::nullopt;
    }
    if (server_close) {
      ::close(fd);
    } else {
      release(fd);
    }
    return resp;
  }
  if (error && error->empty()) *error = "request failed";
  return std::nullopt;
}

}  // namespace die
