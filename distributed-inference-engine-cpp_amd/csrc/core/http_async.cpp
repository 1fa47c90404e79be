#include <pthread.h>
#include "http_async.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cstring>
#include <deque>
#include <mutex>
#include <unordered_map>

#include "http_util.h"

namespace die {

using namespace http_detail;
using Clock = std::chrono::steady_clock;

struct AsyncHttpClient::Job {
  int upstream = 0;
  std::string head;  // request line + headers
  BodyRef body;
  Callback cb;
  bool retried = false;  // already re-sent once after a stale keep-alive connection
};

struct AsyncHttpClient::Conn {
  enum State { CONNECTING, WRITING, READING, IDLE } state = CONNECTING;
  int fd = -1;
  uint64_t id = 0;
  int upstream = 0;
  bool reused = false;
  bool got_any = false;
  std::unique_ptr<Job> job;
  size_t out_off = 0;
  std::string in;
  size_t header_end = std::string::npos;
  size_t content_len = 0;
  bool has_len = false, chunked = false, server_close = false;
  HttpResponse resp;
  Clock::time_point deadline{};
  bool want_out = false;
};

struct AsyncHttpClient::Loop {
  int ep = -1, efd = -1;
  std::mutex mu;
  std::deque<std::unique_ptr<Job>> inbox;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
  std::vector<std::vector<uint64_t>> idle;  // per upstream
  uint64_t next_id = 16;
};

AsyncHttpClient::AsyncHttpClient(Options opt) : opt_(opt) {
  const int n = std::max(1, opt_.threads);
  for (int i = 0; i < n; ++i) {
    auto L = std::make_unique<Loop>();
    L->ep = epoll_create1(EPOLL_CLOEXEC);
    L->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 1;
    epoll_ctl(L->ep, EPOLL_CTL_ADD, L->efd, &ev);
    loops_.push_back(std::move(L));
  }
  for (auto& L : loops_) threads_.emplace_back([this, p = L.get()] {
    pthread_setname_np(pthread_self(), "die-fwd");
    run(p);
  });
}

AsyncHttpClient::~AsyncHttpClient() { stop(); }

int AsyncHttpClient::add_upstream(const std::string& host, int port) {
  Upstream u;
  u.host = host == "localhost" ? "127.0.0.1" : host;
  u.port = port;
  u.host_header = host + ":" + std::to_string(port);
  ups_.push_back(u);
  for (auto& L : loops_) {
    std::lock_guard<std::mutex> g(L->mu);
    L->idle.resize(ups_.size());
  }
  return static_cast<int>(ups_.size()) - 1;
}

void AsyncHttpClient::post(int upstream, const std::string& path, BodyRef body, const std::string& content_type,
                           const std::string& extra_headers, Callback cb) {
  if (upstream < 0 || upstream >= static_cast<int>(ups_.size()) || !running_.load()) {
    cb(std::nullopt, "client stopped or unknown upstream");
    return;
  }
  auto j = std::make_unique<Job>();
  j->upstream = upstream;
  const Upstream& u = ups_[upstream];
  j->head.reserve(160);
  j->head += "POST ";
  j->head += path;
  j->head += " HTTP/1.1\r\nHost: ";
  j->head += u.host_header;
  j->head += "\r\nContent-Type: ";
  j->head += content_type;
  j->head += "\r\nContent-Length: ";
  j->head += std::to_string(body.size);
  j->head += "\r\n";
  j->head += extra_headers;
  j->head += "Connection: keep-alive\r\n\r\n";
  j->body = std::move(body);
  j->cb = std::move(cb);
  in_flight_.fetch_add(1, std::memory_order_relaxed);
  Loop* L = loops_[rr_.fetch_add(1, std::memory_order_relaxed) % loops_.size()].get();
  {
    std::lock_guard<std::mutex> g(L->mu);
    L->inbox.push_back(std::move(j));
  }
  uint64_t one = 1;
  ssize_t w = ::write(L->efd, &one, sizeof one);
  (void)w;
}

void AsyncHttpClient::stop() {
  if (!running_.exchange(false)) return;
  for (auto& L : loops_) {
    uint64_t one = 1;
    ssize_t w = ::write(L->efd, &one, sizeof one);
    (void)w;
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (auto& L : loops_) {
    for (auto& kv : L->conns) ::close(kv.second->fd);
    L->conns.clear();
    ::close(L->ep);
    ::close(L->efd);
  }
}

void AsyncHttpClient::run(Loop* L) {
  std::vector<epoll_event> events(256);
  std::deque<std::unique_ptr<Job>> jobs;

  auto set_events = [&](Conn* c, bool out) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | (out ? EPOLLOUT : 0);
    ev.data.u64 = c->id;
    epoll_ctl(L->ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = out;
  };
  auto finish = [&](std::unique_ptr<Job> j, std::optional<HttpResponse> r, const std::string& err) {
    in_flight_.fetch_sub(1, std::memory_order_relaxed);
    try {
      j->cb(std::move(r), err);
    } catch (...) {
    }
  };
  auto close_conn = [&](Conn* c) {
    epoll_ctl(L->ep, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
    if (c->state == Conn::IDLE) {
      auto& v = L->idle[c->upstream];
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == c->id) {
          v[i] = v.back();
          v.pop_back();
          break;
        }
    }
    L->conns.erase(c->id);
  };
  std::function<void(std::unique_ptr<Job>)> start;
  // Transport failure of the request on `c`: a stale keep-alive socket (nothing received yet) is
  // retried once on a fresh connection, anything else fails the job.
  auto fail = [&](Conn* c, const std::string& err) {
    std::unique_ptr<Job> j = std::move(c->job);
    const bool retry = c->reused && !c->got_any && err != "read timeout" && j && !j->retried;
    close_conn(c);
    if (!j) return;
    if (retry) {
      j->retried = true;
      start(std::move(j));
      return;
    }
    finish(std::move(j), std::nullopt, err);
  };
  auto begin_write = [&](Conn* c) {
    c->state = Conn::WRITING;
    c->out_off = 0;
    c->in.clear();
    c->header_end = std::string::npos;
    c->content_len = 0;
    c->has_len = c->chunked = c->server_close = c->got_any = false;
    c->resp = HttpResponse{};
    c->deadline = Clock::now() + opt_.read_timeout;
  };
  // Write as much of the request as the socket takes; returns false if the connection failed.
  auto pump_write = [&](Conn* c) -> bool {
    const std::string& h = c->job->head;
    const char* bd = c->job->body.data;
    const size_t bs = bd ? c->job->body.size : 0, total = h.size() + bs;
    while (c->out_off < total) {
      iovec iov[2];
      int n = 0;
      if (c->out_off < h.size()) {
        iov[n++] = {const_cast<char*>(h.data()) + c->out_off, h.size() - c->out_off};
        if (bs) iov[n++] = {const_cast<char*>(bd), bs};
      } else {
        iov[n++] = {const_cast<char*>(bd) + (c->out_off - h.size()), total - c->out_off};
      }
      msghdr mh{};
      mh.msg_iov = iov;
      mh.msg_iovlen = n;
      ssize_t w = ::sendmsg(c->fd, &mh, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          if (!c->want_out) set_events(c, true);
          return true;
        }
        fail(c, std::string("send failed: ") + strerror(errno));
        return false;
      }
      c->out_off += static_cast<size_t>(w);
    }
    c->state = Conn::READING;
    if (c->want_out) set_events(c, false);
    return true;
  };
  // Parse what has arrived; returns true when the response is complete (then handled).
  auto try_complete = [&](Conn* c, bool eof) -> bool {
    if (c->header_end == std::string::npos) {
      c->header_end = c->in.find("\r\n\r\n");
      if (c->header_end == std::string::npos) return false;
      std::string_view all(c->in.data(), c->header_end);
      size_t le = all.find("\r\n");
      std::string_view sl = all.substr(0, le);
      size_t sp = sl.find(' ');
      if (sp == std::string_view::npos || sl.size() < sp + 4) {
        fail(c, "malformed status line");
        return true;
      }
      c->resp.status = std::atoi(std::string(sl.substr(sp + 1, 3)).c_str());
      if (le != std::string_view::npos) parse_headers(all.substr(le + 2), c->resp.headers);
      if (c->resp.status == 100) {
        c->in.erase(0, c->header_end + 4);
        c->header_end = std::string::npos;
        c->resp.headers.clear();
        return false;
      }
      for (auto& kv : c->resp.headers) {
        if (kv.first == "content-length") {
          c->content_len = std::strtoull(kv.second.c_str(), nullptr, 10);
          c->has_len = true;
        } else if (kv.first == "transfer-encoding" && kv.second.find("chunked") != std::string::npos) {
          c->chunked = true;
        } else if (kv.first == "connection" && iequals(kv.second, "close")) {
          c->server_close = true;
        } else if (kv.first == "content-type") {
          c->resp.content_type = kv.second;
        }
      }
    }
    const size_t bstart = c->header_end + 4;
    bool done = false;
    if (c->chunked) {
      std::string dec;
      long used = dechunk(std::string_view(c->in).substr(bstart), dec, size_t{1} << 31);
      if (used < 0) {
        fail(c, "bad chunked response");
        return true;
      }
      if (used > 0) {
        c->resp.body = std::move(dec);
        done = true;
      }
    } else if (c->has_len) {
      if (c->in.size() >= bstart + c->content_len) {
        c->resp.body.assign(c->in.data() + bstart, c->content_len);
        done = true;
      }
    } else if (eof) {
      c->resp.body.assign(c->in.data() + bstart, c->in.size() - bstart);
      c->server_close = true;
      done = true;
    }
    if (!done) return false;
    std::unique_ptr<Job> j = std::move(c->job);
    HttpResponse r = std::move(c->resp);
    if (c->server_close || eof || !running_.load()) {
      close_conn(c);
    } else {
      auto& idle = L->idle[c->upstream];
      if (idle.size() >= opt_.max_idle_per_upstream) {
        close_conn(c);
      } else {
        c->state = Conn::IDLE;
        c->in.clear();
        idle.push_back(c->id);
      }
    }
    finish(std::move(j), std::move(r), "");
    return true;
  };

  start = [&](std::unique_ptr<Job> j) {
    const int u = j->upstream;
    auto& idle = L->idle[u];
    while (!idle.empty()) {
      const uint64_t id = idle.back();
      idle.pop_back();
      auto f = L->conns.find(id);
      if (f == L->conns.end()) continue;
      Conn* c = f->second.get();
      c->reused = true;
      c->job = std::move(j);
      begin_write(c);
      pump_write(c);
      return;
    }
    // new connection
    const Upstream& up = ups_[u];
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons(static_cast<uint16_t>(up.port));
    if (inet_pton(AF_INET, up.host.c_str(), &addr.sin_addr) != 1) {
      addrinfo hints{};
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      addrinfo* res = nullptr;
      if (getaddrinfo(up.host.c_str(), nullptr, &hints, &res) != 0 || !res) {
        finish(std::move(j), std::nullopt, "cannot resolve host " + up.host);
        return;
      }
      addr.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
      freeaddrinfo(res);
    }
    int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (fd < 0) {
      finish(std::move(j), std::nullopt, "socket() failed");
      return;
    }
    set_nodelay(fd, (ntohl(addr.sin_addr.s_addr) >> 24) == 127);
    int rc = ::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof addr);
    if (rc != 0 && errno != EINPROGRESS) {
      const std::string err = std::string("connect failed: ") + strerror(errno);
      ::close(fd);
      finish(std::move(j), std::nullopt, err);
      return;
    }
    opened_.fetch_add(1, std::memory_order_relaxed);
    auto c = std::make_unique<Conn>();
    c->fd = fd;
    c->id = L->next_id++;
    c->upstream = u;
    c->job = std::move(j);
    Conn* cp = c.get();
    L->conns.emplace(cp->id, std::move(c));
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
    ev.data.u64 = cp->id;
    epoll_ctl(L->ep, EPOLL_CTL_ADD, fd, &ev);
    cp->want_out = true;
    cp->state = Conn::CONNECTING;
    cp->deadline = Clock::now() + opt_.connect_timeout;
  };

  auto on_event = [&](Conn* c, uint32_t ev) {
    if (c->state == Conn::IDLE) {  // the server closed (or wrote garbage on) an idle keep-alive socket
      close_conn(c);
      return;
    }
    if (c->state == Conn::CONNECTING) {
      if (!(ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) return;
      int err = 0;
      socklen_t len = sizeof err;
      if (getsockopt(c->fd, SOL_SOCKET, SO_ERROR, &err, &len) != 0 || err != 0) {
        fail(c, std::string("connect failed: ") + strerror(err ? err : errno));
        return;
      }
      begin_write(c);
      if (!pump_write(c)) return;
    } else if (c->state == Conn::WRITING && (ev & EPOLLOUT)) {
      if (!pump_write(c)) return;
    }
    if (c->state != Conn::READING) {
      if (ev & (EPOLLERR | EPOLLHUP)) fail(c, "connection reset");
      return;
    }
    if (!(ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) return;
    while (true) {
      size_t old = c->in.size();
      size_t want = 65536;
      if (c->header_end != std::string::npos && c->has_len && !c->chunked) {
        const size_t need = c->header_end + 4 + c->content_len;
        if (need > old) want = std::max(want, need - old);
      }
      c->in.resize(old + want);
      ssize_t n = ::recv(c->fd, &c->in[old], want, 0);
      c->in.resize(old + (n > 0 ? static_cast<size_t>(n) : 0));
      if (n > 0) {
        c->got_any = true;
        if (try_complete(c, false)) return;
        continue;
      }
      if (n == 0) {
        if (!try_complete(c, true)) fail(c, "connection closed by peer");
        return;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) return;
      fail(c, std::string("recv failed: ") + strerror(errno));
      return;
    }
  };

  auto last_sweep = Clock::now();
  while (running_.load(std::memory_order_relaxed)) {
    int n = epoll_wait(L->ep, events.data(), static_cast<int>(events.size()), 20);
    if (n < 0 && errno != EINTR) break;
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = events[i].data.u64;
      if (tag == 1) {
        uint64_t v;
        ssize_t r = ::read(L->efd, &v, sizeof v);
        (void)r;
        {
          std::lock_guard<std::mutex> g(L->mu);
          jobs.swap(L->inbox);
        }
        while (!jobs.empty()) {
          std::unique_ptr<Job> j = std::move(jobs.front());
          jobs.pop_front();
          start(std::move(j));
        }
        continue;
      }
      auto f = L->conns.find(tag);
      if (f == L->conns.end()) continue;
      on_event(f->second.get(), events[i].events);
    }
    const auto now = Clock::now();
    if (now - last_sweep >= std::chrono::milliseconds(20)) {
      last_sweep = now;
      std::vector<Conn*> late;
      for (auto& kv : L->conns) {
        Conn* c = kv.second.get();
        if (c->state != Conn::IDLE && c->job && now > c->deadline) late.push_back(c);
      }
      for (Conn* c : late) fail(c, c->state == Conn::CONNECTING ? "connection timeout" : "read timeout");
    }
  }
  // shutting down: fail whatever is still pending
  {
    std::lock_guard<std::mutex> g(L->mu);
    for (auto& j : L->inbox) jobs.push_back(std::move(j));
    L->inbox.clear();
  }
  for (auto& j : jobs) finish(std::move(j), std::nullopt, "client stopped");
  for (auto& kv : L->conns)
    if (kv.second->job) finish(std::move(kv.second->job), std::nullopt, "client stopped");
}

}  // namespace die
