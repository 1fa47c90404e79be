#include <pthread.h>
#include "loadgen.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <strings.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <cmath>
#include <random>
#include <thread>

#include "../core/http.h"

namespace die {

namespace {

struct Template {
  std::string body;
  size_t id_pos = 0, id_len = 0;  // fixed-width decimal request number
  size_t v0_pos = 0, v1_pos = 0;  // fixed-width "0.dddd" values patched per request
  size_t vend[3] = {0, 0, 0};     // verify templates: end of the first three values' text (0 = no padding)
};

uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

constexpr int kIdDigits = 10;

// Bijection of [0, 10^10) (parallel/ring_balance.py scramble_id): a 4-round Feistel network on the
// two 5-digit halves with splitmix64 round functions, so distinct request numbers print distinct
// ids that FNV-1a spreads over the gateway ring like random ones.
uint64_t scramble_id(uint64_t i) {
  constexpr uint64_t kHalf = 100000;
  uint64_t left = (i % 10000000000ull) / kHalf, right = i % kHalf;
  for (uint64_t k = 0; k < 4; ++k) {
    const uint64_t next = (left + splitmix64(right * 4 + k) % kHalf) % kHalf;
    left = right;
    right = next;
  }
  return left * kHalf + right;
}

Template make_full_template(const LoadgenOptions& o, uint64_t seed) {
  Template t;
  std::mt19937_64 rng(seed);
  std::string& b = t.body;
  b.reserve(o.input_numel * (o.decimals + 3) + 64);
  b += "{\"request_id\":\"";
  b += o.id_prefix;
  t.id_pos = b.size();
  t.id_len = kIdDigits;
  b.append(kIdDigits, '0');
  b += "\",\"input_data\":[";
  const int d = std::max(1, std::min(o.decimals, 8));
  uint64_t scale = 1;
  for (int k = 0; k < d; ++k) scale *= 10;
  char buf[32];
  for (size_t i = 0; i < o.input_numel; ++i) {
    if (i) b.push_back(',');
    if (i == 0) t.v0_pos = b.size();
    if (i == 1) t.v1_pos = b.size();
    const uint64_t v = rng() % scale;
    int n = std::snprintf(buf, sizeof buf, "0.%0*llu", d, static_cast<unsigned long long>(v));
    b.append(buf, static_cast<size_t>(n));
  }
  b += "]}";
  return t;
}

// Verify-mode body of input k: shortest round-trip float text, so a worker that parses (or decodes
// on the device) exactly gets verify_inputs[k].
Template make_verify_template(const LoadgenOptions& o, size_t k) {
  Template t;
  std::string& b = t.body;
  b += "{\"request_id\":\"";
  b += o.id_prefix;
  t.id_pos = b.size();
  t.id_len = kIdDigits;
  b.append(kIdDigits, '0');
  b += "\",\"input_data\":";
  const size_t arr = b.size();
  // Each value in the full payload's own fixed "%.Nf" form (N = o.decimals) when that text parses
  // back to exactly the float (image-like inputs with N decimals), else the shortest round-trip
  // text: a verified request then looks like every other request to the parser and the device
  // decoder (same token lengths, no exponents), so checking answers costs no throughput.
  const float* xs = o.verify_inputs + k * o.input_numel;
  const int d = std::max(1, std::min(o.decimals, 8));
  b += '[';
  char buf[48];
  for (size_t i = 0; i < o.input_numel; ++i) {
    if (i) b.push_back(',');
    const auto r = std::to_chars(buf, buf + sizeof buf, xs[i], std::chars_format::fixed, d);
    float back = 0.f;
    if (r.ec == std::errc() && std::from_chars(buf, r.ptr, back).ec == std::errc() && back == xs[i]) b.append(buf, r.ptr);
    else b.append(buf, std::to_chars(buf, buf + sizeof buf, xs[i]).ptr);
  }
  b += "]}";
  // the first three values, if plain decimals ("0.5"), can take trailing zeros without changing them
  size_t e[3], from = arr + 1;
  bool ok = true;
  for (int i = 0; i < 3 && ok; ++i) {
    e[i] = b.find(',', from);
    ok = e[i] != std::string::npos;
    if (ok) {
      const std::string v = b.substr(from, e[i] - from);
      ok = v.find('.') != std::string::npos && v.find_first_of("eE") == std::string::npos && v.size() <= 11;
      from = e[i] + 1;
    }
  }
  if (ok)
    for (int i = 0; i < 3; ++i) t.vend[i] = e[i];
  return t;
}

// Variant v of a verify body: v % 16, v / 16 % 16 and v / 256 % 16 zeros after values 0, 1 and 2
// (4,096 distinct texts per input).  At most 15 zeros keep every value within the device decoder's
// 19-significant-digit fast path (kernels/decode.hip), so a verified request is decoded on the GPU
// like every other request instead of taking the host re-parse (round 4: 56 fallbacks, ~5 % of the
// headline).
void verify_body(const Template& t, long v, std::string& out) {
  if (!t.vend[0]) {
    out = t.body;
    return;
  }
  const size_t z[3] = {static_cast<size_t>(v % 16), static_cast<size_t>((v / 16) % 16), static_cast<size_t>((v / 256) % 16)};
  out.clear();
  out.reserve(t.body.size() + z[0] + z[1] + z[2]);
  size_t at = 0;
  for (int i = 0; i < 3; ++i) {
    out.append(t.body, at, t.vend[i] - at);
    out.append(z[i], '0');
    at = t.vend[i];
  }
  out.append(t.body, at, std::string::npos);
}

// Relative L2 error of a response's output_data against `ref` (n floats); < 0 when the body has no
// numeric output_data of length n.  `id_ok` reports whether the request_id echo equals `id`.
double response_error(const std::string& body, const float* ref, size_t n, const std::string& id, bool& id_ok) {
  Json j;
  try {
    j = Json::parse(body);
  } catch (const std::exception&) {
    id_ok = false;
    return -1.0;
  }
  const Json* rid = j.find("request_id");
  id_ok = rid && rid->is_string() && rid->as_string() == id;
  const Json* out = j.find("output_data");
  if (!out || !out->is_array() || out->size() != n) return -1.0;
  double num = 0.0, den = 0.0;
  for (size_t i = 0; i < n; ++i) {
    const Json& v = (*out)[i];
    if (!v.is_number()) return -1.0;
    const double d = v.as_double() - static_cast<double>(ref[i]);
    num += d * d;
    den += static_cast<double>(ref[i]) * ref[i];
  }
  return den > 0.0 ? std::sqrt(num / den) : std::sqrt(num);
}

void patch_digits(std::string& b, size_t pos, size_t width, uint64_t v) {
  for (size_t k = 0; k < width; ++k) {
    b[pos + width - 1 - k] = static_cast<char>('0' + v % 10);
    v /= 10;
  }
}

struct Gate {
  std::mutex mu;
  std::condition_variable cv;
  int waiting = 0, total = 0, gen = 0;
  void arrive() {
    std::unique_lock<std::mutex> lk(mu);
    const int g = gen;
    if (++waiting == total) {
      waiting = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

}  // namespace

Json run_loadgen(const LoadgenOptions& o) {
  const int C = std::max(1, o.connections);
  std::atomic<long> next_warm{0}, next{0};
  std::vector<std::vector<double>> lat(C);
  std::vector<std::vector<std::pair<double, double>>> when(C);  // (start offset in the timed window, latency) ms
  std::vector<long> ok(C, 0), fail(C, 0);
  std::vector<std::map<std::string, long>> errs(C);
  Gate gate;
  gate.total = C + 1;
  std::chrono::steady_clock::time_point t0, t1;
  const bool verify = o.payload == "verify";
  const bool full = o.payload == "full";
  const bool sampled = full && o.verify_every > 0;  // full mode with a verified sample
  if ((verify || sampled) && (!o.verify_inputs || !o.verify_expected || o.verify_count == 0 || o.output_numel == 0))
    throw std::runtime_error("loadgen verify mode needs verify_inputs, verify_expected, verify_count, output_numel");
  std::vector<Template> vt;  // verify mode: one shared template per distinct input
  for (size_t k = 0; (verify || sampled) && k < o.verify_count; ++k) vt.push_back(make_verify_template(o, k));
  auto printed = [&](long id) -> uint64_t {
    return o.scramble_ids ? scramble_id(static_cast<uint64_t>(id)) : static_cast<uint64_t>(id);
  };
  auto is_verify = [&](long id) { return verify || (sampled && id % o.verify_every == 0); };
  auto verify_k = [&](long id) -> size_t {
    return static_cast<size_t>(sampled ? id / o.verify_every : id) % vt.size();
  };
  std::vector<long> verified(C, 0), mismatched(C, 0), bad_id(C, 0);
  std::vector<double> max_err(C, 0.0);
  const int d = std::max(1, std::min(o.decimals, 8));
  uint64_t scale = 1;
  for (int k = 0; k < d; ++k) scale *= 10;

  // Per-connection request bodies: the connection's own copy of the full-payload template (patched
  // in place per request), or a verify / reference body.  A body stays untouched until its request
  // has been sent completely (one request in flight per connection).
  struct Bodies {
    Template tpl;
    std::string vbody, small;
  };
  auto body_for = [&](Bodies& bd, int c, long id) -> const std::string& {
    if (is_verify(id)) {
      const Template& t = vt[verify_k(id)];
      // 512 variants per seed residue: concurrent clients with different seeds (one per rank) never
      // send the same verify text, so none of them is a cache hit on a shared worker.  The texts
      // repeat after 511 * inputs * verify_every requests (reported as verify_repeat_period; bench.py
      // checks its run is shorter).
      if (sampled)
        verify_body(t, (id / o.verify_every) / static_cast<long>(vt.size()) % 511 + 1 + 512 * static_cast<long>(o.seed % 8),
                    bd.vbody);
      else bd.vbody = t.body;
      patch_digits(bd.vbody, t.id_pos, t.id_len, printed(id));
      return bd.vbody;
    }
    const long key = o.distinct > 0 ? id % o.distinct : id;
    if (full) {
      Template& tpl = bd.tpl;
      patch_digits(tpl.body, tpl.id_pos, tpl.id_len, printed(id));
      // unique input: encode (key, connection) in the first two values
      const uint64_t u = static_cast<uint64_t>(key) * 64 + static_cast<uint64_t>(c);
      patch_digits(tpl.body, tpl.v0_pos + 2, static_cast<size_t>(d), u % scale);
      patch_digits(tpl.body, tpl.v1_pos + 2, static_cast<size_t>(d), (u / scale) % scale);
      return tpl.body;
    }
    const long a = key % 10;
    bd.small = "{\"request_id\":\"" + o.id_prefix + std::to_string(printed(id)) + "\",\"input_data\":[" +
               std::to_string(a) + ".0," + std::to_string(a + 1) + ".0," + std::to_string(a + 2) + ".0]}";
    return bd.small;
  };
  // Account one finished request of connection c (status 0 = transport error `err`).
  auto finish = [&](int c, long id, std::chrono::steady_clock::time_point s, int status, const std::string& body,
                    const std::string& err) {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s).count();
    if (status == 200) {
      ++ok[c];
      lat[c].push_back(ms);
      when[c].emplace_back(std::chrono::duration<double, std::milli>(s - t0).count(), ms);
      if (is_verify(id)) {
        const size_t k = verify_k(id);
        char idbuf[32];
        std::snprintf(idbuf, sizeof idbuf, "%0*llu", kIdDigits, static_cast<unsigned long long>(printed(id)));
        bool id_ok = false;
        const double e = response_error(body, o.verify_expected + k * o.output_numel, o.output_numel,
                                        o.id_prefix + idbuf, id_ok);
        ++verified[c];
        if (!id_ok) ++bad_id[c];
        if (e < 0.0 || e > o.verify_tol) ++mismatched[c];
        max_err[c] = std::max(max_err[c], e < 0.0 ? 1e30 : e);
      }
    } else {
      ++fail[c];
      errs[c][status ? "HTTP " + std::to_string(status) : err]++;
    }
  };

  // One epoll loop over connections `mine`: warm-up ids until next_warm runs out, the gate (twice,
  // as the threaded clients), timed ids until next runs out, the gate again.
  auto async_loop = [&](const std::vector<int>& mine) {
    struct AConn {
      int c = 0, fd = -1;
      Bodies bd;
      std::string head, in;
      const std::string* body = nullptr;
      size_t sent = 0, hdr_end = std::string::npos, clen = 0;
      int status = 0;
      long id = -1;
      bool record = false, busy = false;
      std::chrono::steady_clock::time_point start;
    };
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    if (ep < 0) throw std::runtime_error("loadgen: epoll_create1 failed");
    std::vector<AConn> cs(mine.size());
    auto open_conn = [&](AConn& k) -> bool {
      if (k.fd >= 0) {
        epoll_ctl(ep, EPOLL_CTL_DEL, k.fd, nullptr);
        ::close(k.fd);
      }
      k.fd = -1;
      sockaddr_in addr{};
      addr.sin_family = AF_INET;
      addr.sin_port = htons(static_cast<uint16_t>(o.port));
      if (inet_pton(AF_INET, o.host == "localhost" ? "127.0.0.1" : o.host.c_str(), &addr.sin_addr) != 1) return false;
      const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (fd < 0) return false;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0) {
        ::close(fd);
        return false;
      }
      fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK);
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = static_cast<uint64_t>(&k - cs.data());
      epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
      k.fd = fd;
      return true;
    };
    auto want = [&](AConn& k, uint32_t events) {
      epoll_event ev{};
      ev.events = events;
      ev.data.u64 = static_cast<uint64_t>(&k - cs.data());
      epoll_ctl(ep, EPOLL_CTL_MOD, k.fd, &ev);
    };
    // push as much of head + body as the socket takes; false on a transport error
    auto pump_send = [&](AConn& k) -> bool {
      while (true) {
        const size_t hs = k.head.size(), total = hs + k.body->size();
        if (k.sent >= total) return true;
        iovec iov[2];
        int n = 0;
        if (k.sent < hs) iov[n++] = {const_cast<char*>(k.head.data()) + k.sent, hs - k.sent};
        const size_t boff = k.sent > hs ? k.sent - hs : 0;
        iov[n++] = {const_cast<char*>(k.body->data()) + boff, k.body->size() - boff};
        const ssize_t w = ::writev(k.fd, iov, n);
        if (w > 0) {
          k.sent += static_cast<size_t>(w);
          continue;
        }
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;
        if (w < 0 && errno == EINTR) continue;
        return false;
      }
    };
    auto start_req = [&](AConn& k, long id, bool record) {
      k.id = id;
      k.record = record;
      k.busy = true;
      k.body = &body_for(k.bd, k.c, id);
      k.head = "POST " + o.path + " HTTP/1.1\r\nHost: " + o.host + "\r\nContent-Type: application/json\r\nContent-Length: " +
               std::to_string(k.body->size()) + "\r\n\r\n";
      k.sent = 0;
      k.in.clear();
      k.hdr_end = std::string::npos;
      k.clen = 0;
      k.status = 0;
      k.start = std::chrono::steady_clock::now();
      if (k.fd < 0 && !open_conn(k)) {
        k.busy = false;
        if (record) finish(k.c, id, k.start, 0, std::string(), "connect failed");
        return;
      }
      if (!pump_send(k)) {  // a stale keep-alive connection: reconnect once and resend
        if (!open_conn(k) || (k.sent = 0, !pump_send(k))) {
          k.busy = false;
          if (record) finish(k.c, id, k.start, 0, std::string(), "send failed");
          return;
        }
      }
      want(k, k.sent < k.head.size() + k.body->size() ? EPOLLOUT : EPOLLIN);
    };
    auto fail_req = [&](AConn& k, const char* why) {
      k.busy = false;
      if (k.record) finish(k.c, k.id, k.start, 0, std::string(), why);
      open_conn(k);
    };
    // parse what has arrived; true when the whole response is in
    auto parse = [&](AConn& k) -> bool {
      if (k.hdr_end == std::string::npos) {
        k.hdr_end = k.in.find("\r\n\r\n");
        if (k.hdr_end == std::string::npos) return false;
        k.status = k.in.size() > 12 ? std::atoi(k.in.c_str() + 9) : 0;
        bool have_len = false;
        size_t pos = 0;
        while (pos < k.hdr_end) {
          size_t eol = k.in.find("\r\n", pos);
          if (eol == std::string::npos || eol > k.hdr_end) eol = k.hdr_end;
          static const char kCl[] = "content-length:";
          if (eol - pos > sizeof(kCl) - 1 && strncasecmp(k.in.c_str() + pos, kCl, sizeof(kCl) - 1) == 0) {
            k.clen = static_cast<size_t>(std::strtoull(k.in.c_str() + pos + sizeof(kCl) - 1, nullptr, 10));
            have_len = true;
          }
          pos = eol + 2;
        }
        if (!have_len) k.clen = 0;
      }
      return k.in.size() >= k.hdr_end + 4 + k.clen;
    };
    bool timed = false;
    long live = 0;  // requests in flight on this loop
    // the connection's next request; one that fails at once (connect / send error) is accounted and
    // the next id taken, as a blocking client moves on after a failed post
    auto next_id = [&](AConn& k) {
      while (true) {
        const long id = timed ? next.fetch_add(1) : next_warm.fetch_add(1);
        if (id >= (timed ? o.requests : o.warmup)) break;
        start_req(k, timed ? id : 1000000000L + id, timed);
        if (k.busy) return;
      }
      k.busy = false;
    };
    for (size_t i = 0; i < cs.size(); ++i) {
      cs[i].c = mine[i];
      if (full) cs[i].bd.tpl = make_full_template(o, o.seed * 7919 + static_cast<uint64_t>(mine[i]));
      open_conn(cs[i]);
    }
    std::vector<char> rbuf(1 << 16);
    for (int phase = 0; phase < 2; ++phase) {
      timed = phase == 1;
      for (auto& k : cs) next_id(k);
      while (true) {
        live = 0;
        for (auto& k : cs) live += k.busy;
        if (!live) break;
        epoll_event evs[64];
        const int n = epoll_wait(ep, evs, 64, 50);
        const auto now = std::chrono::steady_clock::now();
        for (int e = 0; e < n; ++e) {
          AConn& k = cs[evs[e].data.u64];
          if (!k.busy) continue;
          if (evs[e].events & EPOLLOUT) {
            if (!pump_send(k)) {
              fail_req(k, "send failed");
              next_id(k);
              continue;
            }
            if (k.sent >= k.head.size() + k.body->size()) want(k, EPOLLIN);
          }
          if (evs[e].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
            bool closed = false;
            while (true) {
              const ssize_t r = ::read(k.fd, rbuf.data(), rbuf.size());
              if (r > 0) {
                k.in.append(rbuf.data(), static_cast<size_t>(r));
                continue;
              }
              if (r == 0) closed = true;
              else if (errno == EINTR) continue;
              else if (errno != EAGAIN && errno != EWOULDBLOCK) closed = true;
              break;
            }
            if (parse(k)) {
              k.busy = false;
              if (k.record)
                finish(k.c, k.id, k.start, k.status,
                       is_verify(k.id) ? k.in.substr(k.hdr_end + 4, k.clen) : std::string(), std::string());
              if (closed) open_conn(k);
              next_id(k);
            } else if (closed) {
              fail_req(k, "connection closed");
              next_id(k);
            }
          }
        }
        for (auto& k : cs)  // per-request timeout
          if (k.busy && now - k.start > std::chrono::milliseconds(o.timeout_ms)) {
            fail_req(k, "timeout");
            next_id(k);
          }
      }
      if (phase == 0) {
        gate.arrive();  // all warm
        gate.arrive();  // timed start
      }
    }
    gate.arrive();
    for (auto& k : cs)
      if (k.fd >= 0) ::close(k.fd);
    ::close(ep);
  };

  std::vector<std::thread> threads;
  if (o.io_threads > 0) {
    // Event-driven client: io_threads epoll loops share the C connections (one request in flight
    // per connection, closed loop as below) -- no thread per connection competing with the server
    // under test for the CPU share.
    const int T = std::min(o.io_threads, C);
    gate.total = T + 1;
    for (int t = 0; t < T; ++t)
      threads.emplace_back([&, t, T] {
        pthread_setname_np(pthread_self(), "die-loadgen-io");
        std::vector<int> mine;
        for (int c = t; c < C; c += T) mine.push_back(c);
        async_loop(mine);
      });
  } else {
    for (int c = 0; c < C; ++c) {
      threads.emplace_back([&, c] {
        pthread_setname_np(pthread_self(), "die-loadgen");
        HttpClient client(o.host, o.port, std::chrono::milliseconds(o.timeout_ms), std::chrono::milliseconds(o.timeout_ms), 2);
        Bodies bd;
        if (full) bd.tpl = make_full_template(o, o.seed * 7919 + static_cast<uint64_t>(c));
        auto one = [&](long id, bool record) {
          const std::string& body = body_for(bd, c, id);
          auto s = std::chrono::steady_clock::now();
          std::string err;
          auto r = client.post(o.path, body, "application/json", &err);
          if (!record) return;
          finish(c, id, s, r ? r->status : 0, r ? r->body : std::string(), err);
        };
        while (true) {
          long id = next_warm.fetch_add(1);
          if (id >= o.warmup) break;
          one(1000000000L + id, false);
        }
        gate.arrive();  // all warm
        gate.arrive();  // timed start
        while (true) {
          long id = next.fetch_add(1);
          if (id >= o.requests) break;
          one(id, true);
        }
        gate.arrive();
      });
    }
  }
  gate.arrive();  // every client thread built its payloads and finished the warm-up
  if (o.on_ready) o.on_ready(o.on_ready_arg);
  t0 = std::chrono::steady_clock::now();
  gate.arrive();
  gate.arrive();
  t1 = std::chrono::steady_clock::now();
  for (auto& t : threads) t.join();

  std::vector<double> all;
  long n_ok = 0, n_fail = 0;
  std::map<std::string, long> merged;
  for (int c = 0; c < C; ++c) {
    all.insert(all.end(), lat[c].begin(), lat[c].end());
    n_ok += ok[c];
    n_fail += fail[c];
    for (auto& kv : errs[c]) merged[kv.first] += kv.second;
  }
  std::sort(all.begin(), all.end());
  const double wall = std::chrono::duration<double>(t1 - t0).count();
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, static_cast<size_t>(all.size() * p))]; };
  double mean = 0;
  for (double v : all) mean += v;
  if (!all.empty()) mean /= all.size();
  Json j = Json::object();
  j["requests"] = static_cast<long long>(o.requests);
  j["ok"] = static_cast<long long>(n_ok);
  j["failed"] = static_cast<long long>(n_fail);
  j["connections"] = C;
  j["wall_s"] = wall;
  j["rps"] = wall > 0 ? n_ok / wall : 0.0;
  Json l = Json::object();
  l["mean"] = mean;
  l["p50"] = pct(0.50);
  l["p90"] = pct(0.90);
  l["p95"] = pct(0.95);
  l["p99"] = pct(0.99);
  l["min"] = all.empty() ? 0.0 : all.front();
  l["max"] = all.empty() ? 0.0 : all.back();
  j["latency_ms"] = l;
  // tail attribution: p99 per tenth of the timed window (by request start) and the slowest requests
  // with their start offsets -- a tail clustered at the start is warm-up, a periodic one a stall
  {
    std::vector<std::pair<double, double>> w;
    for (int c = 0; c < C; ++c) w.insert(w.end(), when[c].begin(), when[c].end());
    const double span = wall * 1000.0;
    Json dec = Json::array();
    for (int k = 0; k < 10 && span > 0; ++k) {
      std::vector<double> v;
      for (auto& x : w)
        if (x.first >= span * k / 10 && (x.first < span * (k + 1) / 10 || k == 9)) v.push_back(x.second);
      std::sort(v.begin(), v.end());
      dec.push_back(v.empty() ? 0.0 : v[std::min(v.size() - 1, static_cast<size_t>(v.size() * 0.99))]);
    }
    j["p99_by_tenth_ms"] = dec;
    std::sort(w.begin(), w.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    Json slow = Json::array();
    for (size_t k = 0; k < std::min<size_t>(10, w.size()); ++k) {
      Json e2 = Json::array();
      e2.push_back(std::round(w[k].first * 10) / 10);
      e2.push_back(std::round(w[k].second * 100) / 100);
      slow.push_back(e2);
    }
    j["slowest_ms"] = slow;  // [start offset, latency]
  }
  Json e = Json::object();
  for (auto& kv : merged) e[kv.first] = static_cast<long long>(kv.second);
  j["errors"] = e;
  j["payload"] = o.payload;
  j["body_bytes"] = static_cast<long long>(verify ? vt[0].body.size() : full ? make_full_template(o, 1).body.size() : 60);
  if (verify || sampled) {
    long nv = 0, nm = 0, nb = 0;
    double me = 0.0;
    for (int c = 0; c < C; ++c) {
      nv += verified[c];
      nm += mismatched[c];
      nb += bad_id[c];
      me = std::max(me, max_err[c]);
    }
    j["verified"] = static_cast<long long>(nv);
    j["mismatched"] = static_cast<long long>(nm);
    j["bad_request_id"] = static_cast<long long>(nb);
    j["max_rel_err"] = me;
    // sampled mode: requests after which a verify text repeats (511 variants per input and seed
    // residue), so a longer run would see repeated verify texts as cache hits
    if (sampled) j["verify_repeat_period"] = static_cast<long long>(511) * static_cast<long long>(vt.size()) * o.verify_every;
  }
  return j;
}

}  // namespace die
