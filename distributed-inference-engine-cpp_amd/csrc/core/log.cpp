#include "log.h"

#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>

namespace die {

namespace {

std::atomic<uint64_t> g_emitted{0}, g_suppressed{0};

int initial_level() {
  const char* e = std::getenv("DIE_LOG_LEVEL");
  LogLevel lv = LogLevel::INFO;
  if (e && !parse_log_level(e, &lv)) lv = LogLevel::INFO;
  return static_cast<int>(lv);
}

const char* level_name(LogLevel lv) {
  switch (lv) {
    case LogLevel::TRACE: return "TRACE";
    case LogLevel::DEBUG: return "DEBUG";
    case LogLevel::INFO: return "INFO";
    case LogLevel::WARN: return "WARN";
    case LogLevel::ERROR: return "ERROR";
    default: return "OFF";
  }
}

}  // namespace

namespace log_detail {

std::atomic<int> g_level{initial_level()};

void emit(LogLevel lv, const char* file, int line, const std::string& msg, uint64_t suppressed) {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t;
  gmtime_r(&ts.tv_sec, &t);
  const char* base = std::strrchr(file, '/');
  base = base ? base + 1 : file;
  char head[160];
  int n = std::snprintf(head, sizeof head, "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ %-5s [%ld] %s:%d] ", t.tm_year + 1900,
                        t.tm_mon + 1, t.tm_mday, t.tm_hour, t.tm_min, t.tm_sec, ts.tv_nsec / 1000, level_name(lv),
                        static_cast<long>(syscall(SYS_gettid)), base, line);
  std::string out(head, static_cast<size_t>(n > 0 ? n : 0));
  out += msg;
  if (suppressed) out += " (" + std::to_string(suppressed) + " similar lines suppressed)";
  out += '\n';
  ssize_t w = ::write(2, out.data(), out.size());  // one syscall per line: no interleaving
  (void)w;
  g_emitted.fetch_add(1, std::memory_order_relaxed);
}

}  // namespace log_detail

void set_log_level(LogLevel lv) { log_detail::g_level.store(static_cast<int>(lv), std::memory_order_relaxed); }
LogLevel log_level() { return static_cast<LogLevel>(log_detail::g_level.load(std::memory_order_relaxed)); }

bool parse_log_level(const std::string& name, LogLevel* out) {
  std::string s;
  for (char c : name) s += static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  static const struct {
    const char* n;
    LogLevel l;
  } kNames[] = {{"trace", LogLevel::TRACE}, {"debug", LogLevel::DEBUG}, {"info", LogLevel::INFO},
                {"warn", LogLevel::WARN},   {"warning", LogLevel::WARN}, {"error", LogLevel::ERROR},
                {"off", LogLevel::OFF}};
  for (auto& k : kNames)
    if (s == k.n) {
      *out = k.l;
      return true;
    }
  return false;
}

uint64_t log_lines_emitted() { return g_emitted.load(); }
uint64_t log_lines_suppressed() { return g_suppressed.load(); }

bool LogRateLimiter::allow(int64_t interval_ms, uint64_t* suppressed) {
  const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch())
                          .count();
  int64_t next = next_ns_.load(std::memory_order_relaxed);
  if (now < next || !next_ns_.compare_exchange_strong(next, now + interval_ms * 1000000, std::memory_order_relaxed)) {
    dropped_.fetch_add(1, std::memory_order_relaxed);
    g_suppressed.fetch_add(1, std::memory_order_relaxed);
    return false;
  }
  *suppressed = dropped_.exchange(0, std::memory_order_relaxed);
  return true;
}

}  // namespace die
