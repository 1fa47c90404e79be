// Leveled, rate-limited logging.
//
// The reference writes raw std::cout/std::cerr lines with std::endl, including two flushed lines
// per request on the gateway's hot path (src/gateway.cpp:87,97,105,110-118,124).  Here
// every message has a level, the level check is one relaxed atomic load (nothing is formatted
// below the threshold), a line is emitted with ONE write(2) (no interleaving across threads), and
// DIE_LOG_EVERY_MS limits a call site to one line per interval, counting what it suppressed.
// Level: set_log_level(), or DIE_LOG_LEVEL=trace|debug|info|warn|error|off (default info).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <sstream>
#include <string>

namespace die {

enum class LogLevel : int { TRACE = 0, DEBUG = 1, INFO = 2, WARN = 3, ERROR = 4, OFF = 5 };

namespace log_detail {
extern std::atomic<int> g_level;
void emit(LogLevel lv, const char* file, int line, const std::string& msg, uint64_t suppressed);
}  // namespace log_detail

inline bool log_enabled(LogLevel lv) {
  return static_cast<int>(lv) >= log_detail::g_level.load(std::memory_order_relaxed);
}
void set_log_level(LogLevel lv);
LogLevel log_level();
// "trace" ... "off" (case-insensitive); returns false for an unknown name.
bool parse_log_level(const std::string& name, LogLevel* out);
// Lines emitted / suppressed by rate limits since start (exported on /health and /stats).
uint64_t log_lines_emitted();
uint64_t log_lines_suppressed();

// One call site's rate limiter: allow() is true at most once per interval; the lines it refused
// are reported with the next allowed line.
class LogRateLimiter {
 public:
  bool allow(int64_t interval_ms, uint64_t* suppressed);

 private:
  std::atomic<int64_t> next_ns_{0};
  std::atomic<uint64_t> dropped_{0};
};

}  // namespace die

#define DIE_LOG(level, expr)                                                               \
  do {                                                                                     \
    if (::die::log_enabled(::die::LogLevel::level)) {                                      \
      std::ostringstream die_log_os_;                                                      \
      die_log_os_ << expr;                                                                 \
      ::die::log_detail::emit(::die::LogLevel::level, __FILE__, __LINE__, die_log_os_.str(), 0); \
    }                                                                                      \
  } while (0)

#define DIE_LOG_EVERY_MS(level, interval_ms, expr)                                         \
  do {                                                                                     \
    if (::die::log_enabled(::die::LogLevel::level)) {                                      \
      static ::die::LogRateLimiter die_log_rl_;                                            \
      uint64_t die_log_sup_ = 0;                                                           \
      if (die_log_rl_.allow(interval_ms, &die_log_sup_)) {                                 \
        std::ostringstream die_log_os_;                                                    \
        die_log_os_ << expr;                                                               \
        ::die::log_detail::emit(::die::LogLevel::level, __FILE__, __LINE__, die_log_os_.str(), die_log_sup_); \
      }                                                                                    \
    }                                                                                      \
  } while (0)
