// Three-state circuit breaker, same state machine as the reference (src/circuit_breaker.cpp:12-47):
//  * CLOSED -> OPEN after `failure_threshold` failures without an intervening success;
//  * OPEN -> HALF_OPEN on the first allowRequest() at least `timeout` after the last failure
//    (no limit on concurrent half-open probes, as in the reference);
//  * HALF_OPEN -> CLOSED after `success_threshold` successes; any failure -> OPEN.
// The clock is injectable so tests do not sleep.
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <mutex>
#include <string>

namespace die {

enum class CircuitState { CLOSED, OPEN, HALF_OPEN };

class CircuitBreaker {
 public:
  using Clock = std::function<std::chrono::steady_clock::time_point()>;

  CircuitBreaker(int failure_threshold = 5, int success_threshold = 2,
                 std::chrono::milliseconds timeout = std::chrono::seconds(30), Clock clock = nullptr);

  bool allowRequest();
  void recordSuccess();
  void recordFailure();
  CircuitState getState() const { return state_.load(); }
  std::string getStateString() const;
  int getFailureCount() const;
  int getSuccessCount() const { return success_count_.load(); }
  // Transition counters (observability superset; fault-injection drills assert on them because a
  // HALF_OPEN window can be shorter than any polling interval).
  long long opened() const { return opened_.load(); }
  long long half_opened() const { return half_opened_.load(); }
  long long closed() const { return closed_.load(); }

 private:
  std::chrono::steady_clock::time_point now() const { return clock_ ? clock_() : std::chrono::steady_clock::now(); }
  std::atomic<CircuitState> state_{CircuitState::CLOSED};
  int failure_count_ = 0;
  std::atomic<int> success_count_{0};
  int failure_threshold_;
  int success_threshold_;
  std::chrono::milliseconds timeout_;
  Clock clock_;
  std::chrono::steady_clock::time_point last_failure_;
  mutable std::mutex mutex_;
  std::atomic<long long> opened_{0}, half_opened_{0}, closed_{0};
};

const char* circuit_state_name(CircuitState s);

}  // namespace die
