#include "circuit_breaker.h"

namespace die {

const char* circuit_state_name(CircuitState s) {
  switch (s) {
    case CircuitState::CLOSED: return "CLOSED";
    case CircuitState::OPEN: return "OPEN";
    case CircuitState::HALF_OPEN: return "HALF_OPEN";
  }
  return "UNKNOWN";
}

CircuitBreaker::CircuitBreaker(int failure_threshold, int success_threshold, std::chrono::milliseconds timeout,
                               Clock clock)
    : failure_threshold_(failure_threshold),
      success_threshold_(success_threshold),
      timeout_(timeout),
      clock_(std::move(clock)),
      last_failure_(now()) {}

bool CircuitBreaker::allowRequest() {
  std::lock_guard<std::mutex> g(mutex_);
  if (state_ == CircuitState::OPEN) {
    if (now() - last_failure_ >= timeout_) {
      state_ = CircuitState::HALF_OPEN;
      success_count_ = 0;
      ++half_opened_;
      return true;
    }
    return false;
  }
  return true;
}

void CircuitBreaker::recordSuccess() {
  std::lock_guard<std::mutex> g(mutex_);
  if (state_ == CircuitState::HALF_OPEN) {
    if (++success_count_ >= success_threshold_) {
      state_ = CircuitState::CLOSED;
      failure_count_ = 0;
      ++closed_;
    }
  } else {
    failure_count_ = 0;
  }
}

void CircuitBreaker::recordFailure() {
  std::lock_guard<std::mutex> g(mutex_);
  ++failure_count_;
  last_failure_ = now();
  if ((failure_count_ >= failure_threshold_ || state_ == CircuitState::HALF_OPEN) && state_ != CircuitState::OPEN) {
    state_ = CircuitState::OPEN;
    ++opened_;
  }
}

std::string CircuitBreaker::getStateString() const { return circuit_state_name(getState()); }

int CircuitBreaker::getFailureCount() const {
  std::lock_guard<std::mutex> g(mutex_);
  return failure_count_;
}

}  // namespace die
