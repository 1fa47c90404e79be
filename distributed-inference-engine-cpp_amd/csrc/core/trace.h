// roctx ranges around the serving stages: parse -> cache -> batch dispatch -> H2D ->
// graph launch -> D2H/completion -> respond.  Collected with `rocprofv3 --marker-trace`.  Off unless
// DIE_ROCTX=1, so the hot path pays one predictable branch.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>

namespace die {

inline bool trace_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DIE_ROCTX");
    return e && *e == '1';
  }();
  return on;
}

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) roctxRangePushA(name);
  }
  ~TraceRange() {
    if (on_) roctxRangePop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

inline void trace_mark(const char* name) {
  if (trace_enabled()) roctxMarkA(name);
}

}  // namespace die
