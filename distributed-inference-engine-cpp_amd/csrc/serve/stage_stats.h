// Lock-free latency histograms for the worker's request stages (per-stage
// histograms on /health, extra keys only).  Buckets are powers of two of nanoseconds / 1024
// (~1 us resolution at the bottom, > 1 h at the top); percentiles are bucket upper bounds.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>

#include "../core/json.h"

namespace die {

class StageHist {
 public:
  static constexpr int kBuckets = 40;
  void add(std::chrono::steady_clock::duration d) {
    const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(d).count();
    const uint64_t u = ns > 0 ? static_cast<uint64_t>(ns) >> 10 : 0;  // ~us
    const int b = u ? 64 - __builtin_clzll(u) : 0;
    buckets_[b < kBuckets ? b : kBuckets - 1].fetch_add(1, std::memory_order_relaxed);
    count_.fetch_add(1, std::memory_order_relaxed);
    sum_ns_.fetch_add(ns, std::memory_order_relaxed);
  }
  Json snapshot() const {
    uint64_t c[kBuckets];
    uint64_t n = 0;
    for (int i = 0; i < kBuckets; ++i) n += c[i] = buckets_[i].load(std::memory_order_relaxed);
    Json j = Json::object();
    j["count"] = static_cast<long long>(n);
    j["avg_us"] = n ? sum_ns_.load() / 1e3 / static_cast<double>(n) : 0.0;
    auto pct = [&](double q) {
      const uint64_t target = static_cast<uint64_t>(q * static_cast<double>(n));
      uint64_t acc = 0;
      for (int i = 0; i < kBuckets; ++i) {
        acc += c[i];
        if (acc > target) return static_cast<double>((1ull << i) * 1024) / 1e3;
      }
      return 0.0;
    };
    j["p50_us"] = n ? pct(0.5) : 0.0;
    j["p99_us"] = n ? pct(0.99) : 0.0;
    return j;
  }

 private:
  std::atomic<uint64_t> buckets_[kBuckets] = {};
  std::atomic<uint64_t> count_{0};
  std::atomic<int64_t> sum_ns_{0};
};

}  // namespace die
