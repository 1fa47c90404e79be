// Lock-free latency histograms for the worker's and gateway's request stages (SURVEY §5.1/§5.5:
// per-stage histograms on /health and /stats, extra keys only).  Log-linear buckets: 4 per octave
// of ~microseconds (ns / 1024), i.e. <= 19 % wide above 4 us (tail percentiles to about +-10 %,
// > 1 h at the top); percentiles report bucket upper bounds.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>

#include "../core/json.h"

namespace die {

class StageHist {
 public:
  static constexpr int kSub = 4;                  // buckets per octave
  static constexpr int kBuckets = 4 + 38 * kSub;  // u < 4 exactly, then 4 per octave
  // bucket of u = ns / 1024: u < 4 -> u; else octave o = floor(log2 u) >= 2 split by the next 2 bits
  static int bucket(uint64_t u) {
    if (u < 4) return static_cast<int>(u);
    const int o = 63 - __builtin_clzll(u);
    const int sub = static_cast<int>((u >> (o - 2)) & 3);
    const int b = 4 + (o - 2) * kSub + sub;
    return b < kBuckets ? b : kBuckets - 1;
  }
  // exclusive upper bound of bucket b, in u units
  static double upper(int b) {
    if (b < 4) return b + 1.0;
    const int o = (b - 4) / kSub + 2, sub = (b - 4) % kSub;
    return static_cast<double>(1ull << o) * (1.0 + (sub + 1) / 4.0);
  }
  void add(std::chrono::steady_clock::duration d) {
    const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(d).count();
    const uint64_t u = ns > 0 ? static_cast<uint64_t>(ns) >> 10 : 0;  // ~us
    buckets_[bucket(u)].fetch_add(1, std::memory_order_relaxed);
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
        if (acc > target) return upper(i) * 1024.0 / 1e3;
      }
      return 0.0;
    };
    j["p50_us"] = n ? pct(0.5) : 0.0;
    j["p90_us"] = n ? pct(0.9) : 0.0;
    j["p99_us"] = n ? pct(0.99) : 0.0;
    j["p999_us"] = n ? pct(0.999) : 0.0;
    return j;
  }

 private:
  std::atomic<uint64_t> buckets_[kBuckets] = {};
  std::atomic<uint64_t> count_{0};
  std::atomic<int64_t> sum_ns_{0};
};

}  // namespace die
