// Lock-free latency histograms for the worker's and gateway's request stages (SURVEY §5.1/§5.5:
// per-stage histograms on /health and /stats, extra keys only).  Log-linear buckets: 8 per octave
// of ~microseconds (ns / 1024), i.e. <= 12.5 % wide above 8 us (tail percentiles to about +-6 %,
// days at the top); percentiles report bucket upper bounds.  The snapshot also carries the
// non-empty buckets ("hist": [[bucket, count], ...]) so a client can difference two snapshots and
// take percentiles over a window (bench.py: the timed pass only, warm-up excluded).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>

#include "../core/json.h"

namespace die {

class StageHist {
 public:
  static constexpr int kBits = 3, kSub = 1 << kBits;    // 8 buckets per octave
  static constexpr int kBuckets = kSub + (40 - kBits) * kSub;  // u < 8 exactly, then 8 per octave
  // bucket of u = ns / 1024: u < 8 -> u; else octave o = floor(log2 u) >= 3 split by the next 3 bits
  static int bucket(uint64_t u) {
    if (u < kSub) return static_cast<int>(u);
    const int o = 63 - __builtin_clzll(u);
    const int sub = static_cast<int>((u >> (o - kBits)) & (kSub - 1));
    const int b = kSub + (o - kBits) * kSub + sub;
    return b < kBuckets ? b : kBuckets - 1;
  }
  // exclusive upper bound of bucket b, in u units
  static double upper(int b) {
    if (b < kSub) return b + 1.0;
    const int o = (b - kSub) / kSub + kBits, sub = (b - kSub) % kSub;
    return static_cast<double>(1ull << o) * (1.0 + (sub + 1) / static_cast<double>(kSub));
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
    Json h = Json::array();
    for (int i = 0; i < kBuckets; ++i)
      if (c[i]) {
        Json e = Json::array();
        e.push_back(static_cast<long long>(i));
        e.push_back(static_cast<long long>(c[i]));
        h.push_back(e);
      }
    j["hist"] = h;
    j["bucket_us"] = 1.024;  // u unit in us; bucket b spans [lower, upper(b)) u
    return j;
  }

 private:
  std::atomic<uint64_t> buckets_[kBuckets] = {};
  std::atomic<uint64_t> count_{0};
  std::atomic<int64_t> sum_ns_{0};
};

}  // namespace die
