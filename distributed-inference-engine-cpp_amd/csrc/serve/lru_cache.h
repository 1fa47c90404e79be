// Thread-safe LRU result cache.
//
// Same semantics as the reference (include/lru_cache.h:13-81): a recency list plus a hash map of
// list iterators, `get` promotes, `put` overwrites-and-promotes or evicts the tail at capacity, and
// hit/miss counters.  The worker keys it with `InputKey` instead of the raw vector<float>: the
// reference's VectorHash samples only 3 elements (include/lru_cache.h:84-96), which turns
// 150,528-float ResNet inputs into long collision chains, and storing the raw key costs 600 KB per
// entry.  InputKey is (length, 128-bit hash of every float's bits); equal inputs always map to the
// same key, and two different inputs collide with probability ~2^-128.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <list>
#include <mutex>
#include <optional>
#include <random>
#include <unordered_map>
#include <utility>
#include <vector>

namespace die {

template <typename Key, typename Value, typename Hash = std::hash<Key>>
class LRUCache {
 public:
  explicit LRUCache(size_t capacity) : capacity_(capacity) {}

  std::optional<Value> get(const Key& key) {
    std::lock_guard<std::mutex> g(mutex_);
    auto it = map_.find(key);
    if (it == map_.end()) {
      misses_.fetch_add(1, std::memory_order_relaxed);
      return std::nullopt;
    }
    list_.splice(list_.begin(), list_, it->second);
    hits_.fetch_add(1, std::memory_order_relaxed);
    return it->second->second;
  }

  void put(const Key& key, const Value& value) {
    std::lock_guard<std::mutex> g(mutex_);
    if (capacity_ == 0) return;
    auto it = map_.find(key);
    if (it != map_.end()) {
      it->second->second = value;
      list_.splice(list_.begin(), list_, it->second);
      return;
    }
    if (list_.size() >= capacity_) {
      map_.erase(list_.back().first);
      list_.pop_back();
    }
    list_.emplace_front(key, value);
    map_[key] = list_.begin();
  }

  void clear() {
    std::lock_guard<std::mutex> g(mutex_);
    map_.clear();
    list_.clear();
    hits_ = 0;
    misses_ = 0;
  }
  size_t size() const {
    std::lock_guard<std::mutex> g(mutex_);
    return list_.size();
  }
  size_t capacity() const { return capacity_; }
  size_t getHits() const { return hits_.load(); }
  size_t getMisses() const { return misses_.load(); }
  double getHitRate() const {
    const size_t h = hits_.load(), m = misses_.load();
    return h + m ? static_cast<double>(h) / static_cast<double>(h + m) : 0.0;
  }
  // Keys from most to least recently used (tests).
  std::vector<Key> keys() const {
    std::lock_guard<std::mutex> g(mutex_);
    std::vector<Key> k;
    for (auto& e : list_) k.push_back(e.first);
    return k;
  }

 private:
  size_t capacity_;
  std::list<std::pair<Key, Value>> list_;
  std::unordered_map<Key, typename std::list<std::pair<Key, Value>>::iterator, Hash> map_;
  mutable std::mutex mutex_;
  std::atomic<size_t> hits_{0};
  std::atomic<size_t> misses_{0};
};

struct InputKey {
  uint64_t len = 0;
  uint64_t h0 = 0, h1 = 0;
  bool operator==(const InputKey& o) const { return len == o.len && h0 == o.h0 && h1 == o.h1; }
};
struct InputKeyHash {
  size_t operator()(const InputKey& k) const { return static_cast<size_t>(k.h0 ^ (k.h1 * 0x9E3779B97F4A7C15ull)); }
};

// Per-process random secret of the input hash: which inputs collide cannot be worked out from the
// source (the reference compares whole keys; this cache keeps 128 bits of a keyed hash instead).
inline const uint64_t* cache_hash_secret() {
  static const std::array<uint64_t, 4> s = [] {
    std::random_device rd;
    std::array<uint64_t, 4> v{};
    for (auto& x : v) x = (static_cast<uint64_t>(rd()) << 32 | rd()) | 1ull;  // odd: never a zero multiplier
    return v;
  }();
  return s.data();
}

// 128-bit keyed hash of a byte string: four independent multiply-mix lanes over 64-byte blocks (the
// lanes have no dependency on each other, so a 1 MB body hashes at memory speed), folded at the
// end.  `tag` separates key domains (float bit patterns vs. raw input text).  The mix is the
// "protected" form: a lane keeps its multiplicands XORed in, so a zero product (one operand equal
// to its secret word) does not wipe the lane's history.
inline InputKey hash_bytes(const void* data, size_t bytes, uint64_t tag) {
  auto mum = [](uint64_t a, uint64_t b) {
    __uint128_t r = static_cast<__uint128_t>(a) * b;
    return static_cast<uint64_t>(r) ^ static_cast<uint64_t>(r >> 64) ^ a ^ b;
  };
  const uint64_t* sec = cache_hash_secret();
  const uint64_t k0 = sec[0], k1 = sec[1], k2 = sec[2], k3 = sec[3];
  uint64_t h[4] = {0x243F6A8885A308D3ull ^ bytes, 0x13198A2E03707344ull + bytes, 0xA4093822299F31D0ull ^ tag,
                   0x082EFA98EC4E6C89ull + tag};
  const unsigned char* p = static_cast<const unsigned char*>(data);
  size_t i = 0;
  for (; i + 64 <= bytes; i += 64) {
    uint64_t w[8];
    std::memcpy(w, p + i, 64);
    h[0] = mum(h[0] ^ w[0] ^ k0, w[1] ^ k1);
    h[1] = mum(h[1] ^ w[2] ^ k2, w[3] ^ k3);
    h[2] = mum(h[2] ^ w[4] ^ k1, w[5] ^ k2);
    h[3] = mum(h[3] ^ w[6] ^ k3, w[7] ^ k0);
  }
  for (; i + 16 <= bytes; i += 16) {
    uint64_t w0, w1;
    std::memcpy(&w0, p + i, 8);
    std::memcpy(&w1, p + i + 8, 8);
    h[0] = mum(h[0] ^ w0 ^ k0, w1 ^ k1);
    h[1] = mum(h[1] ^ w1 ^ k2, w0 ^ k3) + h[0];
  }
  uint64_t t0 = 0, t1 = 0;
  if (i < bytes) {
    unsigned char tail[16] = {0};
    std::memcpy(tail, p + i, bytes - i);
    std::memcpy(&t0, tail, 8);
    std::memcpy(&t1, tail + 8, 8);
  }
  uint64_t a = mum(h[0] ^ t0 ^ k1, h[2] ^ t1 ^ k2 ^ bytes);
  uint64_t b = mum(h[1] ^ t1 ^ k3, h[3] ^ t0 ^ k0 ^ a);
  InputKey key;
  key.len = bytes ^ (tag << 56);
  key.h0 = mum(a, k3) ^ b;
  key.h1 = mum(b, k1) ^ a;
  return key;
}

// Key of a parsed input (bit patterns of n floats).
inline InputKey hash_floats(const float* v, size_t n) { return hash_bytes(v, n * sizeof(float), 0); }
// Key of an input still in text form (device decode): byte-exact text of input_data.  Two texts
// of the same numbers spelled differently ("1" vs "1.0") are different keys: a cache miss, never
// a wrong answer.
inline InputKey hash_text(const char* s, size_t n) { return hash_bytes(s, n, 1); }

}  // namespace die
