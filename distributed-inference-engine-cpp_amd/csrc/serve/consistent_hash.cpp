#include "consistent_hash.h"

namespace die {

uint32_t ConsistentHash::fnv1a(const std::string& key) {
  uint32_t h = 2166136261u;
  for (char c : key) {
    // `char` is signed on x86-64: sign-extend exactly like the reference's static_cast.
    h ^= static_cast<uint32_t>(static_cast<int32_t>(c));
    h *= 16777619u;
  }
  return h;
}

void ConsistentHash::addNode(const std::string& node) {
  std::lock_guard<std::mutex> g(mutex_);
  for (int i = 0; i < virtual_nodes_; ++i) ring_[fnv1a(node + "#" + std::to_string(i))] = node;
}

void ConsistentHash::removeNode(const std::string& node) {
  std::lock_guard<std::mutex> g(mutex_);
  for (int i = 0; i < virtual_nodes_; ++i) ring_.erase(fnv1a(node + "#" + std::to_string(i)));
}

std::string ConsistentHash::getNode(const std::string& key) const {
  std::lock_guard<std::mutex> g(mutex_);
  if (ring_.empty()) return "";
  auto it = ring_.lower_bound(fnv1a(key));
  if (it == ring_.end()) it = ring_.begin();
  return it->second;
}

std::vector<std::string> ConsistentHash::getAllNodes() const {
  std::lock_guard<std::mutex> g(mutex_);
  std::vector<std::string> nodes;
  for (const auto& kv : ring_) {
    bool seen = false;
    for (const auto& n : nodes)
      if (n == kv.second) {
        seen = true;
        break;
      }
    if (!seen) nodes.push_back(kv.second);
  }
  return nodes;
}

std::map<std::string, int> ConsistentHash::getDistribution(const std::vector<std::string>& keys) const {
  std::map<std::string, int> dist;
  for (const auto& k : keys) dist[getNode(k)]++;
  return dist;
}

size_t ConsistentHash::ringSize() const {
  std::lock_guard<std::mutex> g(mutex_);
  return ring_.size();
}

}  // namespace die
