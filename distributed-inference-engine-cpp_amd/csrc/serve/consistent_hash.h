// Consistent-hash ring with virtual nodes.
//
// Bit-compatible with the reference (include/consistent_hash.h:10-24, src/consistent_hash.cpp):
// 32-bit FNV-1a over the key bytes (each `char` sign-extended to 32 bits, as the reference's
// `static_cast<uint32_t>(c)` does), `node#i` vnode names for i in [0, vnodes), an ordered ring with
// `lower_bound` + wrap-around, and a later vnode overwriting an earlier one on a hash collision.
// So `request_id -> worker` assignments match the reference for the same worker strings.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace die {

class ConsistentHash {
 public:
  explicit ConsistentHash(int virtual_nodes = 150) : virtual_nodes_(virtual_nodes) {}

  static uint32_t fnv1a(const std::string& key);

  void addNode(const std::string& node);
  void removeNode(const std::string& node);
  // Empty string when the ring is empty.
  std::string getNode(const std::string& key) const;
  // Distinct nodes in ring order (first occurrence walking the ring from hash 0); the order the
  // gateway walks for failover (src/gateway.cpp:51-59).
  std::vector<std::string> getAllNodes() const;
  std::map<std::string, int> getDistribution(const std::vector<std::string>& keys) const;
  size_t ringSize() const;
  int virtualNodes() const { return virtual_nodes_; }

 private:
  int virtual_nodes_;
  std::map<uint32_t, std::string> ring_;
  mutable std::mutex mutex_;
};

}  // namespace die
