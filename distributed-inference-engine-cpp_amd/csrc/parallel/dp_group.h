// Data-parallel process group: the control plane that lets ONE worker (the leader, rank 0) fan a
// batch out over N GPUs, one process per GPU (ranks 1..N-1 are followers).
//
// Everything lives in one POSIX shared-memory segment created by the leader:
//   * a control block: RCCL unique-id exchange, join/stop flags, a ring of batch descriptors with a
//     futex doorbell, per-rank completion sequence numbers, a barrier;
//   * an input arena: the leader's request staging buffers (SamplePool) are carved from it, so a
//     follower reads its shard's inputs from the very pages the HTTP thread wrote (each process
//     hipHostRegister()s the arena, and every GPU pulls its shard over its own PCIe link -- no
//     routing through GPU 0);
//   * gather slots for the host communicator (CPU engines / tests).
// Reference: none (the reference has no intra-worker parallelism); this implements
// the north-star DP mode (BASELINE.json config 4).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace die {

constexpr int kDpMaxRanks = 16;
constexpr int kDpMaxItems = 2048;  // requests per DP batch
constexpr int kDpRing = 4;         // batch descriptors in flight

struct DpItem {
  uint64_t off = 0;  // byte offset of the item's buffer in the arena
  uint64_t len = 0;  // floats, or text bytes when is_text
  uint32_t is_text = 0;
  uint32_t pad = 0;
};

struct DpBatch {
  uint64_t seq = 0;
  int32_t B = 0;    // items in the whole batch
  int32_t per = 0;  // items per rank (ceil(B / world)); rank r owns [r*per, min(B, (r+1)*per))
  DpItem items[kDpMaxItems];
};

class DpGroup {
 public:
  // Leader: create the segment `name` (a leading '/' is added) for `world` ranks with an input
  // arena of `arena_bytes` and `gather_bytes` of host-gather space per rank.
  static std::unique_ptr<DpGroup> create(const std::string& name, int world, size_t arena_bytes,
                                         size_t gather_bytes = 1 << 20);
  // Follower: attach to an existing segment (waits up to timeout_ms for the leader to create it).
  // Returns nullptr if *ext_stop becomes true first.
  static std::unique_ptr<DpGroup> attach(const std::string& name, int rank, int timeout_ms = 60000,
                                         const std::atomic<bool>* ext_stop = nullptr);
  ~DpGroup();

  int rank() const { return rank_; }
  int world() const { return world_; }
  bool leader() const { return rank_ == 0; }

  // ---- input arena (leader allocates; offsets are valid in every process) ----
  uint8_t* arena() const { return arena_; }
  size_t arena_bytes() const { return arena_bytes_; }
  void* arena_alloc(size_t bytes);  // leader only; 4 KiB aligned bump allocation, nullptr when full
  uint64_t offset_of(const void* p) const { return static_cast<uint64_t>(static_cast<const uint8_t*>(p) - arena_); }
  void* at(uint64_t off) const { return arena_ + off; }

  // ---- bootstrap ----
  void publish_id(const void* id, size_t n);      // leader
  bool wait_id(void* id, size_t n, int timeout_ms);  // followers
  void mark_joined();                              // followers, once ready to receive batches
  bool wait_joined(int timeout_ms);                // leader: all followers joined

  // ---- batch ring ----
  // Leader: publish a batch (blocks while the ring is full, i.e. some follower still works on the
  // batch kDpRing positions back).  Returns its sequence number (1, 2, ...).
  uint64_t post(const DpBatch& b);
  // Follower: wait for batch `seq`; false when the group is stopping (or *ext_stop is set).
  bool next(uint64_t seq, DpBatch& out, const std::atomic<bool>* ext_stop = nullptr);
  // Follower: batch `seq` fully processed (its ring slot may be reused).
  void done(uint64_t seq);
  void stop();
  bool stopping() const;

  // ---- host collectives (blocking; all ranks must call in the same order) ----
  void barrier();
  // recv = concat over ranks of each rank's `bytes` (<= gather_bytes)
  void all_gather_host(const void* send, void* recv, size_t bytes);
  void broadcast_host(void* buf, size_t bytes, int root);

  const std::string& name() const { return name_; }

 private:
  DpGroup() = default;
  struct Control;
  Control* ctl_ = nullptr;
  uint8_t* base_ = nullptr;
  size_t total_ = 0;
  uint8_t* arena_ = nullptr;
  size_t arena_bytes_ = 0;
  uint8_t* gather_ = nullptr;
  size_t gather_bytes_ = 0;
  int rank_ = 0, world_ = 1;
  std::string name_;
  bool owner_ = false;
};

}  // namespace die
