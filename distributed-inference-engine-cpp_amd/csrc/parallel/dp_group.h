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
//   * gather slots for the host communicator (CPU engines / tests);
//   * per-rank sub-batch rings: EVERY rank's worker ingests HTTP (the ranks share one listening port
//     through SO_REUSEPORT), parses into the arena and queues its requests as a sub-batch; the
//     leader's dispatcher merges queued sub-batches (oldest first) into one DP batch, so no single
//     process's ingest caps an N-GPU worker.
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
constexpr int kDpSubMax = 256;     // requests per sub-batch (one rank's local batch)
constexpr int kDpSubRing = 32;     // sub-batches queued per rank (a rank pushes whatever it has, eagerly)
constexpr int kDpMaxSubs = 256;    // sub-batches merged into one DP batch

struct DpItem {
  uint64_t off = 0;  // byte offset of the item's buffer in the arena
  uint64_t len = 0;  // floats, or text bytes when is_text
  uint32_t is_text = 0;  // 1 = raw JSON number text, 2 = 4-bit packed text (core/textpack.h)
  uint32_t pad = 0;
};

// Where a rank's sub-batch sits inside a DP batch: items [start, start + n).
struct DpSubRef {
  int32_t rank = 0;
  uint32_t sub_id = 0;
  int32_t start = 0;
  int32_t n = 0;
};

struct DpBatch {
  uint64_t seq = 0;
  int32_t B = 0;    // items in the whole batch
  int32_t per = 0;  // items per rank (ceil(B / world)); rank r computes [r*per, min(B, (r+1)*per))
  int32_t nsub = 0;
  int32_t pad = 0;
  DpSubRef subs[kDpMaxSubs];
  DpItem items[kDpMaxItems];
};

struct DpSub {
  uint64_t gseq = 0;  // group-wide queue order (the dispatcher takes the oldest first)
  uint32_t sub_id = 0;
  int32_t n = 0;
  uint32_t posted_at = 0;  // DP batches the leader had posted when this sub-batch was queued (fairness)
  DpItem items[kDpSubMax];
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
  void* arena_alloc(size_t bytes);  // any rank (atomic bump in the segment); 4 KiB aligned, nullptr when full
  uint64_t offset_of(const void* p) const { return static_cast<uint64_t>(static_cast<const uint8_t*>(p) - arena_); }
  void* at(uint64_t off) const { return arena_ + off; }

  // ---- bootstrap ----
  void publish_id(const void* id, size_t n);      // leader
  bool wait_id(void* id, size_t n, int timeout_ms);  // followers
  void mark_joined();                              // followers, once ready to receive batches
  bool wait_joined(int timeout_ms);                // leader: all followers joined
  // Plan signature (model, precision, local batch, ...): every rank publishes its own, then
  // check_signatures waits for all of them and returns false (with *why) on any mismatch, before
  // a collective could run with different buffer sizes on different ranks.
  void publish_signature(const std::string& sig);
  bool check_signatures(int timeout_ms, std::string* why);

  // ---- batch ring ----
  // Leader: publish a batch (blocks while the ring is full, i.e. some follower still works on the
  // batch kDpRing positions back).  Returns its sequence number (1, 2, ...).
  uint64_t post(const DpBatch& b);
  // Follower: wait for batch `seq`; false when the group is stopping (or *ext_stop is set).
  bool next(uint64_t seq, DpBatch& out, const std::atomic<bool>* ext_stop = nullptr);
  // Follower: batch `seq` fully processed (its ring slot may be reused).
  void done(uint64_t seq);

  // ---- sub-batch queues (every rank produces, the leader consumes) ----
  // Queue a sub-batch of this rank (blocks while its ring is full); false when stopping.
  bool push_sub(const DpSub& s);
  // Leader: take the oldest queued sub-batch of any rank; waits up to timeout_ms (false if none).
  bool pop_sub(DpSub& out, int& rank, int timeout_ms);
  // Leader: oldest queued sub-batch's item count without taking it (-1 when none).
  int peek_sub_items() const;
  // Leader: items in every queued sub-batch of every rank (a snapshot; relaxed reads).
  int queued_items() const;
  // DP batches posted so far (the leader's last posted seq).
  uint32_t posted() const;

  // ---- shared listening port (SO_REUSEPORT ingest on every rank) ----
  void publish_port(int port);
  int wait_port(int timeout_ms) const;
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
