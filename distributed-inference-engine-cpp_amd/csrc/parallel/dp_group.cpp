#include "dp_group.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <climits>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace die {

namespace {

constexpr uint64_t kMagic = 0x44494544504750ull;  // "DIEDPGP"

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Cross-process futex on a 32-bit word in shared memory (no FUTEX_PRIVATE_FLAG).
void futex_wait(std::atomic<uint32_t>* w, uint32_t expected, int timeout_ms) {
  timespec ts{timeout_ms / 1000, (timeout_ms % 1000) * 1000000L};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expected, &ts, nullptr, 0);
}
void futex_wake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

std::string shm_name(const std::string& n) { return n.empty() || n[0] != '/' ? "/" + n : n; }

}  // namespace

struct DpGroup::Control {
  std::atomic<uint64_t> magic;
  int32_t world;
  int32_t pad0;
  uint64_t arena_off, arena_bytes, gather_off, gather_bytes, total;
  std::atomic<uint64_t> arena_top;
  std::atomic<uint32_t> id_ready;
  uint32_t id_len;
  uint8_t id[256];
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> stop;
  std::atomic<uint32_t> head;  // last posted batch seq
  std::atomic<uint32_t> done_seq[kDpMaxRanks];
  std::atomic<uint32_t> done_any;
  std::atomic<uint32_t> bar_count, bar_gen;
  std::atomic<int32_t> port;
  std::atomic<uint64_t> gseq;
  std::atomic<uint32_t> subs_posted, subs_taken;
  std::atomic<uint32_t> sig_ready[kDpMaxRanks];
  std::atomic<uint32_t> sig_any;
  char sig[kDpMaxRanks][192];
  struct SubRing {
    std::atomic<uint32_t> head, tail;  // head: next slot to fill (producer), tail: next to take (leader)
    DpSub slots[kDpSubRing];
  } subq[kDpMaxRanks];
  DpBatch ring[kDpRing];
};

std::unique_ptr<DpGroup> DpGroup::create(const std::string& name, int world, size_t arena_bytes,
                                         size_t gather_bytes) {
  if (world < 1 || world > kDpMaxRanks) throw std::runtime_error("dp world size must be 1.." + std::to_string(kDpMaxRanks));
  std::unique_ptr<DpGroup> g(new DpGroup());
  g->name_ = shm_name(name);
  g->rank_ = 0;
  g->world_ = world;
  g->owner_ = true;
  const size_t ctl = round_up(sizeof(Control), 1 << 16);
  arena_bytes = round_up(arena_bytes, 1 << 16);
  gather_bytes = round_up(gather_bytes, 4096);
  g->total_ = ctl + arena_bytes + gather_bytes * world;
  int fd = shm_open(g->name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0 && errno == EEXIST) {  // stale segment from a crashed run
    shm_unlink(g->name_.c_str());
    fd = shm_open(g->name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  }
  if (fd < 0) throw std::runtime_error("shm_open(" + g->name_ + ") failed: " + std::strerror(errno));
  if (ftruncate(fd, static_cast<off_t>(g->total_)) != 0) {
    close(fd);
    shm_unlink(g->name_.c_str());
    throw std::runtime_error("ftruncate of dp segment failed: " + std::string(std::strerror(errno)));
  }
  void* p = mmap(nullptr, g->total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(g->name_.c_str());
    throw std::runtime_error("mmap of dp segment failed");
  }
  g->base_ = static_cast<uint8_t*>(p);
  g->ctl_ = new (p) Control();
  Control* c = g->ctl_;
  c->world = world;
  c->arena_off = ctl;
  c->arena_bytes = arena_bytes;
  c->gather_off = ctl + arena_bytes;
  c->gather_bytes = gather_bytes;
  c->total = g->total_;
  c->arena_top = 0;
  c->id_ready = 0;
  c->joined = 0;
  c->stop = 0;
  c->head = 0;
  for (auto& d : c->done_seq) d = 0;
  c->done_any = 0;
  c->bar_count = 0;
  c->bar_gen = 0;
  c->port = 0;
  c->gseq = 0;
  c->subs_posted = 0;
  c->subs_taken = 0;
  for (auto& r : c->sig_ready) r = 0;
  c->sig_any = 0;
  for (auto& q : c->subq) {
    q.head = 0;
    q.tail = 0;
  }
  g->arena_ = g->base_ + c->arena_off;
  g->arena_bytes_ = arena_bytes;
  g->gather_ = g->base_ + c->gather_off;
  g->gather_bytes_ = gather_bytes;
  c->magic.store(kMagic, std::memory_order_release);
  return g;
}

std::unique_ptr<DpGroup> DpGroup::attach(const std::string& name, int rank, int timeout_ms,
                                         const std::atomic<bool>* ext_stop) {
  std::unique_ptr<DpGroup> g(new DpGroup());
  g->name_ = shm_name(name);
  g->rank_ = rank;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const int fd = shm_open(g->name_.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= sizeof(Control)) {
        void* p = mmap(nullptr, static_cast<size_t>(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw std::runtime_error("mmap of dp segment failed");
        auto* c = static_cast<Control*>(p);
        if (c->magic.load(std::memory_order_acquire) == kMagic) {
          g->base_ = static_cast<uint8_t*>(p);
          g->ctl_ = c;
          g->total_ = static_cast<size_t>(st.st_size);
          g->world_ = c->world;
          g->arena_ = g->base_ + c->arena_off;
          g->arena_bytes_ = c->arena_bytes;
          g->gather_ = g->base_ + c->gather_off;
          g->gather_bytes_ = c->gather_bytes;
          if (rank < 1 || rank >= g->world_) throw std::runtime_error("dp rank out of range");
          return g;
        }
        munmap(p, static_cast<size_t>(st.st_size));
      } else {
        close(fd);
      }
    }
    if (ext_stop && ext_stop->load()) return nullptr;
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("timed out waiting for dp group " + g->name_);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

DpGroup::~DpGroup() {
  if (base_) munmap(base_, total_);
  if (owner_) shm_unlink(name_.c_str());
}

void* DpGroup::arena_alloc(size_t bytes) {
  bytes = round_up(bytes, 4096);
  const uint64_t off = ctl_->arena_top.fetch_add(bytes);
  if (off + bytes > arena_bytes_) return nullptr;
  return arena_ + off;
}

void DpGroup::publish_id(const void* id, size_t n) {
  if (n > sizeof(ctl_->id)) throw std::runtime_error("dp id too large");
  std::memcpy(ctl_->id, id, n);
  ctl_->id_len = static_cast<uint32_t>(n);
  ctl_->id_ready.store(1, std::memory_order_release);
  futex_wake(&ctl_->id_ready);
}

bool DpGroup::wait_id(void* id, size_t n, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (ctl_->id_ready.load(std::memory_order_acquire) == 0) {
    if (ctl_->stop.load() || std::chrono::steady_clock::now() > deadline) return false;
    futex_wait(&ctl_->id_ready, 0, 50);
  }
  std::memcpy(id, ctl_->id, n);
  return true;
}

void DpGroup::mark_joined() {
  ctl_->joined.fetch_add(1);
  futex_wake(&ctl_->joined);
}

bool DpGroup::wait_joined(int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const uint32_t j = ctl_->joined.load();
    if (static_cast<int>(j) >= world_ - 1) return true;
    if (std::chrono::steady_clock::now() > deadline) return false;
    futex_wait(&ctl_->joined, j, 50);
  }
}

void DpGroup::publish_signature(const std::string& sig) {
  const size_t n = std::min(sig.size(), sizeof(ctl_->sig[0]) - 1);
  std::memcpy(ctl_->sig[rank_], sig.data(), n);
  ctl_->sig[rank_][n] = 0;
  ctl_->sig_ready[rank_].store(1, std::memory_order_release);
  ctl_->sig_any.fetch_add(1, std::memory_order_release);
  futex_wake(&ctl_->sig_any);
}

bool DpGroup::check_signatures(int timeout_ms, std::string* why) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const uint32_t snap = ctl_->sig_any.load(std::memory_order_acquire);
    bool all = true;
    for (int r = 0; r < world_; ++r) all = all && ctl_->sig_ready[r].load(std::memory_order_acquire) != 0;
    if (all) break;
    if (ctl_->stop.load()) {
      if (why) *why = "data-parallel group stopped before every rank published its plan signature";
      return false;
    }
    if (std::chrono::steady_clock::now() > deadline) {
      if (why) *why = "timed out waiting for every rank's plan signature";
      return false;
    }
    futex_wait(&ctl_->sig_any, snap, 50);
  }
  for (int r = 1; r < world_; ++r)
    if (std::strcmp(ctl_->sig[r], ctl_->sig[0]) != 0) {
      if (why)
        *why = "data-parallel rank " + std::to_string(r) + " plans a different program (" + std::string(ctl_->sig[r]) +
               ") than rank 0 (" + std::string(ctl_->sig[0]) + ")";
      return false;
    }
  return true;
}

uint64_t DpGroup::post(const DpBatch& b) {
  if (b.B > kDpMaxItems) throw std::runtime_error("dp batch too large");
  const uint32_t seq = ctl_->head.load() + 1;
  // the ring slot is free once every follower finished batch seq - kDpRing
  while (true) {
    const uint32_t snap = ctl_->done_any.load();
    bool free = true;
    for (int r = 1; r < world_; ++r)
      if (seq > static_cast<uint32_t>(kDpRing) && ctl_->done_seq[r].load() < seq - kDpRing) free = false;
    if (free || ctl_->stop.load()) break;
    futex_wait(&ctl_->done_any, snap, 50);
  }
  DpBatch& slot = ctl_->ring[seq % kDpRing];
  slot.seq = seq;
  slot.B = b.B;
  slot.per = b.per;
  slot.nsub = b.nsub;
  std::memcpy(slot.subs, b.subs, sizeof(DpSubRef) * static_cast<size_t>(b.nsub));
  std::memcpy(slot.items, b.items, sizeof(DpItem) * static_cast<size_t>(b.B));
  ctl_->head.store(seq, std::memory_order_release);
  futex_wake(&ctl_->head);
  return seq;
}

bool DpGroup::next(uint64_t seq, DpBatch& out, const std::atomic<bool>* ext_stop) {
  while (true) {
    const uint32_t h = ctl_->head.load(std::memory_order_acquire);
    if (h >= seq) break;
    if (ctl_->stop.load() || (ext_stop && ext_stop->load())) return false;
    futex_wait(&ctl_->head, h, 50);
  }
  const DpBatch& slot = ctl_->ring[seq % kDpRing];
  out.seq = slot.seq;
  out.B = slot.B;
  out.per = slot.per;
  out.nsub = slot.nsub;
  std::memcpy(out.subs, slot.subs, sizeof(DpSubRef) * static_cast<size_t>(slot.nsub));
  std::memcpy(out.items, slot.items, sizeof(DpItem) * static_cast<size_t>(slot.B));
  return true;
}

void DpGroup::done(uint64_t seq) {
  ctl_->done_seq[rank_].store(static_cast<uint32_t>(seq), std::memory_order_release);
  ctl_->done_any.fetch_add(1);
  futex_wake(&ctl_->done_any);
}

bool DpGroup::push_sub(const DpSub& s) {
  if (s.n < 0 || s.n > kDpSubMax) throw std::runtime_error("dp sub-batch too large");
  auto& q = ctl_->subq[rank_];
  while (true) {  // single producer per rank (the caller serialises its own pushes)
    const uint32_t taken = ctl_->subs_taken.load(std::memory_order_acquire);
    if (q.head.load(std::memory_order_relaxed) - q.tail.load(std::memory_order_acquire) < kDpSubRing) break;
    if (ctl_->stop.load()) return false;
    futex_wait(&ctl_->subs_taken, taken, 50);
  }
  const uint32_t h = q.head.load(std::memory_order_relaxed);
  DpSub& slot = q.slots[h % kDpSubRing];
  slot.gseq = ctl_->gseq.fetch_add(1) + 1;
  slot.sub_id = s.sub_id;
  slot.n = s.n;
  slot.posted_at = ctl_->head.load(std::memory_order_acquire);
  std::memcpy(slot.items, s.items, sizeof(DpItem) * static_cast<size_t>(s.n));
  q.head.store(h + 1, std::memory_order_release);
  ctl_->subs_posted.fetch_add(1, std::memory_order_release);
  futex_wake(&ctl_->subs_posted);
  return !ctl_->stop.load();
}

uint32_t DpGroup::posted() const { return ctl_->head.load(std::memory_order_acquire); }

int DpGroup::queued_items() const {
  int n = 0;
  for (int r = 0; r < world_; ++r) {
    auto& q = ctl_->subq[r];
    const uint32_t h = q.head.load(std::memory_order_acquire);
    for (uint32_t t = q.tail.load(std::memory_order_relaxed); t != h; ++t) n += q.slots[t % kDpSubRing].n;
  }
  return n;
}

int DpGroup::peek_sub_items() const {
  int best = -1;
  uint64_t best_seq = UINT64_MAX;
  for (int r = 0; r < world_; ++r) {
    auto& q = ctl_->subq[r];
    const uint32_t t = q.tail.load(std::memory_order_relaxed);
    if (q.head.load(std::memory_order_acquire) == t) continue;
    const DpSub& s = q.slots[t % kDpSubRing];
    if (s.gseq < best_seq) {
      best_seq = s.gseq;
      best = s.n;
    }
  }
  return best;
}

bool DpGroup::pop_sub(DpSub& out, int& rank, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const uint32_t posted = ctl_->subs_posted.load(std::memory_order_acquire);
    int best = -1;
    uint64_t best_seq = UINT64_MAX;
    for (int r = 0; r < world_; ++r) {
      auto& q = ctl_->subq[r];
      const uint32_t t = q.tail.load(std::memory_order_relaxed);
      if (q.head.load(std::memory_order_acquire) == t) continue;
      const uint64_t gs = q.slots[t % kDpSubRing].gseq;
      if (gs < best_seq) {
        best_seq = gs;
        best = r;
      }
    }
    if (best >= 0) {
      auto& q = ctl_->subq[best];
      const uint32_t t = q.tail.load(std::memory_order_relaxed);
      const DpSub& s = q.slots[t % kDpSubRing];
      out.gseq = s.gseq;
      out.sub_id = s.sub_id;
      out.n = s.n;
      out.posted_at = s.posted_at;
      std::memcpy(out.items, s.items, sizeof(DpItem) * static_cast<size_t>(s.n));
      q.tail.store(t + 1, std::memory_order_release);
      ctl_->subs_taken.fetch_add(1, std::memory_order_release);
      futex_wake(&ctl_->subs_taken);
      rank = best;
      return true;
    }
    if (ctl_->stop.load()) return false;
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() <= 0) return false;
    futex_wait(&ctl_->subs_posted, posted, static_cast<int>(std::min<long long>(left.count(), 50)));
  }
}

void DpGroup::publish_port(int port) {
  ctl_->port.store(port, std::memory_order_release);
  futex_wake(reinterpret_cast<std::atomic<uint32_t>*>(&ctl_->port));
}

int DpGroup::wait_port(int timeout_ms) const {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    const int p = ctl_->port.load(std::memory_order_acquire);
    if (p > 0) return p;
    if (ctl_->stop.load() || std::chrono::steady_clock::now() > deadline) return -1;
    futex_wait(reinterpret_cast<std::atomic<uint32_t>*>(&ctl_->port), 0, 50);
  }
}

void DpGroup::stop() {
  ctl_->stop.store(1);
  futex_wake(&ctl_->head);
  futex_wake(&ctl_->done_any);
  futex_wake(&ctl_->id_ready);
  futex_wake(&ctl_->bar_gen);
  futex_wake(&ctl_->subs_posted);
  futex_wake(&ctl_->subs_taken);
}

bool DpGroup::stopping() const { return ctl_->stop.load() != 0; }

void DpGroup::barrier() {
  const uint32_t gen = ctl_->bar_gen.load(std::memory_order_acquire);
  if (static_cast<int>(ctl_->bar_count.fetch_add(1) + 1) == world_) {
    ctl_->bar_count.store(0);
    ctl_->bar_gen.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&ctl_->bar_gen);
    return;
  }
  while (ctl_->bar_gen.load(std::memory_order_acquire) == gen) {
    if (ctl_->stop.load()) throw std::runtime_error("dp group stopped during a collective");
    futex_wait(&ctl_->bar_gen, gen, 50);
  }
}

void DpGroup::all_gather_host(const void* send, void* recv, size_t bytes) {
  if (bytes > gather_bytes_) throw std::runtime_error("all_gather_host: message exceeds the gather slot");
  std::memcpy(gather_ + static_cast<size_t>(rank_) * gather_bytes_, send, bytes);
  barrier();
  for (int r = 0; r < world_; ++r)
    std::memcpy(static_cast<uint8_t*>(recv) + static_cast<size_t>(r) * bytes, gather_ + static_cast<size_t>(r) * gather_bytes_,
                bytes);
  barrier();
}

void DpGroup::broadcast_host(void* buf, size_t bytes, int root) {
  for (size_t off = 0; off < bytes; off += gather_bytes_) {
    const size_t n = std::min(gather_bytes_, bytes - off);
    if (rank_ == root) std::memcpy(gather_, static_cast<uint8_t*>(buf) + off, n);
    barrier();
    if (rank_ != root) std::memcpy(static_cast<uint8_t*>(buf) + off, gather_, n);
    barrier();
  }
}

}  // namespace die
