// POSIX shared-memory arenas for handing request bodies between co-located processes in place.
//
// The gateway receives a ~1 MB ResNet body from its client straight into a ShmArena block and
// forwards only a descriptor (X-Die-Shm: <segment>:<offset>:<length>) to a worker on the same host;
// the worker parses the body where it lies (ShmReader).  That removes the gateway->worker TCP copy
// pair (~450 us of kernel time per request on loopback, profiles/r2_gateway_cpu.md) while the wire
// protocol to remote workers stays plain HTTP/JSON.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>

namespace die {

// A fresh arena name "/die_gw_<stem>_<16 hex digits of a random token>".  Workers only accept
// descriptors of names in this form, so another client cannot point a worker at a guessed segment.
std::string shm_arena_name(const std::string& stem);

class ShmArena {
 public:
  // Create `name` (from shm_arena_name) of `bytes`, with the pages reserved up
  // front (posix_fallocate), so a full /dev/shm fails here instead of faulting later.  Returns
  // nullptr (and sets *error) when shared memory is unavailable.
  static std::shared_ptr<ShmArena> create(const std::string& name, size_t bytes, std::string* error = nullptr);
  ~ShmArena();

  // 4 KiB-granular first-fit allocation; returns the offset, or -1 when full.
  long long alloc(size_t bytes);
  void free(long long off);
  char* base() const { return base_; }
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }
  size_t in_use() const;

 private:
  ShmArena() = default;
  std::string name_;
  char* base_ = nullptr;
  size_t size_ = 0;
  mutable std::mutex mu_;
  std::map<size_t, size_t> free_;        // offset -> bytes
  std::unordered_map<size_t, size_t> used_;  // offset -> bytes
  size_t in_use_ = 0;
};

// Read-only views of arenas created by other processes, mapped once per segment name.  Views of
// segments that no longer exist are unmapped when a new segment is first seen.
class ShmReader {
 public:
  // Resolve "<segment>:<offset>:<length>"; the view is followed by >= 64 readable bytes and stays
  // valid while *keep (if given) is held.  Returns false with *error set for a malformed
  // descriptor, a foreign segment name or a range outside it.
  bool resolve(std::string_view desc, const char** data, size_t* len, std::string* error,
               std::shared_ptr<const void>* keep = nullptr);
  size_t mapped() const;
  long long unmapped() const { return unmapped_.load(); }
  ~ShmReader();

 private:
  struct Map {
    const char* base = nullptr;
    size_t size = 0;
  };
  mutable std::mutex mu_;
  std::unordered_map<std::string, std::shared_ptr<const Map>> maps_;
  std::atomic<long long> unmapped_{0};
};

}  // namespace die
