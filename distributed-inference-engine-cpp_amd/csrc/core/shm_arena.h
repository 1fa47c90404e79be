// POSIX shared-memory arenas for handing request bodies between co-located processes in place.
//
// The gateway receives a ~1 MB ResNet body from its client straight into a ShmArena block and
// forwards only a descriptor (X-Die-Shm: <segment>:<offset>:<length>) to a worker on the same host;
// the worker parses the body where it lies (ShmReader).  That removes the gateway->worker TCP copy
// pair (~450 us of kernel time per request on loopback, profiles/r2_gateway_cpu.md) while the wire
// protocol to remote workers stays plain HTTP/JSON.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>

namespace die {

class ShmArena {
 public:
  // Create `name` (leading '/'; must start with "/die_gw_") of `bytes`, with the pages reserved up
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

// Read-only views of arenas created by other processes, mapped once per segment name.
class ShmReader {
 public:
  // Resolve "<segment>:<offset>:<length>"; the view is followed by >= 64 readable bytes.  Returns
  // false with *error set for a malformed descriptor, a foreign segment name or a range outside it.
  bool resolve(std::string_view desc, const char** data, size_t* len, std::string* error);
  ~ShmReader();

 private:
  struct Map {
    const char* base = nullptr;
    size_t size = 0;
  };
  std::mutex mu_;
  std::unordered_map<std::string, Map> maps_;
};

}  // namespace die
