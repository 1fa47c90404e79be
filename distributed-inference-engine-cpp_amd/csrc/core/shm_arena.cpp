#include "shm_arena.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <random>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <string_view>

namespace die {

namespace {
constexpr size_t kGrain = 4096;
size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
// "/die_gw_<...>_<16 hex digits>": the trailing random token makes a segment name unguessable, so a
// descriptor can only come from the gateway that created the arena (shm_arena_name).
bool valid_name(const std::string& n) {
  if (n.rfind("/die_gw_", 0) != 0 || n.find('/', 1) != std::string::npos || n.size() >= 200) return false;
  const size_t u = n.rfind('_');
  if (u == std::string::npos || n.size() - u - 1 != 16) return false;
  for (size_t i = u + 1; i < n.size(); ++i)
    if (!std::isxdigit(static_cast<unsigned char>(n[i]))) return false;
  return true;
}
}  // namespace

std::string shm_arena_name(const std::string& stem) {
  std::random_device rd;
  const uint64_t token = (static_cast<uint64_t>(rd()) << 32) ^ rd();
  char hex[17];
  std::snprintf(hex, sizeof hex, "%016llx", static_cast<unsigned long long>(token));
  return "/die_gw_" + stem + "_" + hex;
}

std::shared_ptr<ShmArena> ShmArena::create(const std::string& name, size_t bytes, std::string* error) {
  auto fail = [&](const std::string& why) -> std::shared_ptr<ShmArena> {
    if (error) *error = why;
    return nullptr;
  };
  if (!valid_name(name)) return fail("bad shm arena name " + name);
  bytes = round_up(bytes, 1 << 20);
  shm_unlink(name.c_str());
  const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return fail(std::string("shm_open: ") + std::strerror(errno));
  if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
    const int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    return fail(std::string("ftruncate: ") + std::strerror(e));
  }
  const int fe = posix_fallocate(fd, 0, static_cast<off_t>(bytes));
  if (fe != 0) {
    close(fd);
    shm_unlink(name.c_str());
    return fail(std::string("posix_fallocate: ") + std::strerror(fe));
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    return fail("mmap of shm arena failed");
  }
  std::shared_ptr<ShmArena> a(new ShmArena());
  a->name_ = name;
  a->base_ = static_cast<char*>(p);
  a->size_ = bytes;
  a->free_[0] = bytes;
  return a;
}

ShmArena::~ShmArena() {
  if (base_) munmap(base_, size_);
  if (!name_.empty()) shm_unlink(name_.c_str());
}

long long ShmArena::alloc(size_t bytes) {
  bytes = round_up(std::max<size_t>(bytes, 1), kGrain);
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = free_.begin(); it != free_.end(); ++it) {
    if (it->second < bytes) continue;
    const size_t off = it->first, left = it->second - bytes;
    free_.erase(it);
    if (left) free_[off + bytes] = left;
    used_[off] = bytes;
    in_use_ += bytes;
    return static_cast<long long>(off);
  }
  return -1;
}

void ShmArena::free(long long off_) {
  if (off_ < 0) return;
  const size_t off = static_cast<size_t>(off_);
  std::lock_guard<std::mutex> g(mu_);
  auto u = used_.find(off);
  if (u == used_.end()) return;
  size_t start = off, len = u->second;
  in_use_ -= len;
  used_.erase(u);
  auto next = free_.lower_bound(start);
  if (next != free_.end() && next->first == start + len) {  // merge with the following hole
    len += next->second;
    next = free_.erase(next);
  }
  if (next != free_.begin()) {  // merge with the preceding hole
    auto prev = std::prev(next);
    if (prev->first + prev->second == start) {
      start = prev->first;
      len += prev->second;
      free_.erase(prev);
    }
  }
  free_[start] = len;
}

size_t ShmArena::in_use() const {
  std::lock_guard<std::mutex> g(mu_);
  return in_use_;
}

bool ShmReader::resolve(std::string_view desc, const char** data, size_t* len, std::string* error,
                        std::shared_ptr<const void>* keep) {
  const size_t c2 = desc.rfind(':');
  const size_t c1 = c2 == std::string_view::npos || c2 == 0 ? std::string_view::npos : desc.rfind(':', c2 - 1);
  if (c1 == std::string_view::npos) {
    *error = "malformed shm descriptor";
    return false;
  }
  const std::string name(desc.substr(0, c1));
  char* e1 = nullptr;
  char* e2 = nullptr;
  const std::string so(desc.substr(c1 + 1, c2 - c1 - 1)), sl(desc.substr(c2 + 1));
  const unsigned long long off = std::strtoull(so.c_str(), &e1, 10), n = std::strtoull(sl.c_str(), &e2, 10);
  if (!valid_name(name) || so.empty() || sl.empty() || *e1 || *e2) {
    *error = "malformed shm descriptor";
    return false;
  }
  std::shared_ptr<const Map> m;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = maps_.find(name);
    if (it == maps_.end()) {
      const int fd = shm_open(name.c_str(), O_RDONLY, 0);
      if (fd < 0) {
        *error = "cannot open shm segment " + name;
        return false;
      }
      struct stat st;
      if (fstat(fd, &st) != 0 || st.st_size <= 0) {
        close(fd);
        *error = "cannot stat shm segment " + name;
        return false;
      }
      void* p = mmap(nullptr, static_cast<size_t>(st.st_size), PROT_READ, MAP_SHARED, fd, 0);
      close(fd);
      if (p == MAP_FAILED) {
        *error = "cannot map shm segment " + name;
        return false;
      }
      // A new gateway arena: drop views of arenas whose segment is gone (a restarted gateway's
      // old arena is unlinked; without this every worker would keep its pages pinned).  In-flight
      // parses hold their own reference, so the unmap waits for them.
      for (auto o = maps_.begin(); o != maps_.end();) {
        const int ofd = shm_open(o->first.c_str(), O_RDONLY, 0);
        if (ofd < 0 && errno == ENOENT) {
          o = maps_.erase(o);
          unmapped_++;
          continue;
        }
        if (ofd >= 0) close(ofd);
        ++o;
      }
      auto map = std::shared_ptr<Map>(new Map{static_cast<const char*>(p), static_cast<size_t>(st.st_size)}, [](Map* mp) {
        munmap(const_cast<char*>(mp->base), mp->size);
        delete mp;
      });
      it = maps_.emplace(name, std::move(map)).first;
    }
    m = it->second;
  }
  if (off > m->size || n > m->size - off || m->size - off - n < 64) {
    *error = "shm range outside the segment";
    return false;
  }
  *data = m->base + off;
  *len = static_cast<size_t>(n);
  if (keep) *keep = m;
  return true;
}

size_t ShmReader::mapped() const {
  std::lock_guard<std::mutex> g(mu_);
  return maps_.size();
}

ShmReader::~ShmReader() = default;

}  // namespace die
