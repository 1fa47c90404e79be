// Collective communicator for the data-parallel engine.
//   * RCCL (ncclBroadcast / ncclAllGather on device buffers, enqueued on a HIP stream): the
//     production path -- weights broadcast once from GPU 0, logits all-gathered every batch over
//     xGMI.  Bootstrap: the leader's ncclUniqueId travels through the DpGroup segment.
//   * host: the same two collectives over host buffers through the DpGroup segment (CPU engines
//     and the multi-process CPU tests; the SURVEY §2.5 "fake communicator").
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>

#include "dp_group.h"

namespace die {

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual const char* backend() const = 0;
  // Device buffers for RCCL, host buffers for the host communicator (which ignores `stream` and
  // completes before returning).  All ranks call collectives in the same order.
  virtual void broadcast(void* buf, size_t bytes, int root, hipStream_t stream) = 0;
  virtual void all_gather(const void* send, void* recv, size_t bytes_per_rank, hipStream_t stream) = 0;
  // Collectives issued between group_begin() and group_end() go out as ONE fused operation (RCCL:
  // ncclGroupStart / ncclGroupEnd -- one launch and one latency for a batch's logits + status
  // gathers).  The host communicator runs them one by one.
  virtual void group_begin() {}
  virtual void group_end() {}
};

// Collective constructor: every rank of `g` must call it (after hipSetDevice on its GPU).
std::unique_ptr<Communicator> make_rccl_comm(DpGroup& g, int timeout_ms = 120000);
std::unique_ptr<Communicator> make_host_comm(DpGroup& g);
// Times an RCCL communicator init changed the calling thread's CPU mask (restored afterwards).
int rccl_affinity_restores();

}  // namespace die
