#include "comm.h"

#include <pthread.h>
#include <rccl/rccl.h>
#include <sched.h>

#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>

namespace die {

std::atomic<int> g_affinity_restores{0};

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + " failed: " + ncclGetErrorString(r));
}

class RcclComm : public Communicator {
 public:
  RcclComm(DpGroup& g, int timeout_ms) : rank_(g.rank()), world_(g.world()) {
    ncclUniqueId id;
    if (g.leader()) {
      nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
      g.publish_id(&id, sizeof(id));
    } else if (!g.wait_id(&id, sizeof(id), timeout_ms)) {
      throw std::runtime_error("timed out waiting for the RCCL unique id from rank 0");
    }
    // The communicator init may pin the calling thread to the CPUs it deems local to the GPU.  This
    // thread goes on to create the worker's reactors, parse pool and batcher, which inherit its
    // mask: restore the mask the process chose (bench.py / worker_main bind per NUMA node).
    cpu_set_t before;
    CPU_ZERO(&before);
    const bool have = pthread_getaffinity_np(pthread_self(), sizeof before, &before) == 0;
    nccl_check(ncclCommInitRank(&comm_, world_, id, rank_), "ncclCommInitRank");
    if (have) {
      cpu_set_t after;
      CPU_ZERO(&after);
      if (pthread_getaffinity_np(pthread_self(), sizeof after, &after) == 0 && !CPU_EQUAL(&before, &after)) {
        pthread_setaffinity_np(pthread_self(), sizeof before, &before);
        g_affinity_restores.fetch_add(1);
      }
    }
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* backend() const override { return "rccl"; }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t s) override {
    nccl_check(ncclBroadcast(buf, buf, bytes, ncclChar, root, comm_, s), "ncclBroadcast");
  }
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    nccl_check(ncclAllGather(send, recv, bytes, ncclChar, comm_, s), "ncclAllGather");
  }
  void group_begin() override { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() override { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }

 private:
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
};

class HostComm : public Communicator {
 public:
  explicit HostComm(DpGroup& g) : g_(g) {}
  int rank() const override { return g_.rank(); }
  int world() const override { return g_.world(); }
  const char* backend() const override { return "host"; }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t) override { g_.broadcast_host(buf, bytes, root); }
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t) override {
    g_.all_gather_host(send, recv, bytes);
  }

 private:
  DpGroup& g_;
};

}  // namespace

std::unique_ptr<Communicator> make_rccl_comm(DpGroup& g, int timeout_ms) {
  return std::make_unique<RcclComm>(g, timeout_ms);
}
std::unique_ptr<Communicator> make_host_comm(DpGroup& g) { return std::make_unique<HostComm>(g); }

int rccl_affinity_restores() { return g_affinity_restores.load(); }

}  // namespace die
