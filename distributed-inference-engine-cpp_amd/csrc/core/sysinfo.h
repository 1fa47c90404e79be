// CPU budget of this process: min(affinity mask size, cgroup v2 cpu.max quota).  GPU boxes expose
// the whole machine in the affinity mask (hundreds of CPUs) but enforce a quota of ~16 CPUs per
// GPU; sizing thread pools from hardware_concurrency() there oversubscribes the quota.  When
// several ranks share one node (one process per GPU), the launcher sets DIE_CPUS to this
// process's share (native.bind_local_cpus).
#pragma once

#include <sched.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>

namespace die {

// HIP runtime environment of a serving process; call first thing in main(), before any HIP call
// (the runtime reads it once, at initialisation).  GPU_MAX_HW_QUEUES >= 8: HIP shares hardware
// queues between streams beyond that limit (default 4, also what the GPU boxes export), and the
// engine's 3-4 streams plus an RCCL communicator's internal ones then serialise copies behind
// kernels (data-parallel ranks lost 13-23 % of throughput at 4; profiles/r3_rccl_hw_queues.md).
// Values below 8 are raised; DIE_HIP_HW_QUEUES sets it explicitly (same rule as die_amd/__init__.py).
inline void configure_hip_runtime_env() {
  if (const char* want = std::getenv("DIE_HIP_HW_QUEUES"); want && *want) {
    setenv("GPU_MAX_HW_QUEUES", want, 1);
  } else {
    const char* cur = std::getenv("GPU_MAX_HW_QUEUES");
    if (!cur || std::atoi(cur) < 8) setenv("GPU_MAX_HW_QUEUES", "8", 1);
  }
  setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);
}

inline int available_cpus() {
  static const int n = [] {
    int cpus = static_cast<int>(std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = CPU_COUNT(&set);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[64] = {0};
      long period = 0;
      if (std::fscanf(f, "%63s %ld", quota, &period) == 2 && period > 0 && quota[0] != 'm') {
        const double q = std::atof(quota) / static_cast<double>(period);
        if (q > 0) cpus = std::min(cpus, static_cast<int>(std::ceil(q)));
      }
      std::fclose(f);
    }
    if (const char* e = std::getenv("DIE_CPUS")) {
      const int share = std::atoi(e);
      if (share > 0) cpus = std::min(cpus, share);
    }
    return cpus < 1 ? 1 : cpus;
  }();
  return n;
}

}  // namespace die
