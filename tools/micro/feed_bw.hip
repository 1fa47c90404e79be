// Operand-feed calibration: how many bytes per clock a CU pulls from an L2-resident buffer into
// (a) LDS by LDS-DMA (global_load_lds_dwordx4), (b) VGPRs by global_load_dwordx4, (c) VGPRs then
// ds_write_b128.  Each block moves `kb` KiB per iteration (the conv kernels' 32 KiB split stage),
// `blocks_per_cu` blocks resident per CU.  Prints GB/s per CU for each mode.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

template <int MODE, int KB>
__global__ __launch_bounds__(256) void feed(const uint4* src, size_t src_elems, int iters, uint4* sink) {
  __shared__ __attribute__((aligned(16))) uint4 lds[KB * 64];  // KB KiB
  const int tid = threadIdx.x;
  constexpr int PER_THREAD = KB * 64 / 256;  // uint4 per thread per iteration
  size_t base = (static_cast<size_t>(blockIdx.x) * 7919u * KB * 64) % (src_elems - KB * 64);
  base &= ~static_cast<size_t>(63);
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int it = 0; it < iters; ++it) {
    const uint4* g = src + base;
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i * 256 + tid),
                                         (__attribute__((address_space(3))) void*)(lds + i * 256 + (tid & ~63)), 16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      acc.x ^= lds[(tid * 17 + it) % (KB * 64)].x;
      __syncthreads();
    } else if constexpr (MODE == 1) {
      uint4 v[PER_THREAD];
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) v[i] = g[i * 256 + tid];
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) {
        acc.x ^= v[i].x; acc.y ^= v[i].y; acc.z ^= v[i].z; acc.w ^= v[i].w;
      }
    } else {
      uint4 v[PER_THREAD];
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) v[i] = g[i * 256 + tid];
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) lds[i * 256 + tid] = v[i];
      __syncthreads();
      acc.x ^= lds[(tid * 17 + it) % (KB * 64)].x;
      __syncthreads();
    }
    base += KB * 64;
    if (base + KB * 64 > src_elems) base = 0;
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[blockIdx.x] = acc;
}

// Ring: DEPTH stages of KB KiB in flight per block (LDS-DMA), waiting only for the oldest.
template <int DEPTH, int KB>
__global__ __launch_bounds__(256) void feed_ring(const uint4* src, size_t src_elems, int iters, uint4* sink) {
  __shared__ __attribute__((aligned(16))) uint4 lds[DEPTH * KB * 64];
  const int tid = threadIdx.x;
  constexpr int PER_THREAD = KB * 64 / 256;
  size_t base = (static_cast<size_t>(blockIdx.x) * 7919u * KB * 64) % (src_elems - KB * 64);
  base &= ~static_cast<size_t>(63);
  auto issue = [&](int slot) {
    const uint4* g = src + base;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i * 256 + tid),
                                       (__attribute__((address_space(3))) void*)(lds + slot * KB * 64 + i * 256 + (tid & ~63)),
                                       16, 0, 0);
    base += KB * 64;
    if (base + KB * 64 > src_elems) base = 0;
  };
  for (int d = 0; d < DEPTH - 1; ++d) issue(d);
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    issue((it + DEPTH - 1) % DEPTH);
    // wait until at most (DEPTH-1) stages (PER_THREAD instrs each) are outstanding
    constexpr int N = (DEPTH - 1) * PER_THREAD;
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    __syncthreads();
    acc ^= lds[(it % DEPTH) * KB * 64 + (tid * 17 + it) % (KB * 64)].x;
    __syncthreads();
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (acc == 0x12345678u) sink[blockIdx.x] = make_uint4(acc, 0, 0, 0);
}

template <int DEPTH, int KB>
double run_ring(const uint4* src, size_t n, uint4* sink, int blocks, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((feed_ring<DEPTH, KB>), dim3(blocks), dim3(256), 0, 0, src, n, 2, sink);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((feed_ring<DEPTH, KB>), dim3(blocks), dim3(256), 0, 0, src, n, iters, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return static_cast<double>(blocks) * iters * KB * 1024.0 / (ms * 1e-3) / 1e9;
}

template <int MODE, int KB>
double run(const uint4* src, size_t n, uint4* sink, int blocks, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((feed<MODE, KB>), dim3(blocks), dim3(256), 0, 0, src, n, 2, sink);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((feed<MODE, KB>), dim3(blocks), dim3(256), 0, 0, src, n, iters, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = static_cast<double>(blocks) * iters * KB * 1024.0;
  return bytes / (ms * 1e-3) / 1e9;  // GB/s total
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoi(argv[1]) : 16;  // working set (MiB): 16 = L2-ish/MALL, 2048 = HBM
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const size_t n = mb * 1024 * 1024 / 16;
  uint4* src;
  uint4* sink;
  CK(hipMalloc(&src, n * 16));
  CK(hipMemset(src, 1, n * 16));
  CK(hipMalloc(&sink, 1 << 20));
  if (argc > 2) {  // ring mode: stages in flight per block, 1 and 2 blocks per CU
    for (int bpc : {1, 2}) {
      const int blocks = cus * bpc, iters = 400;
      std::printf("ws %zu MiB blocks/CU %d ring(32K) depth1 %6.1f depth2 %6.1f depth3 %6.1f depth4 %6.1f GB/s/CU\n", mb, bpc,
                  run<0, 32>(src, n, sink, blocks, iters) / cus, run_ring<2, 32>(src, n, sink, blocks, iters) / cus,
                  run_ring<3, 32>(src, n, sink, blocks, iters) / cus,
                  bpc == 1 ? run_ring<4, 32>(src, n, sink, blocks, iters) / cus : 0.0);
    }
    return 0;
  }
  const char* names[3] = {"lds-dma", "vgpr", "vgpr+ds_write"};
  for (int bpc : {2, 4, 5, 8}) {
    const int blocks = cus * bpc;
    const int iters = 400;
    double g[3] = {run<0, 32>(src, n, sink, blocks, iters), run<1, 32>(src, n, sink, blocks, iters),
                   run<2, 32>(src, n, sink, blocks, iters)};
    for (int m = 0; m < 3; ++m)
      std::printf("ws %zu MiB blocks/CU %d %-14s %8.0f GB/s total %6.1f GB/s/CU\n", mb, bpc, names[m], g[m],
                  g[m] / cus);
  }
  return 0;
}
