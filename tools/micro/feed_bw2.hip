// Does the ADDRESS PATTERN of a GEMM K-step set the LDS-DMA feed rate?  (gemm_probe2 found the
// split 1x1 GEMM's DMA-only loop at ~45 GB/s per CU whether the operands sit in L2 or not, against
// ~128 GB/s per CU for contiguous 1 KiB pieces in feed_bw.hip.)
// Each block moves 32 KiB per iteration (one split 64x64 K-step: 32 LDS-DMA wave-instructions of
// 1 KiB), 2 blocks per CU, one stage (issue, wait, barrier), from an L2-sized window per block.
// Piece layouts: 8 rows x 128 B per instruction at row stride S (S = 128 B is contiguous), lane
// chunk order plain or XOR-swizzled (the GEMM's (row >> 1) & 7 permutation); plus VGPR loads of
// the same pattern (global_load_dwordx4) for comparison.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/micro/feed_bw2.hip -o tools/micro/feed_bw2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

// MODE 0: LDS-DMA, 1: VGPR loads (kept alive), 2: VGPR loads + ds_write_b128
template <int MODE, bool XOR>
__global__ __launch_bounds__(256) void feed(const uint16_t* src, long long window_elems, int stride_elems, int iters,
                                            uint4* sink) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[16384];  // 32 KiB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // this block's window: rows of `stride_elems`, 256 rows per iteration (32 instrs x 8 rows)
  const long long rows_per_it = 256;
  const long long win_rows = window_elems / stride_elems;
  const uint16_t* base = src + (static_cast<long long>(blockIdx.x) * 977 % 64) * 64;  // spread channels
  uint4 acc = make_uint4(0, 0, 0, 0);
  long long r0 = (static_cast<long long>(blockIdx.x) * 1237) % win_rows;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // 8 instructions per wave = 64 rows per wave
      const int row = wave * 64 + i * 8 + lane / 8;
      long long rr = r0 + row;
      if (rr >= win_rows) rr -= win_rows;
      const int chunk = XOR ? ((lane % 8) ^ ((row >> 1) & 7)) : lane % 8;
      const uint16_t* g = base + rr * stride_elems + chunk * 8;
      if constexpr (MODE == 0) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)(lds + (wave * 64 + i * 8) * 64), 16, 0,
                                         0);
      } else {
        const uint4 v = *reinterpret_cast<const uint4*>(g);
        if constexpr (MODE == 1) {
          acc.x ^= v.x;
          acc.y ^= v.y;
          acc.z ^= v.z;
          acc.w ^= v.w;
        } else {
          *reinterpret_cast<uint4*>(lds + (wave * 64 + i * 8) * 64 + lane * 8) = v;
        }
      }
    }
    if constexpr (MODE != 1) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      acc.x ^= reinterpret_cast<const uint32_t*>(lds)[(tid * 17 + it) % 8192];
      __syncthreads();
    }
    r0 += rows_per_it;
    if (r0 >= win_rows) r0 -= win_rows;
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[blockIdx.x] = acc;
}

template <int MODE, bool XOR>
double run(const uint16_t* src, long long win, int stride, uint4* sink, int blocks, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((feed<MODE, XOR>), dim3(blocks), dim3(256), 0, 0, src, win, stride, 2, sink);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL((feed<MODE, XOR>), dim3(blocks), dim3(256), 0, 0, src, win, stride, iters, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return static_cast<double>(blocks) * iters * 32768.0 / (ms * 1e-3) / 1e9;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const long long total = 512ll << 20;  // bytes
  uint16_t* src;
  uint4* sink;
  CK(hipMalloc(&src, total));
  CK(hipMemset(src, 1, total));
  CK(hipMalloc(&sink, 1 << 20));
  std::printf("| window MiB | row stride B | blocks/CU | DMA plain | DMA xor | VGPR xor | VGPR+ds_write xor | (GB/s per CU) |\n");
  std::printf("|---:|---:|---:|---:|---:|---:|---:|---|\n");
  for (long long win_mb : {2ll, 24ll}) {
    for (int stride_b : {128, 512, 1024, 2048, 4096}) {
      for (int bpc : {2, 4}) {
        const long long win = (win_mb << 20) / 2;
        const int st = stride_b / 2, blocks = cus * bpc, iters = 200;
        std::printf("| %lld | %d | %d | %.1f | %.1f | %.1f | %.1f | |\n", win_mb, stride_b, bpc,
                    run<0, false>(src, win, st, sink, blocks, iters) / cus, run<0, true>(src, win, st, sink, blocks, iters) / cus,
                    run<1, true>(src, win, st, sink, blocks, iters) / cus, run<2, true>(src, win, st, sink, blocks, iters) / cus);
      }
    }
  }
  return 0;
}
