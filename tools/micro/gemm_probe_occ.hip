// Where does a split (fp32-mode) 1x1-conv GEMM spend its time?  Standalone probe of the LDS-DMA
// main loop of conv_glds_kernel (MODE 0, SPLIT) on ResNet50 1x1 shapes, timed with events over a
// burst of launches, in four builds of the same loop:
//   PROBE 0  the loop as in production (DMA every K-step, three MFMAs per fragment pair)
//   PROBE 1  DMA only: no LDS fragment reads, no MFMAs
//   PROBE 2  compute only: K-step 0 is loaded once, every later K-step re-reads it from LDS
//   PROBE 3  DMA + LDS fragment reads, no MFMAs
// The epilogue (f32 tile store through LDS) is the same in all four.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/micro/gemm_probe.hip -o /tmp/gemm_probe && /tmp/gemm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ void glds16(const uint16_t* g, uint16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
template <int BKS>
__device__ __forceinline__ int swk(int row, int chunk) {
  constexpr int CPR = BKS / 8;
  return row * BKS + ((chunk ^ ((row >> 1) & (CPR - 1))) << 3);
}

struct Args {
  const uint16_t* x;  // [M][K] hi plane, lo plane xplane later
  const uint16_t* w;  // [N][K] hi, lo wplane later
  float* out;         // [M][N]
  int M, N, K;
  long long xplane, wplane;
};

// STAGES 1: issue, wait, barrier, compute per K-step.  STAGES 2: issue K-step t+1 before computing t.
template <int BM, int BN, int STAGES, int PROBE, int BK, int MINW>
__global__ __launch_bounds__(256, MINW) void probe_kernel(const Args p) {
  constexpr int CPR = BK / 8, RPI = 512 / BK, KSUB = BK / 32;
  auto sw = [](int row, int chunk) { return swk<BK>(row, chunk); };
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_ELEMS = BN * BK, B_ELEMS = BM * BK, PLANE = A_ELEMS + B_ELEMS, STAGE = 2 * PLANE;
  constexpr int GA = BN / 4 / RPI, GB = BM / 4 / RPI;
  constexpr int LDS_ELEMS = STAGES * STAGE > BM * BN * 2 ? STAGES * STAGE : BM * BN * 2;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = p.N / BN;
  const int tile = blockIdx.x;
  const int tile_m = tile / ntn, tile_n = tile - tile_m * ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = p.K / BK;
  const uint16_t* asrc[GA];
  const uint16_t* bsrc[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = wave * (BN / 4) + i * RPI + lane / CPR;
    asrc[i] = p.w + static_cast<size_t>(n0 + r) * p.K + ((lane % CPR) ^ ((r >> 1) & (CPR - 1))) * 8;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = wave * (BM / 4) + i * RPI + lane / CPR;
    const int m = min(m0 + r, p.M - 1);
    bsrc[i] = p.x + static_cast<size_t>(m) * p.K + ((lane % CPR) ^ ((r >> 1) & (CPR - 1))) * 8;
  }
  auto issue = [&](int buf, int k0) {
    uint16_t* A = lds + buf * STAGE;
    uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      glds16(asrc[i] + k0, A + (wave * (BN / 4) + i * RPI) * BK);
      glds16(asrc[i] + p.wplane + k0, A + PLANE + (wave * (BN / 4) + i * RPI) * BK);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      glds16(bsrc[i] + k0, Bt + (wave * (BM / 4) + i * RPI) * BK);
      glds16(bsrc[i] + p.xplane + k0, Bt + PLANE + (wave * (BM / 4) + i * RPI) * BK);
    }
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const uint16_t* A) {
    const uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int s = 0; s < KSUB; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[TN], bfr[TM], afl[TN], bfl[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(A + sw(wn * WN + i * 16 + (lane & 15), chunk));
        afl[i] = *reinterpret_cast<const bf16x8*>(A + PLANE + sw(wn * WN + i * 16 + (lane & 15), chunk));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + sw(wm * WM + j * 16 + (lane & 15), chunk));
        bfl[j] = *reinterpret_cast<const bf16x8*>(Bt + PLANE + sw(wm * WM + j * 16 + (lane & 15), chunk));
      }
      if constexpr (PROBE == 3) {  // reads kept alive without MFMAs
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            acc[i][j][0] += static_cast<float>(af[i][0]) + static_cast<float>(bfr[j][0]) +
                            static_cast<float>(afl[i][1]) + static_cast<float>(bfl[j][1]);
      } else {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          }
      }
    }
  };
  if constexpr (STAGES == 1) {
    for (int t = 0; t < nk; ++t) {
      if (t) __syncthreads();
      if (PROBE != 2 || t == 0) issue(0, t * BK);
      __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (PROBE != 1) compute(lds);
    }
  } else {
    constexpr int G = 2 * (GA + GB);  // DMA instructions per wave per stage
    for (int s = 0; s < STAGES - 1 && s < nk; ++s)
      if (PROBE != 2 || s == 0) issue(s, s * BK);
    for (int t = 0; t < nk; ++t) {
      // younger stages still in flight: min(STAGES - 2, nk - 1 - t)
      const int y = PROBE == 2 ? 0 : min(STAGES - 2, nk - 1 - t);
      if (y >= 2) __builtin_amdgcn_s_waitcnt(((2 * G) & 15) | (((2 * G) >> 4) << 14) | (7 << 4) | (15 << 8));
      else if (y == 1) __builtin_amdgcn_s_waitcnt((G & 15) | ((G >> 4) << 14) | (7 << 4) | (15 << 8));
      else __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + STAGES - 1 < nk && PROBE != 2) issue((t + STAGES - 1) % STAGES, (t + STAGES - 1) * BK);
      if (PROBE != 1) compute(lds + (PROBE == 2 ? 0 : (t % STAGES) * STAGE));
    }
  }
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
  __syncthreads();
  // epilogue: registers -> global f32 (row-per-lane 16-B stores, no LDS staging)
  const int lm = lane & 15, ln = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + lm, n = n0 + wn * WN + i * 16 + ln;
      if (m < p.M) *reinterpret_cast<f32x4*>(p.out + static_cast<size_t>(m) * p.N + n) = acc[i][j];
    }
}

template <int BM, int BN, int STAGES, int PROBE, int BK, int MINW>
float run(const Args& a, int reps) {
  const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((probe_kernel<BM, BN, STAGES, PROBE, BK, MINW>), dim3(tiles), dim3(256), 0, 0, a);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe_kernel<BM, BN, STAGES, PROBE, BK, MINW>), dim3(tiles), dim3(256), 0, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1000.f / reps;
}

template <int BM, int BN, int STAGES, int BK = 64, int MINW = 1>
void row(const char* name, const Args& a) {
  const int reps = 50;
  const float t0 = run<BM, BN, STAGES, 0, BK, MINW>(a, reps), t1 = run<BM, BN, STAGES, 1, BK, MINW>(a, reps);
  const float t2 = run<BM, BN, STAGES, 2, BK, MINW>(a, reps), t3 = run<BM, BN, STAGES, 3, BK, MINW>(a, reps);
  const double gflop = 2.0 * a.M * a.N * a.K * 1e-9;
  const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
  const double mb = tiles * (a.K / 64) * (BM + BN) * 64 * 4.0 / 1e6;
  std::printf("| %s | %d | %d | %d | %dx%d/%d/k%d/w%d | %d | %.1f | %.1f | %.1f | %.1f | %.0f | %.1f |\n", name, a.M, a.N, a.K, BM,
              BN, STAGES, BK, MINW, tiles, t0, t1, t2, t3, gflop / (t0 * 1e-6) * 1e-3, mb / t0);
}

int main() {
  struct Shape {
    const char* name;
    int M, N, K;
  } shapes[] = {{"s1.reduce", 100352, 64, 256}, {"s2.reduce", 25088, 128, 512}, {"s3.reduce", 6272, 256, 1024},
                {"s1.proj", 100352, 256, 64}, {"s2.proj", 25088, 512, 256}, {"s3.reduce.b20", 3920, 256, 1024}};
  size_t maxx = 0, maxw = 0, maxo = 0;
  for (auto& s : shapes) {
    maxx = std::max(maxx, static_cast<size_t>(s.M + 128) * s.K * 2);
    maxw = std::max(maxw, static_cast<size_t>(s.N) * s.K * 2);
    maxo = std::max(maxo, static_cast<size_t>(s.M + 128) * s.N);
  }
  uint16_t *x, *w;
  float* o;
  CK(hipMalloc(&x, maxx * 2));
  CK(hipMalloc(&w, maxw * 2));
  CK(hipMalloc(&o, maxo * 4));
  {
    std::vector<uint16_t> h(maxx);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint16_t>(0x3c00 + (i * 2654435761u >> 24) % 512);
    CK(hipMemcpy(x, h.data(), maxx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, h.data(), maxw * 2, hipMemcpyHostToDevice));
  }
  std::printf("| shape | M | N | K | tile/stages | blocks | full us | DMA only | compute only | DMA+reads | TFLOP/s logical | MB/us (LDS-DMA) |\n");
  std::printf("|---|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|\n");
  for (auto& s : shapes) {
    Args a{x, w, o, s.M, s.N, s.K, static_cast<long long>(s.M) * s.K, static_cast<long long>(s.N) * s.K};
    row<64, 64, 1, 64, 1>(s.name, a);
    row<64, 64, 1, 64, 5>(s.name, a);
    row<64, 64, 1, 32, 1>(s.name, a);
    row<64, 64, 1, 32, 8>(s.name, a);
    row<64, 64, 1, 32, 6>(s.name, a);
    row<64, 64, 2, 32, 4>(s.name, a);
  }
  CK(hipFree(x));
  CK(hipFree(w));
  CK(hipFree(o));
  return 0;
}
