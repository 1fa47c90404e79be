// Two waves per SIMD for the split GEMM main loop?  gemm_probe_vit found the 128x128 1-stage loop's
// compute-only and DMA-only times each ~2/3 of the full time (one wave per SIMD per block: a wave's
// LDS-read latency, its DMA waits and the barrier are exposed; overlap only comes from a second
// block).  Here a block has WAVES = 4 or 8 waves (8 = two per SIMD: while one waits, the other
// issues MFMAs) over the same tile, a STAGES-deep LDS-DMA ring of BK-wide K-steps with counted
// vmcnt waits, and every wave shares the DMA issue.  PROBE 0 full, 1 DMA only, 2 compute only.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/micro/gemm_probe3.hip -o tools/micro/gemm_probe3
#include <hip/hip_runtime.h>

#include <algorithm>
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
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

struct Args {
  const uint16_t* x;
  const uint16_t* w;
  float* out;
  int M, N, K;
  long long xplane, wplane;
};

template <int BM, int BN, int WAVES, int STAGES, int BK, int PROBE>
__global__ __launch_bounds__(WAVES * 64) void g3(const Args p) {
  constexpr int NT = WAVES * 64;
  constexpr int WGM = 2, WGN = WAVES / 2;  // wave grid over the tile
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int CPR = BK / 8, RPI = 512 / BK, KSUB = BK / 32;
  constexpr int A_ELEMS = BN * BK, B_ELEMS = BM * BK, PLANE = A_ELEMS + B_ELEMS, STAGE = 2 * PLANE;
  constexpr int GA = BN / WAVES / RPI, GB = BM / WAVES / RPI, G = 2 * (GA + GB);
  static_assert(GA >= 1 && GB >= 1, "every wave loads whole pieces");
  __shared__ __attribute__((aligned(16))) uint16_t lds[STAGES * STAGE];
  auto sw = [](int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & (CPR - 1))) << 3); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int ntn = p.N / BN;
  const int tile = blockIdx.x, tm = tile / ntn, tn = tile - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN, nk = p.K / BK;
  const uint16_t* asrc[GA];
  const uint16_t* bsrc[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = wave * (BN / WAVES) + i * RPI + lane / CPR;
    asrc[i] = p.w + static_cast<size_t>(n0 + r) * p.K + ((lane % CPR) ^ ((r >> 1) & (CPR - 1))) * 8;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = wave * (BM / WAVES) + i * RPI + lane / CPR;
    bsrc[i] = p.x + static_cast<size_t>(min(m0 + r, p.M - 1)) * p.K + ((lane % CPR) ^ ((r >> 1) & (CPR - 1))) * 8;
  }
  auto issue = [&](int slot, int k0) {
    uint16_t* A = lds + slot * STAGE;
    uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      glds16(asrc[i] + k0, A + (wave * (BN / WAVES) + i * RPI) * BK);
      glds16(asrc[i] + p.wplane + k0, A + PLANE + (wave * (BN / WAVES) + i * RPI) * BK);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      glds16(bsrc[i] + k0, Bt + (wave * (BM / WAVES) + i * RPI) * BK);
      glds16(bsrc[i] + p.xplane + k0, Bt + PLANE + (wave * (BM / WAVES) + i * RPI) * BK);
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
      bf16x8 af[TN], afl[TN], bfr[TM], bfl[TM];
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
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
  };
  if constexpr (STAGES == 1) {
    for (int t = 0; t < nk; ++t) {
      if (t) __syncthreads();
      if (PROBE != 2 || t == 0) issue(0, t * BK);
      wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (PROBE != 1) compute(lds);
    }
  } else {
    for (int s = 0; s < STAGES - 1 && s < nk; ++s)
      if (PROBE != 2 || s == 0) issue(s, s * BK);
    for (int t = 0; t < nk; ++t) {
      const int y = PROBE == 2 ? 0 : min(STAGES - 2, nk - 1 - t);
      if (y >= 2) wait_vm<2 * G>();
      else if (y == 1) wait_vm<G>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + STAGES - 1 < nk && PROBE != 2) issue((t + STAGES - 1) % STAGES, (t + STAGES - 1) * BK);
      if (PROBE != 1) compute(lds + (PROBE == 2 ? 0 : (t % STAGES) * STAGE));
    }
  }
  wait_vm<0>();
  const int lm = lane & 15, ln = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + lm, n = n0 + wn * WN + i * 16 + ln;
      if (m < p.M) *reinterpret_cast<f32x4*>(p.out + static_cast<size_t>(m) * p.N + n) = acc[i][j];
    }
}

template <int BM, int BN, int WAVES, int STAGES, int BK, int PROBE>
float run(const Args& a, int reps) {
  const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((g3<BM, BN, WAVES, STAGES, BK, PROBE>), dim3(tiles), dim3(WAVES * 64), 0, 0, a);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((g3<BM, BN, WAVES, STAGES, BK, PROBE>), dim3(tiles), dim3(WAVES * 64), 0, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

template <int BM, int BN, int WAVES, int STAGES, int BK>
void row(const char* name, const Args& a) {
  const int reps = 30;
  const float t0 = run<BM, BN, WAVES, STAGES, BK, 0>(a, reps), t1 = run<BM, BN, WAVES, STAGES, BK, 1>(a, reps);
  const float t2 = run<BM, BN, WAVES, STAGES, BK, 2>(a, reps);
  const double gflop = 2.0 * a.M * a.N * a.K * 1e-9;
  std::printf("| %s | %d | %d | %d | %dx%d | %d | %d | k%d | %.1f | %.1f | %.1f | %.0f |\n", name, a.M, a.N, a.K, BM, BN,
              WAVES, STAGES, BK, t0, t1, t2, gflop / (t0 * 1e-6) * 1e-3);
}

int main() {
  struct Shape {
    const char* name;
    int M, N, K;
  } shapes[] = {{"vit.mlp1.b32", 6304, 3072, 768}, {"vit.mlp1.b24", 4728, 3072, 768}, {"vit.qkv.b24", 4728, 2304, 768},
                {"vit.mlp2.b24", 4728, 768, 3072}};
  size_t maxx = 0, maxw = 0, maxo = 0;
  for (auto& s : shapes) {
    maxx = std::max(maxx, static_cast<size_t>(s.M + 256) * s.K * 2);
    maxw = std::max(maxw, static_cast<size_t>(s.N) * s.K * 2);
    maxo = std::max(maxo, static_cast<size_t>(s.M + 256) * s.N);
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
  std::printf("| shape | M | N | K | tile | waves | stages | K-step | full us | DMA only | compute only | TFLOP/s logical |\n");
  std::printf("|---|---:|---:|---:|---|---:|---:|---|---:|---:|---:|---:|\n");
  for (auto& s : shapes) {
    Args a{x, w, o, s.M, s.N, s.K, static_cast<long long>(s.M) * s.K, static_cast<long long>(s.N) * s.K};
    row<128, 128, 4, 1, 64>(s.name, a);
    row<256, 256, 8, 2, 32>(s.name, a);
    row<256, 256, 8, 1, 32>(s.name, a);
    if (s.N % 256 == 0) row<128, 256, 8, 2, 32>(s.name, a);
  }
  CK(hipFree(x));
  CK(hipFree(w));
  CK(hipFree(o));
  return 0;
}
