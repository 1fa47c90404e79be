// Persistent, continuous-ring split GEMM probe (follow-up of gemm_probe.hip).
// G = CUs x bpc blocks; block L (XCD-remapped) owns iterations [L*I/G, (L+1)*I/G) of the global
// (tile, K-step) space (stream-K order: a tile's K-steps are contiguous), and ONE LDS ring of STAGES
// slots runs across tile boundaries, so the loads of the next tile overlap the last K-steps of the
// current one.  Fragments of both 32-wide substeps are read up front each K-step.  Partial tiles are
// stored as they are (timing only: no fix-up).  PROBE 0 full, 1 DMA only, 2 compute only.
// `hot` = every A/B row index wraps inside 512 rows (L2-resident operands).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/micro/gemm_probe2.hip -o tools/micro/gemm_probe2
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

constexpr int BK = 64;

__device__ __forceinline__ void glds16(const uint16_t* g, uint16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
__device__ __forceinline__ int sw(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
template <int G, int J>
__device__ __forceinline__ void wait_stages(int j) {
  if constexpr (J == 0) {
    wait_vmcnt<0>();
  } else {
    if (j >= J) wait_vmcnt<G * J>();
    else wait_stages<G, J - 1>(j);
  }
}

struct Args {
  const uint16_t* x;
  const uint16_t* w;
  float* out;
  int M, N, K, hot;
  long long xplane, wplane;
};

template <int BM, int BN, int STAGES, int PROBE>
__global__ __launch_bounds__(256) void pgemm(const Args p) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_ELEMS = BN * BK, B_ELEMS = BM * BK, PLANE = A_ELEMS + B_ELEMS, STAGE = 2 * PLANE;
  constexpr int GA = BN / 4 / 8, GB = BM / 4 / 8, GI = 2 * (GA + GB);
  __shared__ __attribute__((aligned(16))) uint16_t lds[STAGES * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = p.N / BN, ntm = (p.M + BM - 1) / BM, nk = p.K / BK;
  const long long I = static_cast<long long>(ntm) * ntn * nk;
  const int G = gridDim.x, b = blockIdx.x;
  const int L = (b & 7) * (G >> 3) + (b >> 3);  // same-XCD blocks own adjacent ranges (G % 8 == 0)
  const long long it0 = I * L / G, it1 = I * (L + 1) / G;
  if (it0 >= it1) return;
  const bool nfast = static_cast<long long>(p.N) <= static_cast<long long>(p.M);
  auto tile_of = [&](long long it, int& tm, int& tn, int& ks) {
    const long long t = it / nk;
    ks = static_cast<int>(it - t * nk);
    if (nfast) {
      tm = static_cast<int>(t / ntn);
      tn = static_cast<int>(t - static_cast<long long>(tm) * ntn);
    } else {
      tn = static_cast<int>(t / ntm);
      tm = static_cast<int>(t - static_cast<long long>(tn) * ntm);
    }
  };
  // per-lane row / chunk of the DMA pieces
  int arow[GA], brow[GB], achk[GA], bchk[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    arow[i] = wave * (BN / 4) + i * 8 + lane / 8;
    achk[i] = ((lane % 8) ^ ((arow[i] >> 1) & 7)) * 8;
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    brow[i] = wave * (BM / 4) + i * 8 + lane / 8;
    bchk[i] = ((lane % 8) ^ ((brow[i] >> 1) & 7)) * 8;
  }
  auto issue = [&](long long it, int slot) {
    int tm, tn, ks;
    tile_of(it, tm, tn, ks);
    uint16_t* A = lds + slot * STAGE;
    uint16_t* Bt = A + A_ELEMS;
    const int k0 = ks * BK;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const uint16_t* s = p.w + static_cast<size_t>(tn * BN + arow[i]) * p.K + achk[i] + k0;
      glds16(s, A + (wave * (BN / 4) + i * 8) * BK);
      glds16(s + p.wplane, A + PLANE + (wave * (BN / 4) + i * 8) * BK);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      int m = min(tm * BM + brow[i], p.M - 1);
      if (p.hot) m &= 511;
      const uint16_t* s = p.x + static_cast<size_t>(m) * p.K + bchk[i] + k0;
      glds16(s, Bt + (wave * (BM / 4) + i * 8) * BK);
      glds16(s + p.xplane, Bt + PLANE + (wave * (BM / 4) + i * 8) * BK);
    }
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const uint16_t* A) {
    const uint16_t* Bt = A + A_ELEMS;
    bf16x8 af[2][TN], bfr[2][TM], afl[2][TN], bfl[2][TM];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        af[s][i] = *reinterpret_cast<const bf16x8*>(A + sw(wn * WN + i * 16 + (lane & 15), chunk));
        afl[s][i] = *reinterpret_cast<const bf16x8*>(A + PLANE + sw(wn * WN + i * 16 + (lane & 15), chunk));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        bfr[s][j] = *reinterpret_cast<const bf16x8*>(Bt + sw(wm * WM + j * 16 + (lane & 15), chunk));
        bfl[s][j] = *reinterpret_cast<const bf16x8*>(Bt + PLANE + sw(wm * WM + j * 16 + (lane & 15), chunk));
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[s][i], bfr[s][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s][i], bfl[s][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s][i], bfr[s][j], acc[i][j], 0, 0, 0);
        }
  };
  const long long n = it1 - it0;
  const int pre = static_cast<int>(std::min<long long>(STAGES - 1, n));
  for (int s = 0; s < pre; ++s)
    if (PROBE != 2 || s == 0) issue(it0 + s, s);
  int rd = 0, wr = STAGES - 1;
  for (long long j = 0; j < n; ++j) {
    if (PROBE == 2) {
      wait_vmcnt<0>();
    } else {
      const long long left = n - 1 - j;  // younger issues still outstanding: min(STAGES-2, left)
      wait_stages<GI, STAGES - 2>(static_cast<int>(std::min<long long>(left, STAGES - 2)));
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (j + STAGES - 1 < n && PROBE != 2) issue(it0 + j + STAGES - 1, wr);
    wr = wr + 1 == STAGES ? 0 : wr + 1;
    const uint16_t* A = lds + (PROBE == 2 ? 0 : rd) * STAGE;
    rd = rd + 1 == STAGES ? 0 : rd + 1;
    if (PROBE != 1) compute(A);
    int tm, tn, ks;
    tile_of(it0 + j, tm, tn, ks);
    if (ks == nk - 1 || j == n - 1) {  // tile (or this block's share of it) done: store, reset
      const int lm = lane & 15, ln = (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int q = 0; q < TM; ++q) {
          const int m = tm * BM + wm * WM + q * 16 + lm, nn = tn * BN + wn * WN + i * 16 + ln;
          if (m < p.M) *reinterpret_cast<f32x4*>(p.out + static_cast<size_t>(m) * p.N + nn) = acc[i][q];
          acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  }
  wait_vmcnt<0>();
}

template <int BM, int BN, int STAGES, int PROBE>
float run(const Args& a, int grid, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((pgemm<BM, BN, STAGES, PROBE>), dim3(grid), dim3(256), 0, 0, a);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((pgemm<BM, BN, STAGES, PROBE>), dim3(grid), dim3(256), 0, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1000.f / reps;
}

template <int BM, int BN, int STAGES>
void row(const char* name, const Args& a, int cus, int bpc) {
  const int reps = 50, grid = cus * bpc;
  const float t0 = run<BM, BN, STAGES, 0>(a, grid, reps), t1 = run<BM, BN, STAGES, 1>(a, grid, reps);
  const float t2 = run<BM, BN, STAGES, 2>(a, grid, reps);
  const double gflop = 2.0 * a.M * a.N * a.K * 1e-9;
  const double mb = static_cast<double>((a.M + BM - 1) / BM) * (a.N / BN) * (a.K / BK) * (BM + BN) * BK * 4.0 / 1e6;
  std::printf("| %s%s | %d | %d | %d | %dx%d | %d | %d | %.1f | %.1f | %.1f | %.0f | %.1f |\n", name, a.hot ? " (hot)" : "",
              a.M, a.N, a.K, BM, BN, STAGES, grid, t0, t1, t2, gflop / (t0 * 1e-6) * 1e-3, mb / t0);
}

int main() {
  int dev = 0, cus = 256;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  struct Shape {
    const char* name;
    int M, N, K;
  } shapes[] = {{"s3.reduce", 6272, 256, 1024}, {"s3.reduce.b16", 3136, 256, 1024}, {"s4.reduce", 1568, 512, 2048},
                {"s3.expand", 6272, 1024, 256}, {"s2.reduce", 25088, 128, 512}, {"s4.expand", 1568, 2048, 512}};
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
  std::printf("CUs %d\n\n| shape | M | N | K | tile | stages | grid | full us | DMA only | compute only | TFLOP/s logical | MB/us |\n", cus);
  std::printf("|---|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|\n");
  for (auto& s : shapes) {
    for (int hot = 0; hot < 2; ++hot) {
      Args a{x, w, o, s.M, s.N, s.K, hot, static_cast<long long>(s.M) * s.K, static_cast<long long>(s.N) * s.K};
      if (hot && s.M < 4096) continue;
      row<64, 64, 2>(s.name, a, cus, 2);
      row<64, 64, 3>(s.name, a, cus, 1);
      row<64, 64, 4>(s.name, a, cus, 1);
      if (!hot) {
        row<64, 64, 2>(s.name, a, cus, 1);
        row<64, 64, 1 + 1>(s.name, a, cus, 4);
        row<128, 64, 2>(s.name, a, cus, 1);
        row<64, 128, 2>(s.name, a, cus, 1);
      }
    }
  }
  CK(hipFree(x));
  CK(hipFree(w));
  CK(hipFree(o));
  return 0;
}
