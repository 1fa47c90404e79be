// Batched MatMul of two activations (rows): C[b] = A[b] (M x K) * B[b] (K x N), MFMA 16x16x32 bf16,
// split (fp32) operands with three MFMAs per fragment pair.  For the MatMuls that are not part of the
// fused attention pattern (kernels/transformer.hip): token mixing, Gram matrices, gated products.
//
// Block = 64 x 64 output tile of one sample, 4 waves (2 x 2, 32 x 32 each = 2 x 2 fragments).  Per
// 32-wide K step the A tile [64][32] is staged row-major and the B tile [32][64] transposed to
// [64 n][32 k] in LDS (so both MFMA operands read 16 contiguous bytes per lane), 8-element row
// padding against bank conflicts.  A's columns >= K (the logical inner size) are read as 0: pad
// columns of an activation may hold act(0) != 0 (sigmoid).  Output pad columns [N, ldc) are 0.
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

constexpr int BT = 64, KT = 32, LP = KT + 8;

template <bool SPLIT>
__global__ __launch_bounds__(256) void bmm_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bm,
                                                  uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                  int ldc, long long aplane, long long bplane, long long cplane,
                                                  const long long* __restrict__ live) {
  constexpr int NP = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t As[NP][BT][LP];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NP][BT][LP];
  const int b = blockIdx.z;
  if (live && b >= *live) return;  // whole block, before any barrier
  const int m0 = blockIdx.y * BT, n0 = blockIdx.x * BT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const uint16_t* Ab = A + static_cast<long long>(b) * M * lda;
  const uint16_t* Bb = Bm + static_cast<long long>(b) * K * ldb;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ar = tid >> 2, ak = (tid & 3) * 8;  // A: row, 8 k
  const int bk = tid >> 3, bn = (tid & 7) * 8;  // B: k row, 8 n
  for (int k0 = 0; k0 < K; k0 += KT) {
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      uint4 av = make_uint4(0, 0, 0, 0);
      const int m = m0 + ar, k = k0 + ak;
      if (m < M && k < K) {
        av = *reinterpret_cast<const uint4*>(Ab + pl * aplane + static_cast<long long>(m) * lda + k);
        if (k + 8 > K) {  // mask the columns past the logical K (pad columns), in registers
          const int valid = K - k;
          uint32_t wd[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            wd[q] &= (2 * q < valid ? 0x0000FFFFu : 0u) | (2 * q + 1 < valid ? 0xFFFF0000u : 0u);
          av = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
      }
      *reinterpret_cast<uint4*>(&As[pl][ar][ak]) = av;
      uint4 bv = make_uint4(0, 0, 0, 0);
      const int kk = k0 + bk, n = n0 + bn;
      if (kk < K && n < ldb) bv = *reinterpret_cast<const uint4*>(Bb + pl * bplane + static_cast<long long>(kk) * ldb + n);
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&bv);
#pragma unroll
      for (int t = 0; t < 8; ++t) Bs[pl][bn + t][bk] = e[t];
    }
    __syncthreads();
    const int j = lane >> 4, r = lane & 15;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm) {
      bf16x8 a[NP];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) a[pl] = *reinterpret_cast<const bf16x8*>(&As[pl][wm * 32 + fm * 16 + r][j * 8]);
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        bf16x8 bb[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) bb[pl] = *reinterpret_cast<const bf16x8*>(&Bs[pl][wn * 32 + fn * 16 + r][j * 8]);
        if constexpr (SPLIT) {
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[0], acc[fm][fn], 0, 0, 0);
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[1], acc[fm][fn], 0, 0, 0);
        }
        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0], acc[fm][fn], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // D layout: lane (r = lane & 15, j = lane >> 4) holds rows 4j..4j+3 of column r of each fragment
  const int j = lane >> 4, r = lane & 15;
  uint16_t* Cb = C + static_cast<long long>(b) * M * ldc;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) {
      const int n = n0 + wn * 32 + fn * 16 + r;
      if (n >= ldc) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int m = m0 + wm * 32 + fm * 16 + 4 * j + t;
        if (m >= M) continue;
        const float v = n < N ? acc[fm][fn][t] : 0.f;
        store1v(Cb + static_cast<long long>(m) * ldc + n, cplane, SPLIT, v);
      }
    }
}

}  // namespace

hipError_t bmm_rows(const uint16_t* A, const uint16_t* Bm, uint16_t* C, int batch, int M, int N, int K, int lda, int ldb,
                    int ldc, hipStream_t s, const long long* live, int split) {
  if (batch < 1 || M < 1 || N < 1 || K < 1 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < N || ldc < N)
    return hipErrorInvalidValue;
  const dim3 grid((ldc + BT - 1) / BT, (M + BT - 1) / BT, batch);
  const long long ap = static_cast<long long>(batch) * M * lda, bp = static_cast<long long>(batch) * K * ldb,
                  cp = static_cast<long long>(batch) * M * ldc;
  if (split)
    hipLaunchKernelGGL(bmm_kernel<true>, grid, dim3(256), 0, s, A, Bm, C, M, N, K, lda, ldb, ldc, ap, bp, cp, live);
  else
    hipLaunchKernelGGL(bmm_kernel<false>, grid, dim3(256), 0, s, A, Bm, C, M, N, K, lda, ldb, ldc, ap, bp, cp, live);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
