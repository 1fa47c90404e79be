// Skinny dense GEMM: variant 8 of the GEMM config space (tile 0 only, cfg 32), for the few-row
// heads -- ResNet's FC at the serving batch is M = B <= 32 rows x N = 1000 x K = 2048, where the
// 64-row tiles waste most of their MFMA rows and the split-K forms pay a global hand-off (the
// fused split-K FC took 15-17 us at B = 20-24, profiles/r5_ops_resnet50_fp32_b24.md).
//
// One block owns 16 output channels for all (<= 32) rows; its 8 waves split K eight ways, so every
// operand is loaded exactly once, straight from global memory into MFMA fragments (16-byte loads,
// no LDS staging: each fragment is used once).  v_mfma_f32_16x16x32_bf16 with the weights as the A
// operand and the pixels as B, so a lane ends with 4 consecutive channels of one row; fp32 (split)
// mode takes the three products hi*hi + lo*hi + hi*lo as everywhere else (common.h).  The 8 partial
// tiles meet in LDS and are summed in wave order (deterministic), then the shared epilogue8 runs.
// Measured (tools/gemm_sweep.py --tokens 1 --shapes fc, ResNet50 FC at B = 20 / 24): 11.8 / 12.4 us,
// level with the fused split-K 64x64 form (12.1 / 12.5 us): with 16 channels per block only 63 CUs
// stream the 8 MB of split weights, while the split-K form pays a global hand-off instead.  It stays
// a tuner candidate (cfg 32) for the few-row dense heads; the autotuner keeps whichever is faster.
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {
namespace {

constexpr int kSkRows = 32;   // pixel rows (two 16-row MFMA fragments)
constexpr int kSkCols = 16;   // output channels per block
constexpr int kSkWaves = 8;   // K split inside the block

template <bool SPLIT>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const ConvArgs p) {
  __shared__ float red[kSkWaves][kSkRows][kSkCols + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * kSkCols;
  const int Ml = p.live ? min(p.M, static_cast<int>(*p.live) * p.Ho * p.Wo) : p.M;
  const int r = lane & 15, kq = (lane >> 4) * 8;
  // clamped rows read valid memory; their results are never stored
  const int nrow = min(n0 + r, p.N - 1);
  const int ma = min(r, p.M - 1), mb = min(16 + r, p.M - 1);
  const int kper = p.K / kSkWaves;
  const int k0 = wave * kper + kq;
  const uint16_t* wr = p.w + static_cast<size_t>(nrow) * p.Kpad + k0;
  const uint16_t* xa = p.x + static_cast<size_t>(ma) * p.K + k0;
  const uint16_t* xb = p.x + static_cast<size_t>(mb) * p.K + k0;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k = 0; k < kper; k += 32) {
    const bf16x8 wh = *reinterpret_cast<const bf16x8*>(wr + k);
    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(xa + k);
    const bf16x8 bh = *reinterpret_cast<const bf16x8*>(xb + k);
    if constexpr (SPLIT) {
      const bf16x8 wl = *reinterpret_cast<const bf16x8*>(wr + k + p.wplane);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(xa + k + p.xplane);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(xb + k + p.xplane);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, ah, acc0, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, al, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, bh, acc1, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, bl, acc1, 0, 0, 0);
    }
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, ah, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, bh, acc1, 0, 0, 0);
  }
  // lane: channels 4 (lane >> 4) + t of pixel lane & 15 (acc0) / 16 + lane & 15 (acc1)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    red[wave][r][(lane >> 4) * 4 + t] = acc0[t];
    red[wave][16 + r][(lane >> 4) * 4 + t] = acc1[t];
  }
  __syncthreads();
  if (tid < kSkRows * 2) {
    const int m = tid >> 1, c0 = (tid & 1) * 8, n = n0 + c0;
    if (m < Ml && n < p.N) {
      float v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kSkWaves; ++w) s += red[w][m][c0 + c];
        v[c] = s;
      }
      epilogue8(p, m, n, v);
    }
  }
}

}  // namespace

hipError_t launch_tile_skinny(const ConvArgs& a, hipStream_t s, int tile) {
  if (tile != TILE_128x128) return hipErrorInvalidValue;
  const bool dense = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad_h == 0 && a.pad_w == 0 && a.H == a.Ho &&
                     a.W == a.Wo && a.Cin == a.K && a.K <= a.Kpad;
  // rows <= 32, whole 32-wide K-steps per wave, 8-channel epilogue groups, no split-K, no LayerNorm
  // statistics / pre-activation on load (those belong to the row GEMMs of the tiled kernels)
  if (!dense || a.M < 1 || a.M > kSkRows || a.K % (32 * kSkWaves) != 0 || a.N % 8 != 0 || a.splits > 1 ||
      a.in_scale || a.row_parts || a.stats_out || a.tail || (a.split && a.wplane <= 0))
    return hipErrorInvalidValue;
  ConvArgs b = a;
  b.splits = 1;
  b.counters = nullptr;
  if (a.split) {
    b.xplane = static_cast<long long>(a.B) * a.H * a.W * a.Cin;
    b.oplane = static_cast<long long>(a.M) * a.N;
  } else {
    b.xplane = b.oplane = 0;
  }
  const dim3 grid((a.N + kSkCols - 1) / kSkCols);
  if (a.split) hipLaunchKernelGGL(gemm_skinny_kernel<true>, grid, dim3(512), 0, s, b);
  else hipLaunchKernelGGL(gemm_skinny_kernel<false>, grid, dim3(512), 0, s, b);
  return hipGetLastError();
}

}  // namespace igemm
}  // namespace kern
}  // namespace die
