// Implicit-GEMM convolution / GEMM for gfx950 on MFMA (v_mfma_f32_16x16x32_bf16).
//
// Replaces the Conv / FusedConv / Gemm kernels ONNX Runtime would run for the reference
// (src/inference_engine.cpp:114-121,176-183 -> [ext] ORT CUDA EP).  Design (CDNA4-first):
//  * NHWC bf16 activations, weights pre-packed as [Npad][Kpad] bf16 with k = (ky, kx, ci), so both
//    MFMA operands are K-contiguous and a BK=64 K-step of the activation tile is a plain 128-byte
//    row per output pixel (padding pixels -> zeros, predicated loads).
//  * The GEMM is computed transposed (A = weights, B = pixels): the 16x16 accumulator then holds
//    4 consecutive output channels of one pixel per lane, i.e. 8-byte contiguous NHWC stores and
//    float4 bias/scale loads in the fused epilogue.
//  * 256-thread blocks = 4 wave64s in a 2x2 grid; BMxBN in {128,64}^2; 64-wide K-steps double-
//    buffered in LDS with the next tile's global loads issued before the MFMAs of the current one
//    (async-STAGE split) and ONE barrier per K-step.
//  * LDS rows are 128 B; the 16-byte chunk index is XOR-swizzled with (row>>1)&7, which makes the
//    ds_read_b128 fragment reads of both operands bank-conflict-free for the gfx950 b128 lane
//    groups ({0-3,12-15,20-27}, ...).
//  * Fused epilogue: + bias (folded BatchNorm), + residual, ReLU, bf16 or f32 store, and an
//    optional second output act(v*scale2+shift2) (the next pre-activation unit's BN+ReLU), which
//    removes every standalone BatchNormalization / Relu / Add of ResNet-v2.
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int BM, int BN, int MODE, int VEC>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const ConvArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;  // per-wave pixels / channels
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_ELEMS = BN * BK, B_ELEMS = BM * BK, STAGE = A_ELEMS + B_ELEMS;
  constexpr int W_CH = BN / 32;                       // 16-B weight chunks per thread per stage
  constexpr int X_CH = VEC == 8 ? BM / 32 : BM / 16;  // activation units per thread per stage
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = (p.N + BN - 1) / BN;
  const int tile_n = blockIdx.x % ntn;
  const int tile_m = blockIdx.x / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---- per-thread loader state ----
  const int wc = tid & 7;
  const int wr = tid >> 3;
  const uint16_t* wsrc = p.w + static_cast<size_t>(n0 + wr) * p.Kpad + wc * 8;

  constexpr int XC_SHIFT = VEC == 8 ? 3 : 4;  // threads per row
  const int xc = tid & ((1 << XC_SHIFT) - 1);
  const int xr = tid >> XC_SHIFT;
  constexpr int XR_STEP = 256 >> XC_SHIFT;
  bool mvalid[X_CH];
  int ih0[X_CH], iw0[X_CH];
  size_t xbase[X_CH];
#pragma unroll
  for (int i = 0; i < X_CH; ++i) {
    const int m = m0 + xr + XR_STEP * i;
    mvalid[i] = m < p.M;
    const int mm = mvalid[i] ? m : 0;
    if (MODE == 0) {
      xbase[i] = static_cast<size_t>(mm) * p.Cin;
      ih0[i] = iw0[i] = 0;
    } else {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int r = mm - b * hw;
      const int oh = r / p.Wo;
      const int ow = r - oh * p.Wo;
      ih0[i] = oh * p.stride - p.pad_h;
      iw0[i] = ow * p.stride - p.pad_w;
      xbase[i] = static_cast<size_t>(b) * p.H * p.W * p.Cin;
    }
  }

  uint4 wreg[W_CH];
  uint4 xreg8[VEC == 8 ? X_CH : 1];
  uint2 xreg4[VEC == 4 ? X_CH : 1];

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < W_CH; ++i)
      wreg[i] = *reinterpret_cast<const uint4*>(wsrc + static_cast<size_t>(32 * i) * p.Kpad + k0);
    const int kk = k0 + xc * VEC;
    bool kvalid = kk < p.K;
    int off = 0, ky = 0, kx = 0;
    if (MODE == 0) {
      off = kk;
    } else if (kvalid) {
      const int t = kk / p.Cin;
      const int ci = kk - t * p.Cin;
      ky = t / p.KW;
      kx = t - ky * p.KW;
      off = ci;
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      bool v = kvalid && mvalid[i];
      size_t addr = xbase[i] + off;
      if (MODE == 1) {
        const int ih = ih0[i] + ky * p.dil;
        const int iw = iw0[i] + kx * p.dil;
        v = v && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        addr += (static_cast<size_t>(ih) * p.W + iw) * p.Cin;
      }
      if (VEC == 8) {
        xreg8[i] = v ? *reinterpret_cast<const uint4*>(p.x + addr) : make_uint4(0, 0, 0, 0);
      } else {
        xreg4[i] = v ? *reinterpret_cast<const uint2*>(p.x + addr) : make_uint2(0, 0);
      }
    }
  };

  auto store_stage = [&](int buf) {
    uint16_t* A = lds + buf * STAGE;
    uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int i = 0; i < W_CH; ++i) *reinterpret_cast<uint4*>(A + swz(wr + 32 * i, wc)) = wreg[i];
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int row = xr + XR_STEP * i;
      if (VEC == 8) {
        *reinterpret_cast<uint4*>(Bt + swz(row, xc)) = xreg8[i];
      } else {
        *reinterpret_cast<uint2*>(Bt + swz(row, xc >> 1) + 4 * (xc & 1)) = xreg4[i];
      }
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kpad / BK;
  load_stage(0);
  store_stage(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_stage((kt + 1) * BK);  // in flight under the MFMAs below
    const uint16_t* A = lds + cur * STAGE;
    const uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + swz(wn * WN + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + swz(wm * WM + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue ----
  const int lm = lane & 15;
  const int ln = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn * WN + i * 16 + ln;
    if (n >= p.N) continue;
    float4 bias = p.bias ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 sc2 = make_float4(1.f, 1.f, 1.f, 1.f), sh2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.out2) {
      sc2 = *reinterpret_cast<const float4*>(p.scale2 + n);
      sh2 = *reinterpret_cast<const float4*>(p.shift2 + n);
    }
    if (p.N & 3) {  // ragged N (e.g. a 10-class head): element-wise path
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WM + j * 16 + lm;
        if (m >= p.M) continue;
        const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
        const float s2[4] = {sc2.x, sc2.y, sc2.z, sc2.w};
        const float h2[4] = {sh2.x, sh2.y, sh2.z, sh2.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (n + r >= p.N) break;
          const size_t o = static_cast<size_t>(m) * p.N + n + r;
          float v = acc[i][j][r] + bb[r];
          if (p.res) v += bf2f(p.res[o]);
          if (p.relu) v = fmaxf(v, 0.f);
          if (p.out) p.out[o] = f2bf(v);
          if (p.out_f32) p.out_f32[o] = v;
          if (p.out2) {
            float u = v * s2[r] + h2[r];
            if (p.relu2) u = fmaxf(u, 0.f);
            p.out2[o] = f2bf(u);
          }
        }
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + lm;
      if (m >= p.M) continue;
      const size_t o = static_cast<size_t>(m) * p.N + n;
      float v0 = acc[i][j][0] + bias.x, v1 = acc[i][j][1] + bias.y;
      float v2 = acc[i][j][2] + bias.z, v3 = acc[i][j][3] + bias.w;
      if (p.res) {
        const uint2 r = *reinterpret_cast<const uint2*>(p.res + o);
        float r0, r1, r2, r3;
        unpack2(r.x, r0, r1);
        unpack2(r.y, r2, r3);
        v0 += r0;
        v1 += r1;
        v2 += r2;
        v3 += r3;
      }
      if (p.relu) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
        v2 = fmaxf(v2, 0.f);
        v3 = fmaxf(v3, 0.f);
      }
      if (p.out) *reinterpret_cast<uint2*>(p.out + o) = make_uint2(pack2(v0, v1), pack2(v2, v3));
      if (p.out_f32) *reinterpret_cast<float4*>(p.out_f32 + o) = make_float4(v0, v1, v2, v3);
      if (p.out2) {
        float u0 = v0 * sc2.x + sh2.x, u1 = v1 * sc2.y + sh2.y;
        float u2 = v2 * sc2.z + sh2.z, u3 = v3 * sc2.w + sh2.w;
        if (p.relu2) {
          u0 = fmaxf(u0, 0.f);
          u1 = fmaxf(u1, 0.f);
          u2 = fmaxf(u2, 0.f);
          u3 = fmaxf(u3, 0.f);
        }
        *reinterpret_cast<uint2*>(p.out2 + o) = make_uint2(pack2(u0, u1), pack2(u2, u3));
      }
    }
  }
}

template <int BM, int BN>
hipError_t launch_cfg(const ConvArgs& a, hipStream_t s) {
  const bool dense1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad_h == 0 && a.pad_w == 0 && a.H == a.Ho &&
                        a.W == a.Wo;
  const int vec = a.Cin % 8 == 0 ? 8 : 4;
  const int grid = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (dense1x1 && vec == 8) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 0, 8>), dim3(grid), dim3(256), 0, s, a);
  } else if (vec == 8) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 8>), dim3(grid), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 4>), dim3(grid), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace

void tile_dims(int cfg, int& bm, int& bn) {
  switch (cfg) {
    case TILE_128x128: bm = 128; bn = 128; break;
    case TILE_128x64: bm = 128; bn = 64; break;
    case TILE_64x128: bm = 64; bn = 128; break;
    default: bm = 64; bn = 64; break;
  }
}

int choose_tile(int M, int N, int K) {
  (void)K;
  auto blocks = [&](int cfg) {
    int bm, bn;
    tile_dims(cfg, bm, bn);
    return static_cast<long>((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  };
  if (N <= 64) return blocks(TILE_128x64) >= 512 ? TILE_128x64 : TILE_64x64;
  if (blocks(TILE_128x128) >= 512) return TILE_128x128;
  if (blocks(TILE_64x128) >= 384) return TILE_64x128;
  return TILE_64x64;
}

hipError_t conv_igemm(const ConvArgs& a, int cfg, hipStream_t s) {
  if (a.Cin % 4 != 0 || a.Kpad % BK != 0 || a.K > a.Kpad) return hipErrorInvalidValue;
  if (!a.out && !a.out_f32 && !a.out2) return hipErrorInvalidValue;
  if (a.out2 && (!a.scale2 || !a.shift2)) return hipErrorInvalidValue;
  switch (cfg) {
    case TILE_128x128: return launch_cfg<128, 128>(a, s);
    case TILE_128x64: return launch_cfg<128, 64>(a, s);
    case TILE_64x128: return launch_cfg<64, 128>(a, s);
    default: return launch_cfg<64, 64>(a, s);
  }
}

}  // namespace kern
}  // namespace die
