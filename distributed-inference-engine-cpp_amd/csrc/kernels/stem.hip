// 7x7 / stride 2 / pad 3 stem convolution (ResNet conv0) on MFMA, gfx950.
//
// The generic implicit-GEMM kernel runs this layer at ~75 TFLOP/s: with 4 input channels every
// lane gathers 8-byte pieces of 16 different pixels per k-step.  Here a block owns an 8 x 16 tile of
// output pixels and all 64 output channels:
//   * the 21 x 38 x 4-channel input patch it needs (rows 2*8+5, cols 2*16+6) is staged in LDS once;
//   * K is ordered (ky, kx, c) with kx padded 7 -> 8 (zero weights), so K = 7*8*4 = 224 = 7 MFMA
//     k-steps and k-step s is exactly filter row ky = s.  Lane group j of v_mfma_f32_16x16x32_bf16
//     reads taps (2j, 2j+1) of that row: 16 contiguous, 16-byte-aligned bytes of the patch, and the
//     16 lanes of a group read 16 consecutive output pixels = 256 contiguous bytes (no bank
//     conflicts);
//   * weights [64][224] (BN folded) sit in LDS with a 240-element pitch (conflict-free A reads for the b128 lane groups);
//   * epilogue: + bias, optional ReLU, bf16, staged through LDS (XOR-swizzled) so each output pixel's
//     128 bytes go out as 16-byte stores.
//   * SPLIT (fp32 mode, common.h): input, weights and output are hi/lo planes; both planes of the
//     patch and the weights sit in LDS and each fragment pair takes three MFMAs.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

constexpr int TY = 8, TX = 16;               // output tile
constexpr int PY = 2 * TY + 5, PX = 2 * TX + 6;  // patch (PX even: kx padded to 8)
constexpr int KS = 224, WP = 240;            // K and weight LDS pitch (elements): conflict-free A reads
constexpr int NCH = 64;

template <bool SPLIT>
__global__ __launch_bounds__(256) void stem7x7_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                      int H, int W, int Ho, int Wo, int relu, int tiles_x,
                                                      const long long* __restrict__ live) {
  constexpr int NP = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t wl[NP * NCH * WP];
  __shared__ __attribute__((aligned(16))) uint16_t patch[NP * PY * PX * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y;
  const long long xplane = static_cast<long long>(gridDim.y) * H * W * 4;
  const long long oplane = static_cast<long long>(gridDim.y) * Ho * Wo * NCH;
  if (live && b >= *live) return;  // padding sample of the bucket: whole block, before any barrier
  const int ty0 = (blockIdx.x / tiles_x) * TY, tx0 = (blockIdx.x % tiles_x) * TX;
  // weights -> LDS (64 x 224 bf16 = 28 chunks of 16 B per row; SPLIT: the lo plane follows)
  for (int i = tid; i < NP * NCH * (KS / 8); i += 256) {
    const int pl = i / (NCH * (KS / 8)), q = i % (NCH * (KS / 8));
    const int r = q / (KS / 8), c = q % (KS / 8);
    *reinterpret_cast<uint4*>(wl + pl * NCH * WP + r * WP + c * 8) =
        *reinterpret_cast<const uint4*>(w + pl * NCH * KS + r * KS + c * 8);
  }
  // input patch -> LDS: pixel (iy, ix) = 4 bf16 = 8 bytes; outside the image -> 0
  const int iy0 = 2 * ty0 - 3, ix0 = 2 * tx0 - 3;
  const uint16_t* xb = x + static_cast<size_t>(b) * H * W * 4;
  for (int i = tid; i < NP * PY * PX; i += 256) {
    const int pl = i / (PY * PX), q = i % (PY * PX);
    const int py = q / PX, px = q % PX;
    const int iy = iy0 + py, ix = ix0 + px;
    uint2 v = make_uint2(0, 0);
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const uint2*>(xb + pl * xplane + (static_cast<size_t>(iy) * W + ix) * 4);
    *reinterpret_cast<uint2*>(patch + pl * PY * PX * 4 + q * 4) = v;
  }
  __syncthreads();
  // wave w: output rows 2w, 2w+1 of the tile (16 pixels each) x 64 channels
  f32x4 acc[4][2];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int j = lane >> 4, px_l = lane & 15;
#pragma unroll
  for (int ky = 0; ky < 7; ++ky) {
    bf16x8 bf[NP][2];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int oy = 2 * wave + m;
        const int py = 2 * oy + ky, px = 2 * px_l + 2 * j;
        bf[pl][m] = *reinterpret_cast<const bf16x8*>(patch + pl * PY * PX * 4 + (py * PX + px) * 4);
      }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int wo = (n * 16 + (lane & 15)) * WP + ky * 32 + j * 8;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + wo);
      if constexpr (SPLIT) {
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(wl + NCH * WP + wo);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bf[0][m], acc[n][m], 0, 0, 0);
          acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[NP - 1][m], acc[n][m], 0, 0, 0);
        }
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[0][m], acc[n][m], 0, 0, 0);
    }
  }
  __syncthreads();  // weights -> output stage [128 px][64 ch] bf16, 16-B chunk c of pixel p at chunk c ^ (p & 7)
  uint16_t* stage = wl;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int ch = n * 16 + 4 * j;  // this lane's 4 consecutive channels
    const float4 bv = *reinterpret_cast<const float4*>(bias + ch);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int p = (2 * wave + m) * TX + px_l;
      float v0 = acc[n][m][0] + bv.x, v1 = acc[n][m][1] + bv.y, v2 = acc[n][m][2] + bv.z, v3 = acc[n][m][3] + bv.w;
      if (relu) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
        v2 = fmaxf(v2, 0.f);
        v3 = fmaxf(v3, 0.f);
      }
      const int chunk = (ch >> 3) ^ (p & 7);
      uint16_t* dst = stage + p * NCH + chunk * 8 + (ch & 7);
      if constexpr (SPLIT) {
        const float vv[4] = {v0, v1, v2, v3};
        uint16_t h[4], l[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) split1(vv[t], h[t], l[t]);
        *reinterpret_cast<uint2*>(dst) = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
        *reinterpret_cast<uint2*>(dst + TY * TX * NCH) =
            make_uint2(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16));
      } else {
        *reinterpret_cast<uint2*>(dst) = make_uint2(pack2(v0, v1), pack2(v2, v3));
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < NP * TY * TX * (NCH / 8); i += 256) {
    const int pl = i / (TY * TX * (NCH / 8)), q = i % (TY * TX * (NCH / 8));
    const int p = q >> 3, c = q & 7;
    const int oy = ty0 + p / TX, ox = tx0 + p % TX;
    if (oy >= Ho || ox >= Wo) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(stage + pl * TY * TX * NCH + p * NCH + ((c ^ (p & 7)) << 3));
    *reinterpret_cast<uint4*>(out + pl * oplane + ((static_cast<size_t>(b) * Ho + oy) * Wo + ox) * NCH + c * 8) = v;
  }
}

// Fused variant: reads the graph input itself (fp32 NCHW, C <= 4 channels), applies the input's
// pending BatchNormalization (scale/shift per channel, the former input_prep pass), and is
// persistent: a block stages the weights in LDS ONCE and then walks output tiles (blockIdx.x,
// + gridDim.x, ...), prefetching the next tile's patch into registers while the MFMAs of the
// current one run.  The epilogue stores straight from the accumulators (8 bytes = 4 channels per
// lane and plane) because the LDS holds the weights for the whole walk.  8 waves per block (one
// output row each) and 2 blocks per CU: 4 waves per SIMD to overlap one wave's patch staging and
// stores with the others' MFMAs.
constexpr int SNT = 512;                       // 8 waves: one output row of the tile each
constexpr int PPT = (PY * PX + SNT - 1) / SNT;  // patch pixels per thread

template <bool SPLIT>
__global__ __launch_bounds__(SNT, 2) void stem7x7_nchw_kernel(const float* __restrict__ x, int C,
                                                             const float* __restrict__ in_scale,
                                                             const float* __restrict__ in_shift,
                                                             const uint16_t* __restrict__ w,
                                                             const float* __restrict__ bias, uint16_t* __restrict__ out,
                                                             int B, int H, int W, int Ho, int Wo, int relu, int tiles_x,
                                                             int tiles_per_img, const long long* __restrict__ live) {
  constexpr int NP = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t wl[NP * NCH * WP];
  __shared__ __attribute__((aligned(16))) uint16_t patch[NP * PY * PX * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long oplane = static_cast<long long>(B) * Ho * Wo * NCH;
  const int nb = live ? min(B, static_cast<int>(*live)) : B;
  const int total = nb * tiles_per_img;
  if (static_cast<int>(blockIdx.x) >= total) return;  // whole block, before any barrier
  for (int i = tid; i < NP * NCH * (KS / 8); i += SNT) {
    const int pl = i / (NCH * (KS / 8)), q = i % (NCH * (KS / 8));
    const int r = q / (KS / 8), c = q % (KS / 8);
    *reinterpret_cast<uint4*>(wl + pl * NCH * WP + r * WP + c * 8) =
        *reinterpret_cast<const uint4*>(w + pl * NCH * KS + r * KS + c * 8);
  }
  float sc[4], sh[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    sc[c] = (c < C && in_scale) ? in_scale[c] : 1.f;
    sh[c] = (c < C && in_shift) ? in_shift[c] : 0.f;
  }
  const size_t HW = static_cast<size_t>(H) * W;
  // raw input of this thread's patch pixels for tile t (0 outside the image; BN applied on store)
  float pre[PPT][4];
  bool inb[PPT];
  auto fetch = [&](int t) {
    const int b = t / tiles_per_img, tt = t - b * tiles_per_img;
    const int iy0 = 2 * ((tt / tiles_x) * TY) - 3, ix0 = 2 * ((tt % tiles_x) * TX) - 3;
    const float* xb = x + static_cast<size_t>(b) * C * HW;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int q = tid + k * SNT;
      const int py = q / PX, px = q - (q / PX) * PX;
      const int iy = iy0 + py, ix = ix0 + px;
      inb[k] = q < PY * PX && iy >= 0 && iy < H && ix >= 0 && ix < W;
#pragma unroll
      for (int c = 0; c < 4; ++c) pre[k][c] = (inb[k] && c < C) ? xb[c * HW + static_cast<size_t>(iy) * W + ix] : 0.f;
    }
  };
  fetch(blockIdx.x);
  const int j = lane >> 4, px_l = lane & 15;
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    __syncthreads();  // weights staged / every wave done reading the previous tile's patch
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int q = tid + k * SNT;
      if (q >= PY * PX) continue;
      float v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = (inb[k] && c < C) ? fmaf(pre[k][c], sc[c], sh[c]) : 0.f;
      uint16_t h[4], l[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr (SPLIT) split1(v[c], h[c], l[c]);
        else h[c] = f2bf(v[c]);
      }
      *reinterpret_cast<uint2*>(patch + q * 4) = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
      if constexpr (SPLIT)
        *reinterpret_cast<uint2*>(patch + PY * PX * 4 + q * 4) =
            make_uint2(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16));
    }
    __syncthreads();
    const int tn = t + static_cast<int>(gridDim.x);
    if (tn < total) fetch(tn);  // in flight during this tile's MFMAs
    f32x4 acc[4][1];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      bf16x8 bf[NP][1];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const int py = 2 * wave + ky, px = 2 * px_l + 2 * j;
        bf[pl][0] = *reinterpret_cast<const bf16x8*>(patch + pl * PY * PX * 4 + (py * PX + px) * 4);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int wo = (n * 16 + (lane & 15)) * WP + ky * 32 + j * 8;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + wo);
        if constexpr (SPLIT) {
          const bf16x8 al = *reinterpret_cast<const bf16x8*>(wl + NCH * WP + wo);
          acc[n][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bf[0][0], acc[n][0], 0, 0, 0);
          acc[n][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[NP - 1][0], acc[n][0], 0, 0, 0);
        }
        acc[n][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[0][0], acc[n][0], 0, 0, 0);
      }
    }
    const int b = t / tiles_per_img, tt = t - b * tiles_per_img;
    const int ty0 = (tt / tiles_x) * TY, tx0 = (tt % tiles_x) * TX;
    constexpr int m = 0;
    const int oy = ty0 + wave, ox = tx0 + px_l;
    if (oy < Ho && ox < Wo) {
      uint16_t* o = out + ((static_cast<size_t>(b) * Ho + oy) * Wo + ox) * NCH;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int ch = n * 16 + 4 * j;
        const float4 bv = *reinterpret_cast<const float4*>(bias + ch);
        float v[4] = {acc[n][m][0] + bv.x, acc[n][m][1] + bv.y, acc[n][m][2] + bv.z, acc[n][m][3] + bv.w};
        if (relu) {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
        }
        if constexpr (SPLIT) {
          uint16_t h[4], l[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) split1(v[q], h[q], l[q]);
          *reinterpret_cast<uint2*>(o + ch) = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
          *reinterpret_cast<uint2*>(o + oplane + ch) = make_uint2(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16));
        } else {
          *reinterpret_cast<uint2*>(o + ch) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
    }
  }
}

// Stem + 3x3/2 max pool (pad 1) + the pooled value's BN/ReLU in one kernel (ResNet conv0 -> pool0
// -> stage-1 pre-activation): the 112x112x64 stem map (64 MB per 20 images in fp32 mode) is never
// stored or re-read; only the 56x56 pooled map is written.
//   * a block owns a segment of pool rows [p0, p1) of one image over the FULL stem width: wave w
//     computes stem columns [16w, 16w + 16) (CG = ceil(Ws / 16) <= 8 waves), and per pool row p the
//     two stem rows 2p, 2p + 1 (acc[4][2], the stem7x7_nchw MFMA schedule); stem row 2p - 1 is
//     carried in registers from the previous row (recomputed once at the segment start);
//   * the input rows sit in an LDS ring of 11 rows (fp32 NCHW -> input BN -> bf16 / split on the
//     way in); the 4 rows the next pool row adds are fetched into registers during this row's MFMAs;
//   * pooling: vertical max of the 3 stem rows in registers, horizontal max over lanes px-1 / px+1
//     with DPP row shifts (a 16-lane DPP row = the 16 stem columns of the wave), the column left of
//     the wave's first one through LDS; the max runs on the stored representation (hi + lo), as the
//     unfused pool reads it, so the fusion is bit-exact;
//   * weight rows are permuted by pair_permute_row: lane group j holds logical channels
//     32 blk + 8 j + [0, 8) of the two fragments 2 blk, 2 blk + 1 -> 16-byte pooled stores.
constexpr int RING = 11;  // input rows: halo stem row (7) + two stem rows (9) share 11 at the segment start

__device__ __forceinline__ float dpp_shr1(float v) {  // lane - 1 within its 16-lane row (-inf at column 0)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_shl1(float v) {  // lane + 1 within its 16-lane row (-inf at column 15)
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), 0x101, 0xf, 0xf, false));
}

template <bool SPLIT>
__global__ __launch_bounds__(512) void stem_pool_nchw_kernel(
    const float* __restrict__ x, int C, const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    const uint16_t* __restrict__ w, const float* __restrict__ bias, int relu, const float* __restrict__ pscale,
    const float* __restrict__ pshift, int pact, uint16_t* __restrict__ out, int B, int H, int W, int Hs, int Ws, int Hp,
    int Wp, int seg_len, int segs_per_img, const long long* __restrict__ live) {
  constexpr int NP = SPLIT ? 2 : 1;
  const int CG = blockDim.x >> 6, PXF = 32 * CG + 6;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* wl = smem;                           // NP x [64][WP]
  uint16_t* ring = wl + NP * NCH * WP;           // NP x [RING][PXF][4]
  float* xbuf = reinterpret_cast<float*>(ring + NP * RING * PXF * 4);  // [CG][64]: column 15 of each wave
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
  const int b = blockIdx.x / segs_per_img;
  const int p0 = (blockIdx.x % segs_per_img) * seg_len, p1 = min(p0 + seg_len, Hp);
  if ((live && b >= *live) || b >= B || p0 >= Hp) return;  // whole block, before any barrier
  const long long oplane = static_cast<long long>(B) * Hp * Wp * NCH;
  const long long ring_plane = static_cast<long long>(RING) * PXF * 4;
  float sc[4], sh[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    sc[c] = (c < C && in_scale) ? in_scale[c] : 1.f;
    sh[c] = (c < C && in_shift) ? in_shift[c] : 0.f;
  }
  const size_t HW = static_cast<size_t>(H) * W;
  const float* xb = x + static_cast<size_t>(b) * C * HW;
  // input pixel (row iy, patch column q) -> ring (input BN, then bf16 / split; 0 outside the image)
  auto put = [&](int iy, int q, const float* raw, bool inb) {
    float v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (inb && c < C) ? fmaf(raw[c], sc[c], sh[c]) : 0.f;
    uint16_t h[4], l[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if constexpr (SPLIT) split1(v[c], h[c], l[c]);
      else h[c] = f2bf(v[c]);
    }
    uint16_t* d = ring + (static_cast<long long>((iy + 5 * RING) % RING) * PXF + q) * 4;
    *reinterpret_cast<uint2*>(d) = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
    if constexpr (SPLIT)
      *reinterpret_cast<uint2*>(d + ring_plane) = make_uint2(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16));
  };
  // Branch-free: raw buffer loads of the image (num_records = its C planes), off-image pixels and
  // channels past C at an offset past the end, which the buffer returns as 0 -- no per-lane branch
  // around a load, so a round's loads all stay in flight (behind `inb ? x[..] : 0` the compiler
  // sank each pixel's loads into a branch and waited for them before the next pixel's).
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xb), 0, static_cast<int>(C * HW * 4), 0x00020000);
  auto load_px = [&](int iy, int q, float* raw) -> bool {
    const int ix = q - 3;
    const bool inb = iy >= 0 && iy < H && ix >= 0 && ix < W;
    const unsigned pix = inb ? static_cast<unsigned>(iy * W + ix) * 4u : 0x80000000u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned off = c < C ? pix + static_cast<unsigned>(c * HW * 4) : 0x80000000u;
      raw[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
    }
    return inb;
  };
  // Segment start: input rows 4 p0 - 5 .. 4 p0 + 5 (halo stem row 2 p0 - 1 and stem rows 2 p0,
  // 2 p0 + 1) and the weights, all loads issued before the first LDS store.
  constexpr int SPT = 7;  // RING * PXF <= 7 * 64 CG for every CG >= 1 (11 (32 CG + 6) <= 448 CG)
  float sraw[SPT][4];
  bool sin[SPT];
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int i = min(tid + k * nthr, RING * PXF - 1);
    sin[k] = load_px(4 * p0 - 5 + i / PXF, i % PXF, sraw[k]);
  }
  {
    constexpr int WR = 8;  // weight chunks per thread and round (one round at CG >= 7)
    const int nw = NP * NCH * (KS / 8);
    for (int i0 = 0; i0 < nw; i0 += WR * nthr) {
      uint4 wv[WR];
#pragma unroll
      for (int k = 0; k < WR; ++k) {
        const int i = min(i0 + tid + k * nthr, nw - 1);
        const int pl = i / (NCH * (KS / 8)), q = i % (NCH * (KS / 8));
        wv[k] = *reinterpret_cast<const uint4*>(w + pl * NCH * KS + (q / (KS / 8)) * KS + (q % (KS / 8)) * 8);
      }
#pragma unroll
      for (int k = 0; k < WR; ++k) {  // past the end: the last chunk again (same bytes, no branch)
        const int i = min(i0 + tid + k * nthr, nw - 1);
        const int pl = i / (NCH * (KS / 8)), q = i % (NCH * (KS / 8));
        *reinterpret_cast<uint4*>(wl + pl * NCH * WP + (q / (KS / 8)) * WP + (q % (KS / 8)) * 8) = wv[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int i = tid + k * nthr;
    if (i < RING * PXF) put(4 * p0 - 5 + i / PXF, i % PXF, sraw[k], sin[k]);
  }
  __syncthreads();
  const int j = lane >> 4, px_l = lane & 15, sx = 16 * wave + px_l;
  // one stem row (sy) of this wave's 16 columns: acc = 64 channels (4 fragments) of pixel (sy, sx)
  auto stem_rows = [&](int sy0, int nrows, f32x4 (&acc)[4][2]) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int m = 0; m < 2; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
      bf16x8 bf[NP][2];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int iy = 2 * (sy0 + m) - 3 + ky;
          bf[pl][m] = *reinterpret_cast<const bf16x8*>(ring + pl * ring_plane +
                                                       (static_cast<long long>((iy + 5 * RING) % RING) * PXF + 2 * sx + 2 * j) * 4);
        }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int wo = (n * 16 + (lane & 15)) * WP + ky * 32 + j * 8;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(wl + wo);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          if (m >= nrows) continue;
          if constexpr (SPLIT) {
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(wl + NCH * WP + wo);
            acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bf[0][m], acc[n][m], 0, 0, 0);
            acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[NP - 1][m], acc[n][m], 0, 0, 0);
          }
          acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[0][m], acc[n][m], 0, 0, 0);
        }
      }
    }
  };
  // stem epilogue -> the value the unfused pool would read back (hi + lo, or bf16); -inf off the map
  // (max pool padding).  Physical fragment n, lane group j, element t = logical channel
  // 32 (n >> 1) + 8 j + 4 (n & 1) + t.
  // This lane's 16 channels' bias and pooled-value BN, in registers for the whole walk (loaded in
  // the epilogue they were dependent global round trips on every pool row)
  float bb[4][4], psc[4][4], psh[4][4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int ch = 32 * (n >> 1) + 8 * j + 4 * (n & 1);
    const float4 bv = *reinterpret_cast<const float4*>(bias + ch);
    const float4 sv = pscale ? *reinterpret_cast<const float4*>(pscale + ch) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 hv = pscale ? *reinterpret_cast<const float4*>(pshift + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
    bb[n][0] = bv.x, bb[n][1] = bv.y, bb[n][2] = bv.z, bb[n][3] = bv.w;
    psc[n][0] = sv.x, psc[n][1] = sv.y, psc[n][2] = sv.z, psc[n][3] = sv.w;
    psh[n][0] = hv.x, psh[n][1] = hv.y, psh[n][2] = hv.z, psh[n][3] = hv.w;
  }
  auto stem_val = [&](const f32x4 (&acc)[4][2], int m, int sy, float (&r)[4][4]) {
    const bool ok = sy >= 0 && sy < Hs && sx < Ws;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = acc[n][m][t] + bb[n][t];
        if (relu) v = fmaxf(v, 0.f);
        if constexpr (SPLIT) {
          uint16_t h, l;
          split1(v, h, l);
          v = bf2f(h) + bf2f(l);
        } else {
          v = bf2f(f2bf(v));
        }
        r[n][t] = ok ? v : -INFINITY;
      }
    }
  };
  float carry[4][4];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int t = 0; t < 4; ++t) carry[n][t] = -INFINITY;
  f32x4 acc[4][2];
  if (p0 > 0) {  // halo: stem row 2 p0 - 1 (the previous segment's last row)
    stem_rows(2 * p0 - 1, 1, acc);
    stem_val(acc, 0, 2 * p0 - 1, carry);
  }
  constexpr int PPT = 3;  // 4 new input rows x PXF pixels over >= 64 * CG threads (4 * (32 CG + 6) <= 3 * 64 CG)
  float pre[PPT][4];
  bool pin[PPT];
  for (int p = p0; p < p1; ++p) {
    const bool more = p + 1 < p1;
    if (more) {  // input rows 4 p + 6 .. 4 p + 9, in flight during the MFMAs
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int i = tid + k * nthr;
        const int ic = min(i, 4 * PXF - 1);
        pin[k] = load_px(4 * p + 6 + ic / PXF, ic % PXF, pre[k]);
      }
    }
    stem_rows(2 * p, 2, acc);
    float r0[4][4], r1[4][4], vm[4][4];
    stem_val(acc, 0, 2 * p, r0);
    stem_val(acc, 1, 2 * p + 1, r1);
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        vm[n][t] = fmaxf(fmaxf(carry[n][t], r0[n][t]), r1[n][t]);
        carry[n][t] = r1[n][t];
      }
    if (px_l == 15) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int t = 0; t < 4; ++t) xbuf[wave * NCH + 32 * (n >> 1) + 8 * j + 4 * (n & 1) + t] = vm[n][t];
    }
    __syncthreads();  // xbuf written; every wave done reading the ring rows the prefetch replaces
    float pv[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float left = dpp_shr1(vm[n][t]);
        const float right = dpp_shl1(vm[n][t]);
        if (px_l == 0) left = wave > 0 ? xbuf[(wave - 1) * NCH + 32 * (n >> 1) + 8 * j + 4 * (n & 1) + t] : -INFINITY;
        pv[n][t] = fmaxf(fmaxf(left, vm[n][t]), right);
      }
    const int pc = sx >> 1;
    if (!(px_l & 1) && pc < Wp) {
      uint16_t* o = out + ((static_cast<long long>(b) * Hp + p) * Wp + pc) * NCH;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const int ch = 32 * blk + 8 * j;
        float v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          v[t] = pv[2 * blk + (t >> 2)][t & 3];
          if (pscale) v[t] = v[t] * psc[2 * blk + (t >> 2)][t & 3] + psh[2 * blk + (t >> 2)][t & 3];
          if (pact == 1) v[t] = fmaxf(v[t], 0.f);
        }
        store8v(o + ch, oplane, SPLIT, v);
      }
    }
    if (more) {
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int i = tid + k * nthr;
        if (i < 4 * PXF) put(4 * p + 6 + i / PXF, i % PXF, pre[k], pin[k]);
      }
    }
    __syncthreads();  // new rows in the ring; xbuf free for the next row
  }
}

}  // namespace

static_assert(TY * TX * NCH <= NCH * WP, "output stage must fit in the weight buffer");

size_t stem_pool_lds_bytes(int Ws, int split) {
  const int CG = (Ws + 15) / 16, NP = split ? 2 : 1;
  return static_cast<size_t>(NP) * NCH * WP * 2 + static_cast<size_t>(NP) * RING * (32 * CG + 6) * 4 * 2 +
         static_cast<size_t>(CG) * NCH * 4;
}

bool stem_pool_supported(int H, int W, int Hs, int Ws, int Hp, int Wp, int split) {
  return Hs == (H + 6 - 7) / 2 + 1 && Ws == (W + 6 - 7) / 2 + 1 && Hp == (Hs + 2 - 3) / 2 + 1 &&
         Wp == (Ws + 2 - 3) / 2 + 1 && Ws >= 1 && (Ws + 15) / 16 <= 8 && stem_pool_lds_bytes(Ws, split) <= 160 * 1024;
}

hipError_t conv_stem_pool_nchw(const float* x, int C, const float* in_scale, const float* in_shift, const uint16_t* w,
                               const float* bias, int relu, const float* pscale, const float* pshift, int pact,
                               uint16_t* out, int B, int H, int W, int Hs, int Ws, int Hp, int Wp, hipStream_t s,
                               const long long* live, int split, int target_blocks) {
  if (C < 1 || C > 4 || B < 1 || !stem_pool_supported(H, W, Hs, Ws, Hp, Wp, split) || (pscale == nullptr) != (pshift == nullptr))
    return hipErrorInvalidValue;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  // segments of pool rows: about one block per CU over the batch (the halo row is recomputed per segment)
  const int want = std::max(1, (target_blocks > 0 ? target_blocks : cus) / B);
  const int seg_len = std::max(1, (Hp + want - 1) / want);
  const int segs = (Hp + seg_len - 1) / seg_len;
  const int CG = (Ws + 15) / 16;
  const size_t lds = stem_pool_lds_bytes(Ws, split);
  static const bool attr_set = [] {  // once, outside any graph capture's launches
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(stem_pool_nchw_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(stem_pool_nchw_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr_set;
  if (split) {
    hipLaunchKernelGGL(stem_pool_nchw_kernel<true>, dim3(B * segs), dim3(64 * CG), lds, s, x, C, in_scale, in_shift, w,
                       bias, relu, pscale, pshift, pact, out, B, H, W, Hs, Ws, Hp, Wp, seg_len, segs, live);
  } else {
    hipLaunchKernelGGL(stem_pool_nchw_kernel<false>, dim3(B * segs), dim3(64 * CG), lds, s, x, C, in_scale, in_shift, w,
                       bias, relu, pscale, pshift, pact, out, B, H, W, Hs, Ws, Hp, Wp, seg_len, segs, live);
  }
  return hipGetLastError();
}

hipError_t conv_stem7x7(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* out, int B, int H, int W,
                        int Ho, int Wo, int relu, hipStream_t s, const long long* live, int split) {
  if (Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1) return hipErrorInvalidValue;
  const int tiles_x = (Wo + TX - 1) / TX, tiles_y = (Ho + TY - 1) / TY;
  if (split)
    hipLaunchKernelGGL(stem7x7_kernel<true>, dim3(tiles_x * tiles_y, B), dim3(256), 0, s, x, w, bias, out, H, W, Ho,
                       Wo, relu, tiles_x, live);
  else
    hipLaunchKernelGGL(stem7x7_kernel<false>, dim3(tiles_x * tiles_y, B), dim3(256), 0, s, x, w, bias, out, H, W, Ho,
                       Wo, relu, tiles_x, live);
  return hipGetLastError();
}

hipError_t conv_stem7x7_nchw(const float* x, int C, const float* in_scale, const float* in_shift, const uint16_t* w,
                             const float* bias, uint16_t* out, int B, int H, int W, int Ho, int Wo, int relu,
                             hipStream_t s, const long long* live, int split, int max_blocks) {
  if (C < 1 || C > 4 || Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1) return hipErrorInvalidValue;
  const int tiles_x = (Wo + TX - 1) / TX, tiles_y = (Ho + TY - 1) / TY;
  const int per_img = tiles_x * tiles_y;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  int grid = std::min(B * per_img, max_blocks > 0 ? max_blocks : 2 * cus);  // 2 blocks (72 KiB LDS each) per CU
  grid = std::max(grid, 1);
  if (split)
    hipLaunchKernelGGL(stem7x7_nchw_kernel<true>, dim3(grid), dim3(SNT), 0, s, x, C, in_scale, in_shift, w, bias, out, B,
                       H, W, Ho, Wo, relu, tiles_x, per_img, live);
  else
    hipLaunchKernelGGL(stem7x7_nchw_kernel<false>, dim3(grid), dim3(SNT), 0, s, x, C, in_scale, in_shift, w, bias, out,
                       B, H, W, Ho, Wo, relu, tiles_x, per_img, live);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
