// Memory-bound NHWC kernels for gfx950: input preparation, pooling, global average pooling,
// standalone affine/activation, layout conversion.  All loads/stores are 16-byte vectors (8 bf16)
// except where the layout forbids it; grids are capped and grid-strided.
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

inline int grid_for(long long work, int block = 256, int cap = 4096) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  return static_cast<int>(g > cap ? cap : g);
}

// fp32 NCHW -> affine -> bf16 NHWC (Cp channels; Cp in {4, 8}), one thread per pixel.
template <int CP>
__global__ void input_prep_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                  const float* __restrict__ shift, uint16_t* __restrict__ out, int B, int C, int HW,
                                  int split) {
  const long long total = static_cast<long long>(B) * HW;
  const long long plane = total * CP;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long b = i / HW;
    const long long p = i - b * HW;
    float v[CP];
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      if (c < C) {
        const float xv = x[(b * C + c) * HW + p];
        v[c] = scale ? xv * scale[c] + shift[c] : xv;
      } else {
        v[c] = 0.f;
      }
    }
    if (CP == 4) {
      uint16_t h[4], l[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) split1(v[c], h[c], l[c]);
      *reinterpret_cast<uint2*>(out + i * 4) = make_uint2(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16));
      if (split)
        *reinterpret_cast<uint2*>(out + plane + i * 4) =
            make_uint2(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16));
    } else {
      store8v(out + i * 8, plane, split != 0, v);
    }
  }
}


// One thread per (output pixel, 8-channel group).
__global__ void pool2d_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B, int H, int W, int C,
                              int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int is_max, int cip,
                              const long long* __restrict__ live, const float* __restrict__ scale,
                              const float* __restrict__ shift, int act, int split) {
  const long long xplane = static_cast<long long>(B) * H * W * C, yplane = static_cast<long long>(B) * Ho * Wo * C;
  if (live) B = min(B, static_cast<int>(*live));
  const int CG = C / 8;
  const long long total = static_cast<long long>(B) * Ho * Wo * CG;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int cg = static_cast<int>(i % CG);
    long long r = i / CG;
    const int ow = static_cast<int>(r % Wo);
    r /= Wo;
    const int oh = static_cast<int>(r % Ho);
    const int b = static_cast<int>(r / Ho);
    float acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = is_max ? -INFINITY : 0.f;
    int cnt = 0;
    for (int ky = 0; ky < kh; ++ky) {
      const int ih = oh * sh - ph + ky;
      for (int kx = 0; kx < kw; ++kx) {
        const int iw = ow * sw - pw + kx;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) {
          if (cip && ih < H + ph && iw < W + pw) ++cnt;
          continue;
        }
        float v[8];
        load8v(x + ((static_cast<long long>(b) * H + ih) * W + iw) * C + cg * 8, xplane, split != 0, v);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = is_max ? fmaxf(acc[t], v[t]) : acc[t] + v[t];
        ++cnt;
      }
    }
    if (!is_max) {
      const float inv = cnt ? 1.f / cnt : 0.f;
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] *= inv;
    }
    if (scale) {  // fused per-channel affine (+ ReLU) on the pooled value
      const float4 s0 = *reinterpret_cast<const float4*>(scale + cg * 8), s1 = *reinterpret_cast<const float4*>(scale + cg * 8 + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(shift + cg * 8), h1 = *reinterpret_cast<const float4*>(shift + cg * 8 + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sf[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = acc[t] * sc[t] + sf[t];
    }
    if (act == 1) {
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = fmaxf(acc[t], 0.f);
    }
    store8v(y + i * 8, yplane, split != 0, acc);
  }
}

// Grid: (C/8 groups / 8, B) blocks of 256 threads = 8 channel groups x 32 row-slices.  ResNet50's
// head (B~20, 7x7x2048) gets 16x more blocks than one-block-per-64-groups and each thread issues
// its ~3 16-byte loads back to back, so the 4 MB read is not latency-bound on ~80 blocks.
// mode 0 mean, 1 sum, 2 max over the HW pixels of each (sample, channel)
// G 8-channel groups x S = 256 / G pixel slices per block.  G = 32 for wide maps (ResNet50's 2048
// channels): a wave reads 512 contiguous bytes of one pixel row per plane and the slice reduction is
// 8 deep; G = 8 keeps narrow maps (C < 256) from idling most of the block.
template <int G>
__global__ __launch_bounds__(256) void gap_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out,
                                                  float* __restrict__ out_f32, const float* __restrict__ scale,
                                                  const float* __restrict__ shift, int relu, int HW, int C,
                                                  const long long* __restrict__ live, int split, int mode) {
  const long long xplane = static_cast<long long>(gridDim.y) * HW * C, oplane = static_cast<long long>(gridDim.y) * C;
  constexpr int S = 256 / G;
  __shared__ float part[S][G][9];  // +1 pad: the reduction reads S slices of one group
  const int b = blockIdx.y;
  if (live && b >= *live) return;  // whole block: before any barrier
  const int gl = threadIdx.x % G, slice = threadIdx.x / G;
  const int g = blockIdx.x * G + gl;
  const int CG = C / 8;
  const float init = mode == 2 ? -INFINITY : 0.f;
  float acc[8] = {init, init, init, init, init, init, init, init};
  if (g < CG) {
    float sc[8], sf[8];
    auto load_affine = [&]() {  // 16-B loads (g * 8 floats is 32-B aligned)
      if (scale) {
        const float4 s0 = *reinterpret_cast<const float4*>(scale + g * 8), s1 = *reinterpret_cast<const float4*>(scale + g * 8 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(shift + g * 8), h1 = *reinterpret_cast<const float4*>(shift + g * 8 + 4);
        sc[0] = s0.x, sc[1] = s0.y, sc[2] = s0.z, sc[3] = s0.w, sc[4] = s1.x, sc[5] = s1.y, sc[6] = s1.z, sc[7] = s1.w;
        sf[0] = h0.x, sf[1] = h0.y, sf[2] = h0.z, sf[3] = h0.w, sf[4] = h1.x, sf[5] = h1.y, sf[6] = h1.z, sf[7] = h1.w;
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) sc[t] = 1.f, sf[t] = 0.f;
      }
    };
    const uint16_t* src = x + static_cast<long long>(b) * HW * C + g * 8;
    auto add = [&](const float* v) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        float u = v[t] * sc[t] + sf[t];
        if (relu) u = fmaxf(u, 0.f);
        acc[t] = mode == 2 ? fmaxf(acc[t], u) : acc[t] + u;
      }
    };
    constexpr int MAXP = 8;  // pixels per thread in one round of loads (ResNet50's 7x7 map: 6-7 with S = 8)
    if (HW <= MAXP * S) {
      // Every load of the thread in flight at once (one memory round trip), as raw buffer loads: a
      // pixel past the map (and the lo plane of a bf16 map) sits at an offset past num_records and
      // reads as 0, so no per-lane branch surrounds a load (the loop below compiles to one wait per
      // pixel).  Sums in pixel order, as the loop below.
      const long long planeb = xplane * 2;  // bytes per plane
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(x), 0, static_cast<int>(split ? 2 * planeb : planeb), 0x00020000);
      const unsigned base = static_cast<unsigned>((static_cast<long long>(b) * HW * C + g * 8) * 2);
      uint4 hi[MAXP], lo[MAXP];
#pragma unroll
      for (int k = 0; k < MAXP; ++k) {
        const int p = slice + k * S;
        const unsigned off = p < HW ? base + static_cast<unsigned>(p * C * 2) : 0x80000000u;
        hi[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        lo[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                              xr, split ? off + static_cast<unsigned>(planeb) : 0x80000000u, 0, 0));
      }
      load_affine();  // after the pixel loads: one round trip for both
#pragma unroll
      for (int k = 0; k < MAXP; ++k) {
        if (slice + k * S < HW) {
          float v[8];
          unpack8(hi[k], v);
          if (split) {
            float w[8];
            unpack8(lo[k], w);
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] += w[t];
          }
          add(v);
        }
      }
    } else {
      load_affine();
#pragma unroll 4
      for (int p = slice; p < HW; p += S) {
        float v[8];
        load8v(src + static_cast<long long>(p) * C, xplane, split != 0, v);
        add(v);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) part[slice][gl][t] = acc[t];
  __syncthreads();
  if (slice == 0 && g < CG) {
    const float inv = mode == 0 ? 1.f / HW : 1.f;
    float r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float sum = mode == 2 ? -INFINITY : 0.f;
#pragma unroll
      for (int k = 0; k < S; ++k) sum = mode == 2 ? fmaxf(sum, part[k][gl][t]) : sum + part[k][gl][t];
      r[t] = sum * inv;
    }
    if (out) store8v(out + static_cast<long long>(b) * C + g * 8, oplane, split != 0, r);
    if (out_f32) {
      float4* o = reinterpret_cast<float4*>(out_f32 + static_cast<long long>(b) * C + g * 8);
      o[0] = make_float4(r[0], r[1], r[2], r[3]);
      o[1] = make_float4(r[4], r[5], r[6], r[7]);
    }
  }
}

// Global pool + fully-connected head in one launch (ResNet: [B, 7x7, 2048] -> mean -> 2048 x 1000
// GEMM at B ~ 20, where the GEMM is far too small for MFMA tiles and two launches cost ~30 us).
// Block (slice, group): pools channels [c0, c0 + CS) of every live sample into LDS in fp32 (hi + lo
// planes), dots them with the group's <= kGfcCls weight rows (hi + lo -> fp32, VALU FMAs), and
// writes the partial logits [slice][b][n] with write-through (sc1) stores.  The last slice block of
// a group to arrive (one agent-scope ticket per group, the hand-off of the fused split-K epilogue in
// conv_igemm_impl.h) sums the slices in slice order -- deterministic -- adds the bias (+ ReLU) and
// writes the fp32 logits.
constexpr int kGfcRows = 32;   // samples per LDS chunk
constexpr int kGfcCls = 128;   // classes per block: 2 threads per class, each half of the samples
constexpr int kGfcPS = 4;      // pixel slices per (sample, 8-channel group) in the pooling
constexpr int kCpolSc1Gfc = 16;

// CS <= 64: a thread holds its class's CS weights in registers and finishes each sample's partial
// in one pass (a 64-row accumulator array plus 64 weights spilled 6 KB per lane to scratch: 49 us of
// a 73 us kernel).  The pooling splits each (sample, 8-channel group) over kGfcPS pixel slices whose
// sums meet in LDS in slice order (deterministic).
template <int CS>
__global__ __launch_bounds__(256) void gap_fc_kernel(const uint16_t* __restrict__ x, long long xplane, int HW, int C,
                                                     int mode, const uint16_t* __restrict__ w, long long wplane, int Kpad,
                                                     const float* __restrict__ bias, int N, int act,
                                                     float* __restrict__ out, float* ws, int* counters,
                                                     const long long* __restrict__ live, int B, int split,
                                                     int stop) {
  static_assert(CS % 8 == 0 && CS <= 64, "channel slice");
  __shared__ __attribute__((aligned(16))) float part[kGfcPS][kGfcRows][CS];
  __shared__ int flag;
  const int slice = blockIdx.x, grp = blockIdx.y, tid = threadIdx.x;
  const int c0 = slice * CS, n0 = grp * kGfcCls;
  const int Bl = live ? static_cast<int>(min(*live, static_cast<long long>(B))) : B;
  const int nl = tid % kGfcCls, half = tid / kGfcCls;
  const int n = n0 + nl;
  const float inv = mode == 0 ? 1.f / HW : 1.f;
  const float init = mode == 2 ? -INFINITY : 0.f;
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(ws, 0, 0x7fffffff, 0x00020000);
  constexpr int GPR = CS / 8;
  float wv[CS];  // this thread's class row of the weights (hi + lo), loaded once
  if (n < N) {
    const uint16_t* wr = w + static_cast<long long>(n) * Kpad + c0;
#pragma unroll
    for (int q = 0; q < GPR; ++q) load8v(wr + q * 8, wplane, split != 0, wv + q * 8);
  }
  for (int b0 = 0; b0 < Bl; b0 += kGfcRows) {
    const int nb = min(kGfcRows, Bl - b0);
    // pooling: item = (sample, pixel slice, 8-channel group), the group fastest (128-B rows)
    for (int it = tid; it < nb * GPR * kGfcPS; it += 256) {
      const int g = it % GPR, rest = it / GPR, ps = rest % kGfcPS, bi = rest / kGfcPS;
      const uint16_t* src = x + static_cast<long long>(b0 + bi) * HW * C + c0 + g * 8;
      float acc[8] = {init, init, init, init, init, init, init, init};
#pragma unroll 4
      for (int p = ps; p < HW; p += kGfcPS) {
        float v[8];
        load8v(src + static_cast<long long>(p) * C, xplane, split != 0, v);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mode == 2 ? fmaxf(acc[t], v[t]) : acc[t] + v[t];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) part[ps][bi][g * 8 + t] = acc[t];
    }
    __syncthreads();
    for (int e = tid; e < nb * CS; e += 256) {
      const int bi = e / CS, j = e - bi * CS;
      float v = part[0][bi][j];
#pragma unroll
      for (int ps = 1; ps < kGfcPS; ++ps) v = mode == 2 ? fmaxf(v, part[ps][bi][j]) : v + part[ps][bi][j];
      part[0][bi][j] = v * inv;
    }
    __syncthreads();
    if (stop == 1) return;
    if (n < N) {
      for (int bi = half; bi < nb; bi += 2) {
        const float4* pr = reinterpret_cast<const float4*>(&part[0][bi][0]);
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < CS / 4; ++q) {
          const float4 u = pr[q];
          s += u.x * wv[4 * q] + u.y * wv[4 * q + 1] + u.z * wv[4 * q + 2] + u.w * wv[4 * q + 3];
        }
        const unsigned off = static_cast<unsigned>(((static_cast<long long>(slice) * B + b0 + bi) * N + n) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s), wsr, off, 0, kCpolSc1Gfc);
      }
    }
    __syncthreads();  // part is rewritten by the next chunk
  }
  if (stop == 2) return;
  // hand-off: every wave drains its write-through stores, one lane takes the group's ticket; the
  // last arriver's lane runs ONE agent acquire and waits for it before the barrier that releases
  // the other waves onto the partials (MI355X_MICROARCH "Valid forms", "Consumer, always": several
  // blocks share a CU here, so sc1 loads alone do not qualify; same form as conv tile_epilogue)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(counters + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == static_cast<int>(gridDim.x) - 1;
    if (last) {
      __hip_atomic_store(counters + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    flag = last;
  }
  __syncthreads();
  if (!flag || stop == 3) return;
  // The slices' partials are summed in slice order, 8 slices' loads in flight at a time (a serial
  // load -> add chain over 32 slices x 10 items per thread took 165 us at ResNet50's B = 20); with
  // N % 4 == 0 each item is 4 consecutive classes (16-B loads and stores).
  const int ncls = min(kGfcCls, N - n0);
  const int KS = static_cast<int>(gridDim.x);
  const unsigned slab = static_cast<unsigned>(static_cast<long long>(B) * N * 4);  // bytes per slice
  if ((N & 3) == 0) {
    const int nq = ncls / 4;
    for (int it = tid; it < Bl * nq; it += 256) {
      const int bi = it / nq, nn = n0 + 4 * (it - bi * nq);
      const unsigned base = static_cast<unsigned>((static_cast<long long>(bi) * N + nn) * 4);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      int sl = 0;
      for (; sl + 8 <= KS; sl += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wsr, base + (sl + u) * slab, 0,
                                                                                  kCpolSc1Gfc));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc.x += v[u].x;
          acc.y += v[u].y;
          acc.z += v[u].z;
          acc.w += v[u].w;
        }
      }
      for (; sl < KS; ++sl) {
        const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wsr, base + sl * slab, 0,
                                                                                          kCpolSc1Gfc));
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
      float r[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (bias) r[t] += bias[nn + t];
        if (act == 1) r[t] = fmaxf(r[t], 0.f);
      }
      *reinterpret_cast<float4*>(out + static_cast<long long>(bi) * N + nn) = make_float4(r[0], r[1], r[2], r[3]);
    }
    return;
  }
  for (int it = tid; it < Bl * ncls; it += 256) {
    const int bi = it / ncls, nn = n0 + (it - bi * ncls);
    const unsigned base = static_cast<unsigned>((static_cast<long long>(bi) * N + nn) * 4);
    float s = 0.f;
    int sl = 0;
    for (; sl + 8 <= KS; sl += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wsr, base + (sl + u) * slab, 0, kCpolSc1Gfc));
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; sl < KS; ++sl)
      s += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wsr, base + sl * slab, 0, kCpolSc1Gfc));
    if (bias) s += bias[nn];
    if (act == 1) s = fmaxf(s, 0.f);
    out[static_cast<long long>(bi) * N + nn] = s;
  }
}

// act: 0 none, 1 relu.  One thread per 8 elements of a row of C (C % 8 == 0).
__global__ void affine_act_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ z,
                                  const float* __restrict__ scale, const float* __restrict__ shift, int act,
                                  uint16_t* __restrict__ y, long long M, int C, const long long* __restrict__ live,
                                  long long rows_per_sample, int split, float clip_lo, float clip_hi) {
  const long long plane = M * C;
  if (live) M = min(M, *live * rows_per_sample);
  const int CG = C / 8;
  const long long total = M * CG;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int c0 = static_cast<int>(i % CG) * 8;
    float v[8];
    load8v(x + i * 8, plane, split != 0, v);
    if (scale) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = v[t] * scale[c0 + t] + shift[c0 + t];
    }
    if (z) {
      float w[8];
      load8v(z + i * 8, plane, split != 0, w);
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += w[t];
    }
    if (act == 1) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
    } else if (act == 3) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = fminf(fmaxf(v[t], clip_lo), clip_hi);
    }
    store8v(y + i * 8, plane, split != 0, v);
  }
}

__global__ void nhwc_to_nchw_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int B, int HW, int C,
                                        int split) {
  const long long total = static_cast<long long>(B) * HW * C;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    // i indexes the OUTPUT (NCHW) so the f32 stores are coalesced.
    const long long p = i % HW;
    long long r = i / HW;
    const long long c = r % C;
    const long long b = r / C;
    y[i] = load1v(x + (b * HW + p) * C + c, total, split != 0);
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ void bf16_to_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, long long n, int split) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    y[i] = load1v(x + i, n, split != 0);
}

}  // namespace

hipError_t input_prep(const float* x, const float* scale, const float* shift, uint16_t* out, int B, int C, int H,
                      int W, int Cp, hipStream_t s, int split) {
  if (C > Cp || (Cp != 4 && Cp != 8)) return hipErrorInvalidValue;
  const long long work = static_cast<long long>(B) * H * W;
  if (Cp == 4)
    hipLaunchKernelGGL(input_prep_kernel<4>, dim3(grid_for(work)), dim3(256), 0, s, x, scale, shift, out, B, C, H * W, split);
  else
    hipLaunchKernelGGL(input_prep_kernel<8>, dim3(grid_for(work)), dim3(256), 0, s, x, scale, shift, out, B, C, H * W, split);
  return hipGetLastError();
}

hipError_t pool2d(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh,
                  int sw, int ph, int pw, int is_max, int count_include_pad, hipStream_t s, const long long* live,
                  const float* scale, const float* shift, int act, int split) {
  if (C % 8) return hipErrorInvalidValue;
  const long long work = static_cast<long long>(B) * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(pool2d_kernel, dim3(grid_for(work)), dim3(256), 0, s, x, y, B, H, W, C, Ho, Wo, kh, kw, sh, sw,
                     ph, pw, is_max, count_include_pad, live, scale, shift, act, split);
  return hipGetLastError();
}

hipError_t global_avgpool(const uint16_t* x, uint16_t* out, float* out_f32, const float* scale, const float* shift,
                          int relu, int B, int HW, int C, hipStream_t s, const long long* live, int split, int mode) {
  if (C % 8 || mode < 0 || mode > 2) return hipErrorInvalidValue;
  const int CG = C / 8;
  if (CG >= 32) {  // 32 channel groups x 8 pixel slices per block
    hipLaunchKernelGGL(gap_kernel<32>, dim3((CG + 31) / 32, B), dim3(256), 0, s, x, out, out_f32, scale, shift, relu,
                       HW, C, live, split, mode);
  } else {  // 8 channel groups x 32 pixel slices per block
    hipLaunchKernelGGL(gap_kernel<8>, dim3((CG + 7) / 8, B), dim3(256), 0, s, x, out, out_f32, scale, shift, relu, HW,
                       C, live, split, mode);
  }
  return hipGetLastError();
}

// Channel slice: the narrowest that divides C with at most 32 slices (ResNet50: 64 -> 32 x 8 =
// 256 blocks), else the narrowest that divides C; the partials [C/cs][B][N] must fit `ws`.
namespace {
int g_gfc_stop = 0;  // measurement: 1 / 2 / 3 = return after the pooling / the partials / the ticket
}
void set_gap_fc_stop(int v) { g_gfc_stop = v; }

int gap_fc_slice(int C, int B, int N, size_t ws_bytes) {
  static const int kSlices[] = {8, 16, 32, 64};
  auto fits = [&](int cs) {
    const size_t bytes = static_cast<size_t>(C / cs) * B * N * 4;
    return C % cs == 0 && bytes <= ws_bytes && bytes < (size_t(1) << 31);
  };
  for (int cs : kSlices)
    if (C / cs <= 32 && fits(cs)) return cs;
  for (int cs : kSlices)
    if (fits(cs)) return cs;
  return 0;
}

hipError_t gap_fc(const uint16_t* x, int B, int HW, int C, int mode, const uint16_t* w, long long wplane, int Kpad,
                  const float* bias, int N, int act, float* out, float* ws, size_t ws_bytes, int* counters,
                  int counters_n, hipStream_t s, const long long* live, int split) {
  const int cs = gap_fc_slice(C, B, N, ws_bytes);
  const int groups = (N + kGfcCls - 1) / kGfcCls;
  if (!cs || mode < 0 || mode > 2 || Kpad < C || Kpad % 8 || groups > counters_n || act < 0 || act > 1 || !counters ||
      !ws)
    return hipErrorInvalidValue;
  const long long xplane = static_cast<long long>(B) * HW * C;
  dim3 grid(C / cs, groups);
#define GAP_FC_CASE(CSV)                                                                                          \
  case CSV:                                                                                                        \
    hipLaunchKernelGGL(gap_fc_kernel<CSV>, grid, dim3(256), 0, s, x, xplane, HW, C, mode, w, wplane, Kpad, bias, N, \
                       act, out, ws, counters, live, B, split, g_gfc_stop);                                        \
    break;
  switch (cs) {
    GAP_FC_CASE(8)
    GAP_FC_CASE(16)
    GAP_FC_CASE(32)
    GAP_FC_CASE(64)
    default:
      return hipErrorInvalidValue;
  }
#undef GAP_FC_CASE
  return hipGetLastError();
}

hipError_t affine_act(const uint16_t* x, const uint16_t* z, const float* scale, const float* shift, int act,
                      uint16_t* y, long long M, int C, hipStream_t s, const long long* live, long long rows_per_sample,
                      int split, float clip_lo, float clip_hi) {
  if (C % 8) return hipErrorInvalidValue;
  if (live && rows_per_sample <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(affine_act_kernel, dim3(grid_for(M * (C / 8))), dim3(256), 0, s, x, z, scale, shift, act, y, M,
                     C, live, rows_per_sample, split, clip_lo, clip_hi);
  return hipGetLastError();
}

hipError_t nhwc_to_nchw_f32(const uint16_t* x, float* y, int B, int H, int W, int C, hipStream_t s, int split) {
  const long long work = static_cast<long long>(B) * H * W * C;
  hipLaunchKernelGGL(nhwc_to_nchw_f32_kernel, dim3(grid_for(work)), dim3(256), 0, s, x, y, B, H * W, C, split);
  return hipGetLastError();
}

hipError_t f32_to_bf16(const float* x, uint16_t* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}

// Pull a small per-batch table written by the host into device memory from inside a captured graph
// (src = host-coherent pinned memory): no SDMA copy that could queue behind bulk uploads.
__global__ void copy_i64_kernel(const long long* __restrict__ src, long long* __restrict__ dst, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = __builtin_nontemporal_load(src + i);
}

// Reads n float4 (grid-stride) and sinks a value that is never produced by real data.
__global__ void l2_scrub_kernel(const float4* __restrict__ buf, long long n, float* __restrict__ sink) {
  float acc = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += static_cast<long long>(gridDim.x) * 256) {
    const float4 v = buf[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1.2345678e30f) *sink = acc;
}

hipError_t l2_scrub(const void* buf, size_t bytes, float* sink, hipStream_t s) {
  hipLaunchKernelGGL(l2_scrub_kernel, dim3(2048), dim3(256), 0, s, static_cast<const float4*>(buf),
                     static_cast<long long>(bytes / 16), sink);
  return hipGetLastError();
}

hipError_t copy_i64(const long long* src, long long* dst, int n, hipStream_t s) {
  hipLaunchKernelGGL(copy_i64_kernel, dim3(1), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

hipError_t bf16_to_f32(const uint16_t* x, float* y, long long n, hipStream_t s, int split) {
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n, split);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
