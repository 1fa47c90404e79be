// Device-side helpers shared by the CDNA4 (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace die {
namespace k {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

// float -> bf16, round to nearest even (gfx950 lowers this to v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return static_cast<uint32_t>(f2bf(a)) | (static_cast<uint32_t>(f2bf(b)) << 16);
}

__device__ __forceinline__ void unpack2(uint32_t v, float& a, float& b) {
  a = __uint_as_float(v << 16);
  b = __uint_as_float(v & 0xFFFF0000u);
}

// Exact-form GELU, 0.5 v (1 + erf(v / sqrt 2)) = 0.5 v erfc(-v / sqrt 2), with erfc from the
// Chebyshev fit of Numerical Recipes' erfcc (fractional error < 1.2e-7 for every argument) in place
// of ocml's erff: 1 rcp + 1 exp2 + 10 FMAs against ~45 instructions with lane-divergent branches.
// Written without the 1 + erf cancellation, so the negative tail keeps its relative accuracy: max
// relative error 5e-7 for v > -2 (below the split-fp32 representation error, 2^-17 = 7.6e-6) and
// 1.7e-5 in the negative tail v < -2 (ABOVE it, where |GELU(v)| < 0.046; max absolute error 4e-7
// over all v).  fp32-mode parity in that tail is therefore ~2e-5 relative; no reference fixture pins
// it (parity unpinned).  Replaces erff in the GEMM epilogues (ViT MLP1: 19M GELUs per batch-32 forward).
__device__ __forceinline__ float gelu_erf(float v) {
  const float z = fabsf(v) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float p = fmaf(0.17087277f, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float ec = t * __builtin_amdgcn_exp2f((p - z * z) * 1.4426950408889634f);  // erfc(|v| / sqrt 2)
  return v >= 0.f ? v * fmaf(-0.5f, ec, 1.f) : 0.5f * v * ec;
}

// ---- fp32 mode: split (hi, lo) bf16 planes -------------------------------------------------------
// A "split" tensor stores each fp32 value v as hi = bf16(v) in a hi plane and lo = bf16(v - hi) in a
// lo plane `plane` elements after it (same indexing in both).  hi + lo carries ~16 significant bits
// (relative representation error <= 2^-17), and a GEMM over split operands takes three bf16 MFMAs
// per fragment pair (hi*hi + lo*hi + hi*lo; the lo*lo term is below fp32 accumulation noise), so
// the matrix cores keep their bf16 rate (3x the work, ~5x the v_mfma_f32_*_f32 throughput).
__device__ __forceinline__ void split1(float v, uint16_t& hi, uint16_t& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}

// 8 values -> hi/lo 16-byte vectors.
__device__ __forceinline__ void split8(const float* v, uint4& hi, uint4& lo) {
  uint16_t h[8], l[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) split1(v[t], h[t], l[t]);
  hi = make_uint4(h[0] | (uint32_t(h[1]) << 16), h[2] | (uint32_t(h[3]) << 16), h[4] | (uint32_t(h[5]) << 16),
                  h[6] | (uint32_t(h[7]) << 16));
  lo = make_uint4(l[0] | (uint32_t(l[1]) << 16), l[2] | (uint32_t(l[3]) << 16), l[4] | (uint32_t(l[5]) << 16),
                  l[6] | (uint32_t(l[7]) << 16));
}

__device__ __forceinline__ void unpack8(const uint4 q, float* v) {
  unpack2(q.x, v[0], v[1]);
  unpack2(q.y, v[2], v[3]);
  unpack2(q.z, v[4], v[5]);
  unpack2(q.w, v[6], v[7]);
}

// Load 8 consecutive values (16-B aligned) of a bf16 tensor, or of a split tensor (hi + lo).
__device__ __forceinline__ void load8v(const uint16_t* p, long long plane, bool split, float* v) {
  unpack8(*reinterpret_cast<const uint4*>(p), v);
  if (split) {
    float w[8];
    unpack8(*reinterpret_cast<const uint4*>(p + plane), w);
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] += w[t];
  }
}

// Store 8 consecutive values as bf16, or split into the hi/lo planes.
__device__ __forceinline__ void store8v(uint16_t* p, long long plane, bool split, const float* v) {
  if (split) {
    uint4 hi, lo;
    split8(v, hi, lo);
    *reinterpret_cast<uint4*>(p) = hi;
    *reinterpret_cast<uint4*>(p + plane) = lo;
  } else {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
  }
}

__device__ __forceinline__ float load1v(const uint16_t* p, long long plane, bool split) {
  return split ? bf2f(p[0]) + bf2f(p[plane]) : bf2f(p[0]);
}

__device__ __forceinline__ void store1v(uint16_t* p, long long plane, bool split, float v) {
  if (split) {
    uint16_t h, l;
    split1(v, h, l);
    p[0] = h;
    p[plane] = l;
  } else {
    p[0] = f2bf(v);
  }
}

// Cross-lane moves on the VALU (DPP), no LDS round trip (ds_bpermute, which __shfl_xor compiles to,
// puts a dependent LDS latency on every exchange).  CTRL: quad_perm [1,0,3,2] = 0xB1 (lane ^ 1),
// [2,3,0,1] = 0x4E (lane ^ 2); row_half_mirror = 0x141 (lane i <-> 7-i within each 8 lanes).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// LayerNorm statistics partials (kernels.h ConvArgs::stats_out): the 8 consecutive, 8-aligned
// lanes that each hold 8 consecutive channels of one 64-channel group merge (mean, M2) of the 64
// values by three DPP exchanges (lane ^ 1, lane ^ 2, then the two quads, each uniform by then, so
// the mirror pairing is the xor-4 pairing).  Equal counts: mean = (a + b) / 2, M2 = M2a + M2b +
// d^2 n / 2 -- symmetric, so all 8 lanes end with identical bits.  Every lane of the 8 must call it.
__device__ __forceinline__ float2 group64_stats(const float* v) {
  float mu = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) mu += v[t];
  mu *= 0.125f;
  float m2 = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) m2 += (v[t] - mu) * (v[t] - mu);
  float cnt = 8.f;
  auto round = [&](float mu_o, float m2_o) {
    const float d = mu_o - mu;
    m2 = (m2 + m2_o) + d * d * (0.5f * cnt);
    mu = 0.5f * (mu + mu_o);
    cnt *= 2.f;
  };
  round(dpp<0xB1>(mu), dpp<0xB1>(m2));
  round(dpp<0x4E>(mu), dpp<0x4E>(m2));
  round(dpp<0x141>(mu), dpp<0x141>(m2));
  return make_float2(mu, m2);
}

}  // namespace k
}  // namespace die
