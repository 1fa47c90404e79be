// Transformer (ViT) kernels for gfx950: LayerNorm over rows, token assembly (cls + patches +
// position embedding), row gather, and fused multi-head attention on MFMA.
//
// These replace what ONNX Runtime would run for a ViT-B/16 export (LayerNormalization, the
// MatMul -> Div -> Softmax -> MatMul attention chain with its Reshape/Transpose views, Concat/Add
// of the embeddings, Gather of the cls token).  Layouts: activations are bf16 rows [B*S, C] with the
// head h occupying columns [h*D, (h+1)*D) (no transposes are ever materialised).
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over aligned groups of LPR lanes (LPR = 64: the whole wave).
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD affinity for row kernels that read what a GEMM just wrote: the GEMM's XCD-aware mapping
// (conv_igemm_impl.h block_coords) gives XCD x roughly the x-th eighth of the output rows, and
// blocks are dealt round-robin over the 8 XCDs (id % 8).  Block id b -> logical block: XCD b % 8
// takes the (b % 8)-th contiguous eighth of the blocks, so the rows are read where they were
// written (that XCD's L2) instead of through the Infinity Cache.  Bijective for any block count.
__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb, int xcd) {
  if (!xcd) return b;
  const unsigned x = b & 7, k = b >> 3, q = nb >> 3, r = nb & 7;
  return x * q + (x < r ? x : r) + k;
}

// LPR lanes per row (64 / LPR rows per wave); each lane holds up to CPL 8-element chunks of the row
// in registers (two-pass mean/variance in fp32).  C % 8 == 0 (stored pitch), C <= LPR*8*CPL; the
// statistics run over the first Cl (logical) columns and the pad columns are written 0.  C = 768
// (ViT-B) runs as 32 lanes x 3 chunks: every lane busy and two rows' loads in flight per wave (one
// row per wave with 64 x 2 chunks left half the lanes idle in the second round).
// stats != nullptr: statistics mode -- (mean, rstd) per row to stats[2 row], y is not written (the
// normalisation is folded into the consuming GEMM, ConvArgs::row_stats).
template <int CPL, int LPR = 64>
__global__ __launch_bounds__(256) void layernorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        float eps, long long rows, int C, int split, int Cl,
                                                        float* __restrict__ stats, int xcd) {
  constexpr int RPB = 256 / LPR;  // rows per block
  const int lane = threadIdx.x & (LPR - 1);
  const long long row = static_cast<long long>(xcd_block(blockIdx.x, gridDim.x, xcd)) * RPB + (threadIdx.x / LPR);
  if (row >= rows) return;  // a whole row group; the shuffles below stay inside it
  const long long plane = rows * C;
  const int nch = C / 8;
  const uint16_t* xr = x + row * C;
  float v[CPL][8];
  float4 gv[CPL][2], bv[CPL][2];  // gamma / beta fetched with the row, off the reduction's critical path
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + LPR * i;
    if (c < nch) {
      gv[i][0] = *reinterpret_cast<const float4*>(g + c * 8);
      gv[i][1] = *reinterpret_cast<const float4*>(g + c * 8 + 4);
      bv[i][0] = *reinterpret_cast<const float4*>(b + c * 8);
      bv[i][1] = *reinterpret_cast<const float4*>(b + c * 8 + 4);
      load8v(xr + c * 8, plane, split != 0, v[i]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (c * 8 + t >= Cl) v[i][t] = 0.f;  // pad columns: out of the statistics
        s += v[i][t];
      }
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[i][t] = 0.f;
    }
  }
  const float mean = group_sum<LPR>(s) / Cl;
  float q2 = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    if (lane + LPR * i < nch) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float d = (lane + LPR * i) * 8 + t < Cl ? v[i][t] - mean : 0.f;
        q2 += d * d;
      }
    }
  const float inv = rsqrtf(group_sum<LPR>(q2) / Cl + eps);
  if (stats) {
    if (lane == 0) *reinterpret_cast<float2*>(stats + 2 * row) = make_float2(mean, inv);
    return;
  }
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + LPR * i;
    if (c >= nch) continue;
    const float gg[8] = {gv[i][0].x, gv[i][0].y, gv[i][0].z, gv[i][0].w, gv[i][1].x, gv[i][1].y, gv[i][1].z, gv[i][1].w};
    const float bb[8] = {bv[i][0].x, bv[i][0].y, bv[i][0].z, bv[i][0].w, bv[i][1].x, bv[i][1].y, bv[i][1].z, bv[i][1].w};
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] = c * 8 + t < Cl ? (v[i][t] - mean) * inv * gg[t] + bb[t] : 0.f;
    store8v(y + row * C + c * 8, plane, split != 0, o);
  }
}

// Rows wider than the register kernels hold (C > 2048): one 256-thread block per row, the row read
// twice from global / L2 (sum, then squared deviations) and once more for the output; block
// reductions through LDS.
__global__ __launch_bounds__(256) void layernorm_wide_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                             const float* __restrict__ g, const float* __restrict__ b,
                                                             float eps, long long rows, int C, int split, int Cl,
                                                             float* __restrict__ stats, int xcd) {
  __shared__ float red[8];
  const long long row = xcd_block(blockIdx.x, gridDim.x, xcd);
  const long long plane = rows * C;
  const uint16_t* xr = x + row * C;
  const int nch = C / 8, tid = threadIdx.x;
  auto block_sum = [&](float v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();  // red[] free (previous reduction read)
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  float s = 0.f;
  for (int c = tid; c < nch; c += 256) {
    float v[8];
    load8v(xr + c * 8, plane, split != 0, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) s += c * 8 + t < Cl ? v[t] : 0.f;
  }
  const float mean = block_sum(s) / Cl;
  float q2 = 0.f;
  for (int c = tid; c < nch; c += 256) {
    float v[8];
    load8v(xr + c * 8, plane, split != 0, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float d = c * 8 + t < Cl ? v[t] - mean : 0.f;
      q2 += d * d;
    }
  }
  const float inv = rsqrtf(block_sum(q2) / Cl + eps);
  if (stats) {
    if (tid == 0) *reinterpret_cast<float2*>(stats + 2 * row) = make_float2(mean, inv);
    return;
  }
  for (int c = tid; c < nch; c += 256) {
    float v[8];
    load8v(xr + c * 8, plane, split != 0, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = c * 8 + t < Cl ? (v[t] - mean) * inv * g[c * 8 + t] + b[c * 8 + t] : 0.f;
    store8v(y + row * C + c * 8, plane, split != 0, v);
  }
}

// out[b, 0, :] = cls + pos[0];  out[b, 1 + s, :] = patches[b, s, :] + pos[1 + s]
// stats (nullable, C % 64 == 0): LayerNorm statistics partials of the assembled rows, [B*S][C/64]
// float2 (mean, M2) -- ConvArgs::stats_out's layout, for a folded reader's row_parts.  The grid-stride
// loop keeps 8-aligned lane groups on one 64-channel group (256-thread blocks, total % 8 == 0).
__global__ void tokens_kernel(const uint16_t* __restrict__ patches, const float* __restrict__ cls,
                              const float* __restrict__ pos, uint16_t* __restrict__ out, int B, int S0, int C,
                              int split, float* __restrict__ stats) {
  const int S = S0 + 1;
  const int CG = C / 8;
  const long long total = static_cast<long long>(B) * S * CG;
  const long long pplane = static_cast<long long>(B) * S0 * C, oplane = static_cast<long long>(B) * S * C;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int cg = static_cast<int>(i % CG);
    const long long r = i / CG;
    const int s = static_cast<int>(r % S);
    const long long b = r / S;
    float v[8];
    if (s == 0) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = cls ? cls[cg * 8 + t] : 0.f;
    } else {
      load8v(patches + ((b * S0 + s - 1) * C + cg * 8), pplane, split != 0, v);
    }
    if (pos) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += pos[static_cast<long long>(s) * C + cg * 8 + t];
    }
    if (stats) {
      const float2 st = group64_stats(v);
      if ((cg & 7) == 0) reinterpret_cast<float2*>(stats)[r * (C / 64) + cg / 8] = st;
    }
    store8v(out + i * 8, oplane, split != 0, v);
  }
}

__global__ void gather_rows_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B, int S, int idx,
                                   int C, int split) {
  const int CG = C / 8;
  const long long total = static_cast<long long>(B) * CG;
  const long long xplane = static_cast<long long>(B) * S * C, yplane = static_cast<long long>(B) * C;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const long long b = i / CG;
    const int cg = static_cast<int>(i % CG);
    const uint16_t* src = x + ((b * S + idx) * C + cg * 8);
    *reinterpret_cast<uint4*>(y + i * 8) = *reinterpret_cast<const uint4*>(src);
    if (split) *reinterpret_cast<uint4*>(y + yplane + i * 8) = *reinterpret_cast<const uint4*>(src + xplane);
  }
}

// ---- fused attention ------------------------------------------------------------------------------
// FlashAttention-style, on v_mfma_f32_32x32x16_bf16, for head dim 64 and S <= 256 (ViT: 197 tokens).
// A block = one (image b, head h) pair, 8 waves (two per SIMD); wave w owns query tile w (32 queries).
// K and V of the pair are staged in LDS once (K with XOR-swizzled 16-B chunks, V in plain rows padded
// to 96 elements so the transposed reads below are bank-conflict free); every thread issues all of
// its staging loads before its first LDS write, so the whole K/V image is in flight at once (round 2
// staged it in dependent load->store rounds from two blocks per pair: 52 us per ViT layer at B=32).
//  * S^T = K Q^T (A = K rows from LDS, B = this wave's Q fragments kept in registers): the result has
//    the QUERY on the lane and 32 KEYS in the 16 accumulator registers x 2 lane halves, so the
//    softmax over keys is in-lane plus one xor-32 shuffle (online softmax across key tiles, exp2).
//  * O^T += V^T P^T takes P^T straight from the accumulator registers as the B operand (no LDS, no
//    lane movement: register 8s+j of lane half h is key 16s + 8(j>>2) + 4h + (j&3)); the A operand
//    V^T comes from the row-major V image through ds_read_b64_tr_b16 (hardware transpose), two
//    4-key reads per k-step in exactly that key order.
constexpr int AT_D = 64;
constexpr int VP = 96;  // V row pitch (elements)
#ifndef DIE_ATTN_STREAM
#define DIE_ATTN_STREAM 1
#endif
constexpr bool kAttnStream = DIE_ATTN_STREAM != 0;  // streaming (tiled K/V) attention kernel

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x4 ds_read_tr16(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(const_cast<uint16_t*>(p)));
}

// SPLIT (fp32 mode): Q, K, V and the output are hi/lo planes; K and V stage both planes in LDS,
// S = K_hi Q_hi + K_lo Q_hi + K_hi Q_lo and O += V_hi P_hi + V_lo P_hi + V_hi P_lo with P split in
// registers (p_hi = bf16(p), p_lo = bf16(p - p_hi)).  LDS: 2 x (SK x 64 + SK x 96) bf16 -> SK <= 224.
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) { return make_uint2(pack2(a, b), pack2(c, d)); }

template <int NKT, bool SPLIT = false>
__global__ __launch_bounds__(512) void attention_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                        const uint16_t* __restrict__ v, uint16_t* __restrict__ out,
                                                        int S, int ldq, int ldk, int ldv, int ldo, float scale_log2) {
  constexpr int NP = SPLIT ? 2 : 1;
  constexpr int SK = NKT * 32;
  constexpr int NT = 512;
  constexpr int PER = (SK * 8 + NT - 1) / NT;  // 16-B chunks per thread per (tensor, plane)
  __shared__ __attribute__((aligned(16))) uint16_t Ks[NP][SK * AT_D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[NP][SK * VP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long rowbase = static_cast<long long>(b) * S;
  const long long rows = static_cast<long long>(gridDim.z) * S;  // plane distances: rows x pitch
  {
    uint4 kq[NP][PER], vq[NP][PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * NT, s = i >> 3, c = i & 7;
      const bool ok = i < SK * 8 && s < S;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        kq[pl][j] = ok ? *reinterpret_cast<const uint4*>(k + pl * rows * ldk + (rowbase + s) * ldk + h * AT_D + c * 8)
                       : make_uint4(0, 0, 0, 0);
        vq[pl][j] = ok ? *reinterpret_cast<const uint4*>(v + pl * rows * ldv + (rowbase + s) * ldv + h * AT_D + c * 8)
                       : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * NT, s = i >> 3, c = i & 7;
      if (i >= SK * 8) continue;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        *reinterpret_cast<uint4*>(Ks[pl] + s * AT_D + ((c ^ ((s >> 1) & 7)) << 3)) = kq[pl][j];
        *reinterpret_cast<uint4*>(Vs[pl] + s * VP + c * 8) = vq[pl][j];
      }
    }
  }
  __syncthreads();
  const int q0 = wave * 32;
  if (q0 >= S) return;  // whole wave (EXEC stays full for the transposed reads)
  const int r = lane & 31, hh = lane >> 5;
  bf16x8 qf[NP][4];
  {
    const int qr = q0 + r;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        uint4 t = make_uint4(0, 0, 0, 0);
        if (qr < S)
          t = *reinterpret_cast<const uint4*>(q + pl * rows * ldq + (rowbase + qr) * ldq + h * AT_D + ks * 16 + hh * 8);
        qf[pl][ks] = __builtin_bit_cast(bf16x8, t);
      }
  }
  f32x16 o0, o1;
#pragma unroll
  for (int i = 0; i < 16; ++i) o0[i] = o1[i] = 0.f;
  float m = -INFINITY, l = 0.f;
  // transposed-read addressing: lane 4q'+p of each 16-lane group supplies row q', columns 4p..4p+3
  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  for (int kt = 0; kt < NKT; ++kt) {
    f32x16 sc;
#pragma unroll
    for (int i = 0; i < 16; ++i) sc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int key = kt * 32 + r, chunk = 2 * ks + hh;
      const int ko = key * AT_D + ((chunk ^ ((key >> 1) & 7)) << 3);
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks[0] + ko);
      if constexpr (SPLIT) {
        const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Ks[1] + ko);
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qf[0][ks], sc, 0, 0, 0);
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[NP - 1][ks], sc, 0, 0, 0);
      }
      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[0][ks], sc, 0, 0, 0);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      const float x = key < S ? sc[i] * scale_log2 : -INFINITY;
      sc[i] = x;
      mt = fmaxf(mt, x);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    l *= alpha;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o0[i] *= alpha;
      o1[i] *= alpha;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = exp2f(sc[i] - mn);
      sc[i] = p;
      l += p;
    }
    m = mn;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pf, pfl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pf[j] = static_cast<__bf16>(sc[8 * st + j]);
        if constexpr (SPLIT) pfl[j] = static_cast<__bf16>(sc[8 * st + j] - static_cast<float>(pf[j]));
      }
      const int vo = (kt * 32 + 16 * st + 4 * hh + qq) * VP + 16 * g + 4 * pp;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const s16x4 lo = ds_read_tr16(Vs[0] + vo + dt * 32);
        const s16x4 hi = ds_read_tr16(Vs[0] + vo + 8 * VP + dt * 32);
        const bf16x8 af = __builtin_bit_cast(bf16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        f32x16& o = dt == 0 ? o0 : o1;
        if constexpr (SPLIT) {
          const s16x4 lo2 = ds_read_tr16(Vs[NP - 1] + vo + dt * 32);
          const s16x4 hi2 = ds_read_tr16(Vs[NP - 1] + vo + 8 * VP + dt * 32);
          const bf16x8 al =
              __builtin_bit_cast(bf16x8, s16x8{lo2[0], lo2[1], lo2[2], lo2[3], hi2[0], hi2[1], hi2[2], hi2[3]});
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, pf, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, pfl, o, 0, 0, 0);
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, pf, o, 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 32, 64);
  const int qr = q0 + r;
  if (qr >= S) return;
  const float inv = 1.f / l;
  uint16_t* orow = out + (rowbase + qr) * ldo + h * AT_D;
  const long long oplane = rows * ldo;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d = 8 * g4 + 4 * hh;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const f32x16& o = half ? o1 : o0;
      float w[4] = {o[4 * g4] * inv, o[4 * g4 + 1] * inv, o[4 * g4 + 2] * inv, o[4 * g4 + 3] * inv};
      uint16_t* dst = orow + 32 * half + d;
      if constexpr (SPLIT) {
        uint16_t hv[4], lv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) split1(w[t], hv[t], lv[t]);
        *reinterpret_cast<uint2*>(dst) = make_uint2(hv[0] | (uint32_t(hv[1]) << 16), hv[2] | (uint32_t(hv[3]) << 16));
        *reinterpret_cast<uint2*>(dst + oplane) =
            make_uint2(lv[0] | (uint32_t(lv[1]) << 16), lv[2] | (uint32_t(lv[3]) << 16));
      } else {
        *reinterpret_cast<uint2*>(dst) = pack4(w[0], w[1], w[2], w[3]);
      }
    }
  }
}

// Streaming variant: K/V pass through LDS in 32-key tiles, double-buffered (tile kt+1's global loads
// are in flight during tile kt's MFMAs), so a block needs 40 KiB of LDS in fp32 (split) mode instead of
// the whole pair's K/V image (143 KiB at S = 197: one block per CU).  A block = 4 waves = 128 queries
// of one (image, head) pair: ViT-B/16 at B = 32 is 768 blocks, all resident at 4 blocks per CU.
// The per-tile math (S^T = K Q^T, online exp2 softmax, O^T += V^T P^T with transposed V reads, split
// hi/lo MFMAs) is the kernel above's, with tile-local K/V rows.
// DEEP: two register sets of staged K/V -- tile kt+2's loads are issued while tile kt computes and
// tile kt+1 (loaded one step earlier) goes to LDS, so each load has two tiles of MFMAs to land
// (+16 VGPRs; still 3 waves per SIMD at head dim 64).
// HD: head dim 32, 64, 80, 96 or 128 -- HD/16 k-steps of the K Q^T product, ceil(HD/32) output
// accumulators (32 rows of D each) for O^T (at 80 the third one's rows 80..95 read the V rows' pad
// columns and are never stored); K rows of HD/8 16-B chunks (XOR-swizzled when that is a power of
// two), V rows padded to HD + 32.  Past 64 the registers allow 2 waves per SIMD (1 for split at 128).
template <int HD, bool SPLIT>
struct AttnGeom {
  static constexpr int CPR = HD / 8;                             // 16-B chunks per K/V row
  static constexpr int SW = (CPR & (CPR - 1)) == 0 ? (CPR < 8 ? CPR - 1 : 7) : 0;  // K chunk swizzle mask
  static constexpr int VPD = HD + 32;                            // V row pitch (elements)
  static constexpr int LPT = (32 * CPR + 255) / 256;             // 16-B loads per thread per plane per tile
  static constexpr int NKS = HD / 16, NDT = (HD + 31) / 32;
  static constexpr int WAVES_PER_SIMD = HD > 96 && SPLIT ? 1 : (HD > 64 ? 2 : 3);
};

template <bool SPLIT, bool DEEP, int HD>
__global__ __launch_bounds__(256, (AttnGeom<HD, SPLIT>::WAVES_PER_SIMD)) void attention_stream_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    uint16_t* __restrict__ out, int S, int ldq, int ldk, int ldv, int ldo, float scale_log2, int xcd_map) {
  using G = AttnGeom<HD, SPLIT>;
  constexpr int NP = SPLIT ? 2 : 1;
  constexpr int KT = 32;  // keys per tile
  constexpr int CPR = G::CPR, SW = G::SW, VPD = G::VPD, LPT = G::LPT, NKS = G::NKS, NDT = G::NDT;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][NP][KT * HD];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][NP][KT * VPD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware block -> (query block, head, image): blocks are dealt round-robin over the 8 XCDs
  // (linear id % 8), so with the natural mapping the query blocks of one (image, head) pair land on
  // different XCDs and each reads the pair's K/V from the Infinity Cache / HBM (ViT-B/16: 117 MB
  // per layer, 3.7 TB/s).  Here a pair's query blocks take consecutive slots of ONE XCD (pairs
  // interleaved over the XCDs), so the second reads K/V from that XCD's L2.  xcd_map 2 gives XCD x
  // the x-th contiguous eighth of the pairs instead (the images whose rows its QKV GEMM tiles wrote):
  // not measurably different inside the ViT forward (profiles/r4_attention_xcd_map.md).
  int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  {
    const int nqb = gridDim.x, pairs = gridDim.y * gridDim.z;
    if (xcd_map && (pairs & 7) == 0) {
      const int lin = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
      const int slot = lin >> 3;
      const int pair = xcd_map == 2 ? (lin & 7) * (pairs >> 3) + slot / nqb  // contiguous pair ranges
                                    : (lin & 7) + 8 * (slot / nqb);              // interleaved (default)
      qblk = slot % nqb;
      h = pair % gridDim.y;
      b = pair / gridDim.y;
    }
  }
  const long long rowbase = static_cast<long long>(b) * S;
  const long long rows = static_cast<long long>(gridDim.z) * S;  // plane distances: rows x pitch
  const int nkt = (S + KT - 1) / KT;
  // tile loader: load j of a thread = (key row, 16-B chunk) index tid + 256 j of every tensor plane
  typedef uint4 Stage[NP][LPT];
  Stage kr0, vr0, kr1, vr1;
  auto fetch = [&](int kt, Stage& kr, Stage& vr) {
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
      const int idx = tid + 256 * j, ls = idx / CPR, lc = idx % CPR;
      const int s = kt * KT + ls;
      const bool ok = idx < KT * CPR && s < S;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        kr[pl][j] = ok ? *reinterpret_cast<const uint4*>(k + pl * rows * ldk + (rowbase + s) * ldk + h * HD + lc * 8)
                       : make_uint4(0, 0, 0, 0);
        vr[pl][j] = ok ? *reinterpret_cast<const uint4*>(v + pl * rows * ldv + (rowbase + s) * ldv + h * HD + lc * 8)
                       : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto put = [&](int buf, const Stage& kr, const Stage& vr) {
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
      const int idx = tid + 256 * j, ls = idx / CPR, lc = idx % CPR;
      if (idx < KT * CPR) {
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
          *reinterpret_cast<uint4*>(Ks[buf][pl] + ls * HD + ((lc ^ ((ls >> 1) & SW)) << 3)) = kr[pl][j];
          *reinterpret_cast<uint4*>(Vs[buf][pl] + ls * VPD + lc * 8) = vr[pl][j];
        }
      }
    }
  };
  const int q0 = qblk * 128 + wave * 32;
  const bool active = q0 < S;  // wave-uniform; an idle wave still loads tiles and meets every barrier
  const int r = lane & 31, hh = lane >> 5;
  bf16x8 qf[NP][NKS];
  {
    const int qr = q0 + r;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        uint4 t = make_uint4(0, 0, 0, 0);
        if (qr < S)
          t = *reinterpret_cast<const uint4*>(q + pl * rows * ldq + (rowbase + qr) * ldq + h * HD + ks * 16 + hh * 8);
        qf[pl][ks] = __builtin_bit_cast(bf16x8, t);
      }
  }
  // K/V tile 0 after the query loads: put(0)'s wait for the tile also covers the query fragments, so
  // the loop's MFMAs never wait on vmcnt (which would drain the NEXT tile's in-flight loads each step)
  fetch(0, kr0, vr0);
  put(0, kr0, vr0);
  __syncthreads();
  if (DEEP && nkt > 1) fetch(1, kr1, vr1);
  f32x16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  // one key tile; (ka, va): the register set free for a new fetch, (kb, vb): tile kt+1 when DEEP
  auto step = [&](int kt, Stage& ka, Stage& va, Stage& kb, Stage& vb) {
    const int buf = kt & 1;
    if (DEEP) {
      if (kt + 2 < nkt) fetch(kt + 2, ka, va);  // in flight under this tile's and the next tile's MFMAs
    } else {
      if (kt + 1 < nkt) fetch(kt + 1, ka, va);  // in flight under this tile's MFMAs
    }
    if (active) {
      f32x16 sc;
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int chunk = 2 * ks + hh;
        const int ko = r * HD + ((chunk ^ ((r >> 1) & SW)) << 3);
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks[buf][0] + ko);
        if constexpr (SPLIT) {
          const bf16x8 kl = *reinterpret_cast<const bf16x8*>(Ks[buf][1] + ko);
          sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qf[0][ks], sc, 0, 0, 0);
          sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[NP - 1][ks], sc, 0, 0, 0);
        }
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[0][ks], sc, 0, 0, 0);
      }
      float mt = -INFINITY;
      if (kt * KT + KT <= S) {  // full tile (wave-uniform): no key mask
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sc[i] *= scale_log2;
          mt = fmaxf(mt, sc[i]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kt * KT + (i & 3) + 8 * (i >> 2) + 4 * hh;
          const float x = key < S ? sc[i] * scale_log2 : -INFINITY;
          sc[i] = x;
          mt = fmaxf(mt, x);
        }
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);  // m = -inf on the first tile: 0
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sc[i] - mn);  // raw v_exp_f32 (args <= 0)
        sc[i] = p;
        l += p;
      }
      m = mn;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pf, pfl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pf[j] = static_cast<__bf16>(sc[8 * st + j]);
          if constexpr (SPLIT) pfl[j] = static_cast<__bf16>(sc[8 * st + j] - static_cast<float>(pf[j]));
        }
        const int vo = (16 * st + 4 * hh + qq) * VPD + 16 * g + 4 * pp;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const s16x4 lo = ds_read_tr16(Vs[buf][0] + vo + dt * 32);
          const s16x4 hi = ds_read_tr16(Vs[buf][0] + vo + 8 * VPD + dt * 32);
          const bf16x8 af = __builtin_bit_cast(bf16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
          if constexpr (SPLIT) {
            const s16x4 lo2 = ds_read_tr16(Vs[buf][NP - 1] + vo + dt * 32);
            const s16x4 hi2 = ds_read_tr16(Vs[buf][NP - 1] + vo + 8 * VPD + dt * 32);
            const bf16x8 al =
                __builtin_bit_cast(bf16x8, s16x8{lo2[0], lo2[1], lo2[2], lo2[3], hi2[0], hi2[1], hi2[2], hi2[3]});
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, pf, o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, pfl, o[dt], 0, 0, 0);
          }
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, pf, o[dt], 0, 0, 0);
        }
      }
    }
    // the other LDS buffer's last readers passed the previous barrier
    if (kt + 1 < nkt) {
      if (DEEP) put(buf ^ 1, kb, vb);
      else put(buf ^ 1, ka, va);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, kr0, vr0, kr1, vr1);
    if (kt + 1 < nkt) step(kt + 1, kr1, vr1, kr0, vr0);
  }
  if (!active) return;
  l += __shfl_xor(l, 32, 64);
  const int qr = q0 + r;
  if (qr >= S) return;
  const float inv = 1.f / l;
  uint16_t* orow = out + (rowbase + qr) * ldo + h * HD;
  const long long oplane = rows * ldo;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d = 8 * g4 + 4 * hh;
#pragma unroll
    for (int half = 0; half < NDT; ++half) {
      if (32 * half + d >= HD) continue;  // head dim 80: the last accumulator's upper rows
      const f32x16& oh = o[half];
      float w[4] = {oh[4 * g4] * inv, oh[4 * g4 + 1] * inv, oh[4 * g4 + 2] * inv, oh[4 * g4 + 3] * inv};
      uint16_t* dst = orow + 32 * half + d;
      if constexpr (SPLIT) {
        uint16_t hv[4], lv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) split1(w[t], hv[t], lv[t]);
        *reinterpret_cast<uint2*>(dst) = make_uint2(hv[0] | (uint32_t(hv[1]) << 16), hv[2] | (uint32_t(hv[3]) << 16));
        *reinterpret_cast<uint2*>(dst + oplane) =
            make_uint2(lv[0] | (uint32_t(lv[1]) << 16), lv[2] | (uint32_t(lv[3]) << 16));
      } else {
        *reinterpret_cast<uint2*>(dst) = pack4(w[0], w[1], w[2], w[3]);
      }
    }
  }
}

// Softmax over rows (one wave per row, fp32 max / sum with exp2): classifier heads and any softmax
// outside the fused attention.
__global__ __launch_bounds__(256) void softmax_rows_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                           float* __restrict__ yf, long long rows, int C, int ld,
                                                           int split) {
  const int lane = threadIdx.x & 63;
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long plane = rows * ld;
  const uint16_t* xr = x + row * ld;
  const bool sp = split != 0;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, load1v(xr + c, plane, sp));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  constexpr float kLog2e = 1.4426950408889634f;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += exp2f((load1v(xr + c, plane, sp) - m) * kLog2e);
  const float inv = 1.f / wave_sum(s);
  for (int c = lane; c < C; c += 64) {
    const float p = exp2f((load1v(xr + c, plane, sp) - m) * kLog2e) * inv;
    if (y) store1v(y + row * ld + c, plane, sp, p);
    if (yf) yf[row * C + c] = p;
  }
  if (y)  // pad columns of a padded row stay finite (consumers give them zero weight)
    for (int c = C + lane; c < ld; c += 64) store1v(y + row * ld + c, plane, sp, 0.f);
}

inline int grid_for(long long work, int cap = 4096) {
  long long g = (work + 255) / 256;
  if (g < 1) g = 1;
  return static_cast<int>(g > cap ? cap : g);
}

}  // namespace

namespace {
int g_ln_xcd = 0;  // 1: LayerNorm rows read on the XCD that wrote them (xcd_block); 0 (default): natural order
}
void set_layernorm_xcd(int v) { g_ln_xcd = v; }

hipError_t layernorm_rows(const uint16_t* x, uint16_t* y, const float* gamma, const float* beta, float eps,
                          long long rows, int C, hipStream_t s, int split, int Cl, int variant, float* stats) {
  if (!stats && !y) return hipErrorInvalidValue;
  if (C % 8 || Cl < 0 || Cl > C || variant < 0 || variant > 2) return hipErrorInvalidValue;
  if (Cl == 0) Cl = C;
  const int blocks = static_cast<int>((rows + 3) / 4);
  if (variant == 1) {
    if (C > 16 * 8 * 6) return hipErrorInvalidValue;
    hipLaunchKernelGGL((layernorm_kernel<6, 16>), dim3(static_cast<int>((rows + 15) / 16)), dim3(256), 0, s, x, y, gamma,
                       beta, eps, rows, C, split, Cl, stats, g_ln_xcd);
    return hipGetLastError();
  }
  if (variant == 2) {
    hipLaunchKernelGGL(layernorm_wide_kernel, dim3(static_cast<unsigned>(rows)), dim3(256), 0, s, x, y, gamma, beta, eps,
                       rows, C, split, Cl, stats, g_ln_xcd);
    return hipGetLastError();
  }
  if (C > 512 && C <= 32 * 8 * 3) {  // 513..768 (ViT-B: 768): 32 lanes x 3 chunks, 2 rows per wave
    hipLaunchKernelGGL((layernorm_kernel<3, 32>), dim3(static_cast<int>((rows + 7) / 8)), dim3(256), 0, s, x, y, gamma,
                       beta, eps, rows, C, split, Cl, stats, g_ln_xcd);
    return hipGetLastError();
  }
  if (C <= 64 * 8)
    hipLaunchKernelGGL(layernorm_kernel<1>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C, split, Cl, stats, g_ln_xcd);
  else if (C <= 128 * 8)
    hipLaunchKernelGGL(layernorm_kernel<2>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C, split, Cl, stats, g_ln_xcd);
  else if (C <= 256 * 8)
    hipLaunchKernelGGL(layernorm_kernel<4>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C, split, Cl, stats, g_ln_xcd);
  else
    hipLaunchKernelGGL(layernorm_wide_kernel, dim3(static_cast<unsigned>(rows)), dim3(256), 0, s, x, y, gamma, beta, eps,
                       rows, C, split, Cl, stats, g_ln_xcd);
  return hipGetLastError();
}

hipError_t tokens_assemble(const uint16_t* patches, const float* cls, const float* pos, uint16_t* out, int B, int S0,
                           int C, hipStream_t s, int split, float* stats) {
  if (C % 8 || (stats && C % 64)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tokens_kernel, dim3(grid_for(static_cast<long long>(B) * (S0 + 1) * (C / 8))), dim3(256), 0, s,
                     patches, cls, pos, out, B, S0, C, split, stats);
  return hipGetLastError();
}

hipError_t gather_rows(const uint16_t* x, uint16_t* y, int B, int S, int idx, int C, hipStream_t s, int split) {
  if (C % 8 || idx < 0 || idx >= S) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(static_cast<long long>(B) * (C / 8))), dim3(256), 0, s, x, y, B,
                     S, idx, C, split);
  return hipGetLastError();
}

hipError_t softmax_rows(const uint16_t* x, uint16_t* y, float* y_f32, long long rows, int C, hipStream_t s,
                        int split, int ld) {
  if (ld <= 0) ld = C;
  if (C <= 0 || rows <= 0 || ld < C || (!y && !y_f32)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(static_cast<unsigned>((rows + 3) / 4)), dim3(256), 0, s, x, y, y_f32,
                     rows, C, ld, split);
  return hipGetLastError();
}

bool attention_any_length() { return kAttnStream; }

bool attention_supported(int D, int S) {
  if (S <= 0) return false;
  if (kAttnStream) return D == 32 || D == 64 || D == 80 || D == 96 || D == 128;
  return D == AT_D && S <= 256;
}

namespace {
int g_attn_variant = 0;  // 0: K/V staged one tile ahead, 1: two tiles ahead (DEEP), 2: 0 without the XCD map
}
void set_attention_variant(int v) { g_attn_variant = v; }

hipError_t attention(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* out, int B, int S, int H,
                     int D, int ldq, int ldk, int ldv, int ldo, float scale, hipStream_t s, int split) {
  if (!attention_supported(D, S) || ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;  // softmax in exp2
  if (kAttnStream) {  // 4-wave blocks of 128 queries, K/V streamed in 32-key tiles (any S)
    dim3 grid((S + 127) / 128, H, B);
    const bool deep = g_attn_variant == 1;
    // variant 2: the natural block mapping, 3: contiguous pair ranges per XCD (measurement)
    const int xcd_map = g_attn_variant == 2 ? 0 : g_attn_variant == 3 ? 2 : 1;
#define ATTN_LAUNCH(SP, DP, HDV)                                                                                   \
  hipLaunchKernelGGL((attention_stream_kernel<SP, DP, HDV>), grid, dim3(256), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, \
                     sl2, xcd_map)
#define ATTN_HD(HDV)                          \
  if (split && deep) ATTN_LAUNCH(true, true, HDV);    \
  else if (split) ATTN_LAUNCH(true, false, HDV);      \
  else if (deep) ATTN_LAUNCH(false, true, HDV);       \
  else ATTN_LAUNCH(false, false, HDV);
    switch (D) {
      case 32: ATTN_HD(32) break;
      case 64: ATTN_HD(64) break;
      case 80: ATTN_HD(80) break;
      case 96: ATTN_HD(96) break;
      default: ATTN_HD(128) break;
    }
#undef ATTN_HD
#undef ATTN_LAUNCH
    return hipGetLastError();
  }
  dim3 grid(1, H, B);  // one 8-wave block per (image, head): wave w = query tile w (S <= 256)
  if (split) {
    if (S <= 64) hipLaunchKernelGGL((attention_kernel<2, true>), grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
    else if (S <= 128) hipLaunchKernelGGL((attention_kernel<4, true>), grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
    else if (S <= 224) hipLaunchKernelGGL((attention_kernel<7, true>), grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (S <= 64) hipLaunchKernelGGL(attention_kernel<2>, grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
  else if (S <= 128) hipLaunchKernelGGL(attention_kernel<4>, grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
  else if (S <= 224) hipLaunchKernelGGL(attention_kernel<7>, grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
  else hipLaunchKernelGGL(attention_kernel<8>, grid, dim3(512), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, sl2);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
