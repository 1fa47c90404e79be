// Implicit-GEMM conv kernels and their launcher template (included by the per-tile translation
// units conv_tile_*.hip, which instantiate one tile shape each so the build runs them in parallel).
// Design notes: conv_igemm.hip.
#pragma once

#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {
namespace igemm {
namespace {  // internal linkage: each conv_tile_*.hip gets its own copy of what it instantiates

using namespace die::k;


constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

// Epilogue activation: 1 = ReLU, 2 = exact (erf) GELU, 3 = Clip(lo, hi).
__device__ __forceinline__ float act_fn(float v, int act, float lo = 0.f, float hi = 0.f) {
  if (act == 3) return fminf(fmaxf(v, lo), hi);
  return act == 1 ? fmaxf(v, 0.f) : gelu_erf(v);
}

__device__ __forceinline__ float4 ldf4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Write-through (sc1) 16-byte stores / loads of the split-K workspace through a buffer resource
// (aux bit 4 = sc1 on gfx950): the fused split-K producers need no agent-scope release (partials
// written through to memory, drained by every storing wave); the consumer keeps one agent acquire
// (tile_epilogue).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
constexpr int kCpolSc1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, byte_off, 0, kCpolSc1);
}
__device__ __forceinline__ float4 ld4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kCpolSc1));
}

// Chan et al. merge of two (count, mean, M2) summaries in a form symmetric in its operands, so the
// two lanes of a DPP exchange compute bit-identical results (empty summaries: count 0).
__device__ __forceinline__ void chan_sym(float& mean, float& m2, float& cnt, float mean_o, float m2_o, float cnt_o) {
  const float tot = cnt + cnt_o, d = mean_o - mean;
  const float inv = tot > 0.f ? 1.f / tot : 0.f;
  m2 = (m2 + m2_o) + d * d * (cnt * cnt_o * inv);
  mean = (cnt * mean + cnt_o * mean_o) * inv;
  cnt = tot;
}
// Left-to-right merge of 64-column (mean, M2) groups into a running (mean, M2, count).
__device__ __forceinline__ void chan_add64(float& mean, float& m2, float& cnt, float2 g) {
  const float d = g.x - mean, tot = cnt + 64.f;
  mean += d * (64.f / tot);
  m2 += g.y + d * d * (cnt * 64.f / tot);
  cnt = tot;
}

// ConvArgs::row_parts reader: the LayerNorm statistics of the block's BM rows.  TPR = NT / BM
// adjacent threads per row, each holding a contiguous run of the row's K/64 groups.  issue() at the
// block's start puts the loads in flight with the first operand loads; merge() (every thread of the
// block) after the prologue returns (mean, rstd) of the thread's row on all its TPR lanes: each run
// merged left to right, then the runs by a fixed DPP tree -- bitwise repeatable.
template <int BM, int NT = 256>
struct RowParts {
  static constexpr int TPR = NT / BM, MAXG = 8;  // groups held per thread (more: loaded in merge)
  static_assert(TPR == 2 || TPR == 4, "one quad per row");
  float2 q[MAXG];
  const float2* src = nullptr;
  int g0 = 0, g1 = 0;
  __device__ __forceinline__ void issue(const ConvArgs& p, int m0, int tid) {
    const int ng = p.K >> 6, row = tid / TPR, sub = tid % TPR;
    const int m = m0 + row < p.M ? m0 + row : 0;  // tail rows: any valid row, result unused
    g0 = sub * ng / TPR;
    g1 = (sub + 1) * ng / TPR;
    src = reinterpret_cast<const float2*>(p.row_parts) + static_cast<size_t>(m) * ng;
#pragma unroll
    for (int j = 0; j < MAXG; ++j) q[j] = g0 + j < g1 ? src[g0 + j] : make_float2(0.f, 0.f);
  }
  __device__ __forceinline__ float2 merge(const ConvArgs& p) const {
    float mean = q[0].x, m2 = q[0].y, cnt = g1 > g0 ? 64.f : 0.f;  // K < 64 * TPR: some runs empty
#pragma unroll
    for (int j = 1; j < MAXG; ++j)
      if (g0 + j < g1) chan_add64(mean, m2, cnt, q[j]);
    for (int j = g0 + MAXG; j < g1; ++j) chan_add64(mean, m2, cnt, src[j]);
    chan_sym(mean, m2, cnt, dpp<0xB1>(mean), dpp<0xB1>(m2), dpp<0xB1>(cnt));
    if constexpr (TPR == 4) chan_sym(mean, m2, cnt, dpp<0x4E>(mean), dpp<0x4E>(m2), dpp<0x4E>(cnt));
    return make_float2(mean, rsqrtf(m2 / cnt + p.ln_eps));
  }
};
// The same for one row by one thread (the two-kernel split-K epilogue; no prefetch).
__device__ __forceinline__ float2 row_parts_direct(const ConvArgs& p, int m) {
  const int ng = p.K >> 6;
  const float2* src = reinterpret_cast<const float2*>(p.row_parts) + static_cast<size_t>(m) * ng;
  float mean = 0.f, m2 = 0.f, cnt = 0.f;
  for (int j = 0; j < ng; ++j) chan_add64(mean, m2, cnt, src[j]);
  return make_float2(mean, rsqrtf(m2 / cnt + p.ln_eps));
}

// Epilogue for 8 consecutive channels [n, n+8) of output pixel m.  Requires N % 8 == 0.
// fp32 mode (p.split): the residual is read as hi + lo and out/out2 are stored as split planes.
// ms: (mean, rstd) of row m for a p.row_parts reader (tile_epilogue's LDS row cache; null: merged
// here, the two-kernel split-K path).
// p.stats_out: the 8 lanes holding one 64-column group (consecutive lanes, group-aligned n -- every
// caller maps consecutive threads to consecutive 8-channel chunks of one row, and N % 64 == 0)
// merge their (mean, M2) by DPP; the formula is symmetric, so all 8 lanes agree and the result does
// not depend on which lane stores it.
// rpre: the residual's 8 values already loaded (tile_epilogue prefetches a thread's residual rows
// before its first store, so the loads are not serialised behind the previous group's stores).
// This thread's 8 output channels' epilogue parameters (bias, dual-store BN, LayerNorm column sums),
// loaded once before the tile's first store: loaded per group inside epilogue8 they came after the
// previous group's stores, and vmcnt counts loads and stores in issue order, so each group's wait
// for them also drained the previous group's stores (one store round trip per group).
struct EpiChan {
  float b[8], s2[8], h2[8], cs[8];
};
__device__ __forceinline__ void load_epi_chan(const ConvArgs& p, int n, EpiChan& c) {
  auto ld8 = [&](const float* src, float* d) {
    const float4 a = ldf4(src + n), b = ldf4(src + n + 4);
    d[0] = a.x, d[1] = a.y, d[2] = a.z, d[3] = a.w, d[4] = b.x, d[5] = b.y, d[6] = b.z, d[7] = b.w;
  };
  if (p.bias) ld8(p.bias, c.b);
  if (p.out2) {
    ld8(p.scale2, c.s2);
    ld8(p.shift2, c.h2);
  }
  if (p.row_stats || p.row_parts) ld8(p.col_sum, c.cs);
}

__device__ __forceinline__ void epilogue8(const ConvArgs& p, int m, int n, float* v, const float* ms = nullptr,
                                          const float* rpre = nullptr, const EpiChan* ec = nullptr) {
  const size_t o = static_cast<size_t>(m) * p.N + n;
  const bool split = p.split != 0;
  if (p.row_stats || p.row_parts) {
    float mean, rstd;
    if (p.row_stats) {
      mean = p.row_stats[2 * static_cast<size_t>(m)];
      rstd = p.row_stats[2 * static_cast<size_t>(m) + 1];
    } else if (ms) {
      mean = ms[0];
      rstd = ms[1];
    } else {
      const float2 r = row_parts_direct(p, m);
      mean = r.x;
      rstd = r.y;
    }
    float cs[8];
    if (ec) {
#pragma unroll
      for (int t = 0; t < 8; ++t) cs[t] = ec->cs[t];
    } else {
      const float4 c0 = ldf4(p.col_sum + n), c1 = ldf4(p.col_sum + n + 4);
      cs[0] = c0.x, cs[1] = c0.y, cs[2] = c0.z, cs[3] = c0.w, cs[4] = c1.x, cs[5] = c1.y, cs[6] = c1.z, cs[7] = c1.w;
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = rstd * (v[t] - mean * cs[t]);
  }
  if (p.bias) {
    if (ec) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += ec->b[t];
    } else {
      const float4 b0 = ldf4(p.bias + n), b1 = ldf4(p.bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
  }
  if (p.res) {
    float r[8];
    if (rpre) {
#pragma unroll
      for (int t = 0; t < 8; ++t) r[t] = rpre[t];
    } else {
      load8v(p.res + o, p.oplane, split, r);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] += r[t];
  }
  if (p.relu) {
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = act_fn(v[t], p.relu, p.clip_lo, p.clip_hi);
  }
  if (p.stats_out) {
    const float2 st = group64_stats(v);
    if ((n & 63) == 0) reinterpret_cast<float2*>(p.stats_out)[static_cast<size_t>(m) * (p.N >> 6) + (n >> 6)] = st;
  }
  if (p.out) store8v(p.out + o, p.oplane, split, v);
  if (p.out_f32) {
    *reinterpret_cast<float4*>(p.out_f32 + o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p.out_f32 + o + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
  if (p.out2) {
    float u[8];
    if (ec) {
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = v[t] * ec->s2[t] + ec->h2[t];
    } else {
      const float4 s0 = ldf4(p.scale2 + n), s1 = ldf4(p.scale2 + n + 4);
      const float4 h0 = ldf4(p.shift2 + n), h1 = ldf4(p.shift2 + n + 4);
      u[0] = v[0] * s0.x + h0.x, u[1] = v[1] * s0.y + h0.y, u[2] = v[2] * s0.z + h0.z, u[3] = v[3] * s0.w + h0.w;
      u[4] = v[4] * s1.x + h1.x, u[5] = v[5] * s1.y + h1.y, u[6] = v[6] * s1.z + h1.z, u[7] = v[7] * s1.w + h1.w;
    }
    if (p.relu2) {
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = fmaxf(u[t], 0.f);
    }
    store8v(p.out2 + o, p.oplane, split, u);
  }
}

// Row r of a tile -> output pixel m0 + r (GEMM rows are consecutive pixels); -1 = no pixel.
struct LinearRows {
  int m0, M;
  __device__ __forceinline__ int operator()(int r) const { return m0 + r < M ? m0 + r : -1; }
};

// Stream-K partials (ConvArgs::sk = P persistent blocks): block b owns iterations [start(b),
// start(b+1)) of the T x nk (tile, K-step) space, start(b) = floor(b * I / P), I = T * nk.  A tile
// cut between blocks first..last gets one partial from each; block b keeps at most two partial
// slabs (its first and its last segment), slab 2b + which of BM x BN floats in ConvArgs::ws, and
// the tile's last arriver sums them in block order (deterministic for a given P).
struct StreamK {
  long long I = 0;  // total iterations (0: not a stream-K launch)
  int P = 0;
  int nk = 0;       // K-steps per tile
  __device__ __forceinline__ long long start(int b) const { return static_cast<long long>(b) * I / P; }
  __device__ __forceinline__ int owner(long long x) const { return static_cast<int>(((x + 1) * P - 1) / I); }
  // slab of block b's partial of tile t (its first segment unless t began before b's range)
  __device__ __forceinline__ int slab(int b, int t) const {
    return 2 * b + (start(b) >= static_cast<long long>(t) * nk ? 0 : 1);
  }
};

// NT threads = (NT / 64) waves, WAVES_M along the tile's rows (pixels) x NT / 64 / WAVES_M along its
// channels; acc[i][j]: the wave's i-th 16-channel x j-th 16-pixel fragment.
// Split-K: `split` is this block's slice (partial slab) and `nsplit` the tile's slice count (-1:
// p.splits); with a stream-K map (sk.I > 0) `split` is this block's id and the tile's partials are
// those of blocks first..first + nsplit - 1.
template <int BM, int BN, typename RowMap = LinearRows, int NT = 256, int WAVES_M = 2>
__device__ __forceinline__ void tile_epilogue(const ConvArgs& p,
                                              f32x4 (&acc)[BN / 16 / (NT / 64 / WAVES_M)][BM / 16 / WAVES_M],
                                              uint16_t* lds, int m0, int n0, int wm, int wn, int lane, int tid,
                                              int tile, int split, RowMap rows = RowMap{0, 0},
                                              float2 rms = float2{0.f, 0.f}, int flag_off = -1, int nsplit = -1,
                                              StreamK sk = StreamK{}, int sk_first = 0);

// LDS element offset of the fused split-K "last arriver" word past the epilogue staging (epi
// elements), or -1 when the block's LDS has no room there (the word then overwrites the staging
// tile and the last arriver re-reads its own partial from the workspace).
constexpr int epi_flag_off(int lds_elems, int epi_elems) { return lds_elems >= epi_elems + 2 ? epi_elems : -1; }

// XCD-aware block -> (tile, split-K slice).  Blocks are dealt round-robin over the 8 XCDs (linear
// id % 8 labels the blocks that share one XCD and its L2; cdna_hip_programming T1), so the naive
// tile = blockIdx.x spreads the N-tiles of one M-tile (same activation rows) or the M-tiles of
// one N-tile (same weight rows) over 8 L2s.  The bijective remap gives every XCD a contiguous range
// of logical ids; a tile's split-K slices are adjacent (same XCD for the fused reducer), and tiles
// are ordered so the operand with more bytes is the one shared within an XCD: N-fastest (an
// M-tile's activations read once per XCD, every XCD reads all weights) when the weights are the
// smaller operand, M-fastest otherwise (stage-4 3x3 / expand / FC shapes).
// With a live batch (ConvArgs::live) only the tiles holding real samples get work: the first
// live_tiles * S blocks (spread evenly over the XCDs) are remapped over them and the rest exit.
// Tail split-K (ConvArgs::tail): the first Tw = T - T % tail tiles are whole (split = -1: the full
// K range, direct epilogue) and the T - Tw tiles of the last partial round get S slices each.
// Returns false for a block without work.
__device__ __forceinline__ void tile_mn(const ConvArgs& p, int ntm, int ntn, int tile, int& tile_m, int& tile_n);
__device__ __forceinline__ bool block_coords(const ConvArgs& p, int BM, int BN, int& tile_m, int& tile_n, int& split,
                                             int& tile) {
  const int S = p.tail > 0 ? p.splits : static_cast<int>(gridDim.y);  // split-K slices
  const int ntn = (p.N + BN - 1) / BN;
  const int Ml = p.live ? min(p.M, static_cast<int>(*p.live) * p.Ho * p.Wo) : p.M;
  const int ntm = (Ml + BM - 1) / BM;
  const int T = ntm * ntn;
  const int Tw = p.tail > 0 ? (T > p.tail ? T - T % p.tail : T) : 0;  // whole tiles (tail split-K)
  const int nwg = min(static_cast<int>(gridDim.x * gridDim.y), Tw + (T - Tw) * S);
  const int b = blockIdx.x + blockIdx.y * gridDim.x;
  if (b >= nwg) return false;
  const int q = nwg >> 3, r = nwg & 7, x = b & 7;
  const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  const int sid = id - Tw, st = sid / S;
  tile = id < Tw ? id : Tw + st;
  split = id < Tw ? -1 : sid - st * S;
  tile_mn(p, ntm, ntn, tile, tile_m, tile_n);
  return true;
}

// Logical tile index -> (tile_m, tile_n) (block_coords' tile order; also the stream-K walk's).
__device__ __forceinline__ void tile_mn(const ConvArgs& p, int ntm, int ntn, int tile, int& tile_m, int& tile_n) {
  // Replicate (read on every XCD) the operand with fewer bytes: the weights are N x K, the
  // activations the INPUT tensor, B*H*W*Cin -- not the im2col M x K, which counts a 3x3 conv's
  // input 9 times (stage-4 3x3 at batch 16-32: weights 4.7x the input, so M-fastest).
  const long long wts = static_cast<long long>(p.N) * p.K;
  const long long acts = static_cast<long long>(p.B) * p.H * p.W * p.Cin;
  // One division and selects, no branch: with the outputs assigned on two paths the compiler kept
  // them in scratch (a private-memory round trip at the start of every block).
  const bool nfast = p.order == 1 || (p.order == 0 && wts <= acts) || p.order >= 3;
  // order 3 / 4: N split into 2 / 4 panels, tiles panel-major (N-fastest inside a panel), so the
  // contiguous id range an XCD gets needs only its panel's weight rows (a panel of a large GEMM's
  // weights fits the XCD's 4 MiB L2 where all of them do not).  Full panels first; the last panel
  // may be narrower.
  const int P = p.order == 3 ? 2 : p.order == 4 ? 4 : 1;
  const int pw = (ntn + P - 1) / P;               // panel width (N-tiles)
  const int full = ntn / pw;                      // panels of full width
  const int pk = min(tile / (pw * ntm), full);    // panel index (the last one may be partial)
  const int rem = tile - pk * pw * ntm;
  const int w = min(pw, ntn - pk * pw);           // this panel's width
  const int minor = P > 1 ? w : nfast ? ntn : ntm;
  const int hi = rem / minor, lo = rem - hi * minor;
  tile_m = nfast ? hi : lo;
  tile_n = nfast ? lo + pk * pw : hi;
}

// Register-staged main loop (any shape).  SPLIT (fp32 mode): both operands come as hi/lo planes, a
// stage holds four tiles [A_hi][B_hi][A_lo][B_lo] and every fragment pair takes three MFMAs.
template <int BM, int BN, int MODE, int VEC, bool SPLIT = false>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const ConvArgs p, const int kt_per_split) {
  constexpr int NP = SPLIT ? 2 : 1;                   // operand planes
  constexpr int WM = BM / 2, WN = BN / 2;  // per-wave pixels / channels
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_ELEMS = BN * BK, B_ELEMS = BM * BK, STAGE = A_ELEMS + B_ELEMS;
  constexpr int W_CH = BN / 32;                       // 16-B weight chunks per thread per stage
  constexpr int X_CH = VEC == 8 ? BM / 32 : BM / 16;  // activation units per thread per stage
  static_assert(2 * STAGE * NP * 2 >= BM * BN * 4, "epilogue staging must fit in the operand LDS");
  static_assert(!SPLIT || 2 * STAGE * NP >= BM * BN * 2 + BM * 4, "... and the row_parts row cache (fp32)");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STAGE * NP];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  int tile_m, tile_n, split, tile;
  if (!block_coords(p, BM, BN, tile_m, tile_n, split, tile)) return;  // whole block, before any barrier
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk_total = p.Kpad / BK;
  const int kt_begin = split * kt_per_split;
  const int kt_end = min(nk_total, kt_begin + kt_per_split);

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

  uint4 wreg[NP][W_CH];
  uint4 xreg8[NP][VEC == 8 ? X_CH : 1];
  uint2 xreg4[NP][VEC == 4 ? X_CH : 1];

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
#pragma unroll
      for (int i = 0; i < W_CH; ++i)
        wreg[pl][i] = *reinterpret_cast<const uint4*>(wsrc + pl * p.wplane + static_cast<size_t>(32 * i) * p.Kpad + k0);
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
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const uint16_t* src = p.x + addr + pl * p.xplane;
        if (VEC == 8) {
          xreg8[pl][i] = v ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
        } else {
          xreg4[pl][i] = v ? *reinterpret_cast<const uint2*>(src) : make_uint2(0, 0);
        }
      }
    }
  };

  auto store_stage = [&](int buf) {
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      uint16_t* A = lds + (buf * NP + pl) * STAGE;
      uint16_t* Bt = A + A_ELEMS;
#pragma unroll
      for (int i = 0; i < W_CH; ++i) *reinterpret_cast<uint4*>(A + swz(wr + 32 * i, wc)) = wreg[pl][i];
#pragma unroll
      for (int i = 0; i < X_CH; ++i) {
        const int row = xr + XR_STEP * i;
        if (VEC == 8) {
          *reinterpret_cast<uint4*>(Bt + swz(row, xc)) = xreg8[pl][i];
        } else {
          *reinterpret_cast<uint2*>(Bt + swz(row, xc >> 1) + 4 * (xc & 1)) = xreg4[pl][i];
        }
      }
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  RowParts<BM> rp;  // row_parts reader (fp32 only): loads in flight with the first stage's
  float2 rms = make_float2(0.f, 0.f);
  if (SPLIT && p.row_parts) rp.issue(p, m0, tid);
  if (kt_begin < kt_end) load_stage(kt_begin * BK);
  if (SPLIT && p.row_parts) rms = rp.merge(p);
  if (kt_begin < kt_end) {
    store_stage(0);
    __syncthreads();
  }
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = (kt - kt_begin) & 1;
    const bool more = kt + 1 < kt_end;
    if (more) load_stage((kt + 1) * BK);  // in flight under the MFMAs below
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[NP][TN], bfr[NP][TM];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const uint16_t* A = lds + (cur * NP + pl) * STAGE;
        const uint16_t* Bt = A + A_ELEMS;
#pragma unroll
        for (int i = 0; i < TN; ++i)
          af[pl][i] = *reinterpret_cast<const bf16x8*>(A + swz(wn * WN + i * 16 + (lane & 15), chunk));
#pragma unroll
        for (int j = 0; j < TM; ++j)
          bfr[pl][j] = *reinterpret_cast<const bf16x8*>(Bt + swz(wm * WM + j * 16 + (lane & 15), chunk));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          if constexpr (SPLIT) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[1][j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
        }
    }
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }
  tile_epilogue<BM, BN>(p, acc, lds, m0, n0, wm, wn, lane, tid, tile, split, LinearRows{0, 0}, rms,
                        epi_flag_off(2 * STAGE * NP, BM * BN * 2 + (SPLIT ? BM * 4 : 0)));
}

// Shared epilogue of both GEMM main loops.  `lds` must hold >= BM*BN floats and be free (all waves
// past their last operand read).
template <int BM, int BN, typename RowMap, int NT, int WAVES_M>
__device__ __forceinline__ void tile_epilogue(const ConvArgs& p,
                                              f32x4 (&acc)[BN / 16 / (NT / 64 / WAVES_M)][BM / 16 / WAVES_M],
                                              uint16_t* lds, int m0, int n0, int wm, int wn, int lane, int tid,
                                              int tile, int split, RowMap rows, float2 rms, int flag_off, int nsplit,
                                              StreamK sk, int sk_first) {
  if constexpr (std::is_same_v<RowMap, LinearRows>) rows = LinearRows{m0, p.M};
  constexpr int WM = BM / WAVES_M, WN = BN / (NT / 64 / WAVES_M);
  constexpr int TM = WM / 16, TN = WN / 16;
  const int lm = lane & 15;
  const int ln = (lane >> 4) * 4;
  if ((p.N & 7) == 0) {
    // ---- LDS-staged, coalesced epilogue ----
    constexpr int CPR = BN / 4;  // 16-B chunks per staged row
    float* st = reinterpret_cast<float*>(lds);
    // row_parts reader: the tile rows' (mean, rstd) (merged by the kernel, RowParts) into the LDS row
    // cache past the staging tile, published by the staging barrier below
    float* rowc = nullptr;
    if (p.row_parts) {
      rowc = st + BM * BN;
      if (tid % (NT / BM) == 0) *reinterpret_cast<float2*>(rowc + 2 * (tid / (NT / BM))) = rms;
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = wm * WM + j * 16 + lm;
        const int c = (wn * WN + i * 16 + ln) >> 2;
        *reinterpret_cast<f32x4*>(st + row * BN + ((c ^ (row & (CPR - 1))) << 2)) = acc[i][j];
      }
    __syncthreads();
    constexpr int GPR = BN / 8;
    // 8-channel groups per thread: group i of this thread is g = tid + i * NT (row g / GPR)
    constexpr int NG = BM * GPR / NT;
    static_assert(NG * NT == BM * GPR, "whole groups per thread");
    int gm[NG], gn[NG], grow[NG], gcg[NG];
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int g = tid + i * NT;
      grow[i] = g / GPR;
      gcg[i] = g - grow[i] * GPR;
      gm[i] = rows(grow[i]);
      gn[i] = n0 + gcg[i] * 8;
      if (gn[i] >= p.N) gm[i] = -1;
    }
    // every group of a thread has the same 8 channels (NT is a multiple of GPR): their parameters
    // are loaded once, here, before any store of the tile (EpiChan)
    static_assert(NT % GPR == 0, "a thread's groups share their channels");
    EpiChan ec;
    load_epi_chan(p, min(n0 + (tid % GPR) * 8, p.N - 8), ec);
    auto grow_i = [&](int i) { return grow[i]; };
    auto gcg_i = [&](int i) { return gcg[i]; };
    auto gm_i = [&](int i) { return gm[i] < 0 ? 0 : gm[i]; };
    auto gn_i = [&](int i) { return gm[i] < 0 ? 0 : gn[i]; };
    if (nsplit < 0) nsplit = p.splits;
    const bool streamk = sk.I > 0;
    const bool partial = nsplit > 1 && split >= 0;  // (split < 0: a tail split-K launch's whole tile)
    const bool fused = partial && p.counters;
    float* ws = partial && !streamk ? p.ws + static_cast<size_t>(split) * p.M * p.N : nullptr;
    // byte offset of group i in partial slab `slab` (stream-K: tile-local [BM][BN] slabs)
    auto part_off = [&](int slab, int i) -> unsigned {
      return streamk ? static_cast<unsigned>((static_cast<size_t>(slab) * BM * BN + grow_i(i) * BN + gcg_i(i) * 8) * 4)
                     : static_cast<unsigned>(((static_cast<size_t>(slab) * p.M + gm_i(i)) * p.N + gn_i(i)) * 4);
    };
    const __amdgpu_buffer_rsrc_t wsr = ws_rsrc(p.ws);
    auto stage8 = [&](int i, float4& a, float4& b) {
      a = *reinterpret_cast<const float4*>(st + grow[i] * BN + (((2 * gcg[i]) ^ (grow[i] & (CPR - 1))) << 2));
      b = *reinterpret_cast<const float4*>(st + grow[i] * BN + (((2 * gcg[i] + 1) ^ (grow[i] & (CPR - 1))) << 2));
    };
    // Groups go in chunks of CH: the chunk's residual loads (and, last arriver, each split's partial
    // loads) are all in flight before the first of them is used, so a chunk costs one round trip
    // instead of one per group -- with few enough registers held that the main loop's occupancy is
    // unchanged.
    constexpr int CH = NG < 2 ? NG : 2;
    uint4 rr[CH][2];
    auto load_res = [&](int c0) {
      if (!p.res) return;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int i = c0 + j;
        const size_t o = static_cast<size_t>(gm_i(i)) * p.N + gn_i(i);
        rr[j][0] = *reinterpret_cast<const uint4*>(p.res + o);
        rr[j][1] = p.split ? *reinterpret_cast<const uint4*>(p.res + p.oplane + o) : make_uint4(0, 0, 0, 0);
      }
    };
    auto finish = [&](int c0, int j, float* v) {
      const int i = c0 + j;
      float r[8];
      if (p.res) {
        unpack8(rr[j][0], r);
        if (p.split) {
          float l[8];
          unpack8(rr[j][1], l);
#pragma unroll
          for (int t = 0; t < 8; ++t) r[t] += l[t];
        }
      }
      epilogue8(p, gm[i], gn[i], v, rowc ? rowc + 2 * grow[i] : nullptr, p.res ? r : nullptr, &ec);
    };
    if (!partial) {
#pragma unroll
      for (int c0 = 0; c0 < NG; c0 += CH) {
        load_res(c0);
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          if (gm[c0 + j] < 0) continue;
          float4 a, b;
          stage8(c0 + j, a, b);
          float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          finish(c0, j, v);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      if (gm[i] < 0) continue;
      float4 a, b;
      stage8(i, a, b);
      if (fused) {
        const unsigned off = part_off(streamk ? sk.slab(split, tile) : split, i);
        st4_sc1(wsr, off, a);
        st4_sc1(wsr, off + 16, b);
      } else {
        float* o = ws + static_cast<size_t>(gm[i]) * p.N + gn[i];
        *reinterpret_cast<float4*>(o) = a;
        *reinterpret_cast<float4*>(o + 4) = b;
      }
    }
    if (!fused) return;
    // Fused split-K reduction: the last split block of this tile to arrive sums every split's
    // partial (in split order, as splitk_epilogue_kernel does) and runs the epilogue, no second
    // kernel.  Hand-off (MI355X_MICROARCH "Valid forms"): producer side, the partials went out as
    // write-through (sc1) stores, every storing wave drains them (vmcnt(0)) and a block barrier
    // precedes the ONE lane whose agent-scope atomic add takes the ticket.  Consumer side, the
    // "Consumer, always" form: that add's return value is the poll, then ONE agent acquire by the
    // same lane, vmcnt(0) (the invalidate has completed), and the barrier below before any wave
    // reads a partial.  The sc1-loads-instead-of-acquire shortcut (row 1 of the hand-off table)
    // needs one workgroup per CU, which these kernels do not have (several blocks share a CU), so
    // the acquire stays; only the last arriver pays it.  The loads stay sc1 (L2-served) as well.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the broadcast word: past the staging tile where the LDS has room (the last arriver then takes
    // its own partial from the staging tile), else in it -- inside the same LDS array either way
    const bool own_lds = flag_off >= 0;
    int* flag = reinterpret_cast<int*>(own_lds ? lds + flag_off : lds);
    if (tid == 0) {
      int* ctr = p.counters + tile;
      const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == nsplit - 1;
      if (last) {
        __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    // Sum in split order (bit-identical to the two-kernel form): per chunk and split ONE round of
    // loads for the chunk's groups; this block's own partial comes from its staging tile.
    const int own = streamk ? split - sk_first : split;  // this block's place in the summation order
#pragma unroll
    for (int c0 = 0; c0 < NG; c0 += CH) {
      load_res(c0);
      float v[CH][8];
#pragma unroll
      for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int t = 0; t < 8; ++t) v[j][t] = 0.f;
      for (int s = 0; s < nsplit; ++s) {
        const int sl = streamk ? sk.slab(sk_first + s, tile) : s;
        float4 cur[CH][2];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          if (s == own && own_lds) {
            stage8(c0 + j, cur[j][0], cur[j][1]);
          } else {
            const unsigned o = part_off(sl, c0 + j);
            cur[j][0] = ld4_sc1(wsr, o);
            cur[j][1] = ld4_sc1(wsr, o + 16);
          }
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          v[j][0] += cur[j][0].x; v[j][1] += cur[j][0].y; v[j][2] += cur[j][0].z; v[j][3] += cur[j][0].w;
          v[j][4] += cur[j][1].x; v[j][5] += cur[j][1].y; v[j][6] += cur[j][1].z; v[j][7] += cur[j][1].w;
        }
      }
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (gm[c0 + j] >= 0) finish(c0, j, v[j]);
    }
    return;
  }
  // ---- ragged N (e.g. a 10-class head): element-wise epilogue from registers ----
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn * WN + i * 16 + ln;
    if (n >= p.N) continue;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = rows(wm * WM + j * 16 + lm);
      if (m < 0) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (n + r >= p.N) break;
        const size_t o = static_cast<size_t>(m) * p.N + n + r;
        float v = acc[i][j][r];
        if (p.row_stats)
          v = p.row_stats[2 * static_cast<size_t>(m) + 1] * (v - p.row_stats[2 * static_cast<size_t>(m)] * p.col_sum[n + r]);
        v += p.bias ? p.bias[n + r] : 0.f;
        if (p.res) v += load1v(p.res + o, p.oplane, p.split);
        if (p.relu) v = act_fn(v, p.relu, p.clip_lo, p.clip_hi);
        if (p.out) store1v(p.out + o, p.oplane, p.split, v);
        if (p.out_f32) p.out_f32[o] = v;
        if (p.out2) {
          float u = v * p.scale2[n + r] + p.shift2[n + r];
          if (p.relu2) u = fmaxf(u, 0.f);
          store1v(p.out2 + o, p.oplane, p.split, u);
        }
      }
    }
  }
}

// Sum the split-K partials and apply the epilogue; one thread per 8 channels of one pixel.
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const ConvArgs p) {
  const int GPR = p.N / 8;
  const long long total = static_cast<long long>(p.M) * GPR;
  const size_t slab = static_cast<size_t>(p.M) * p.N;
  for (long long g = blockIdx.x * 256ll + threadIdx.x; g < total; g += static_cast<long long>(gridDim.x) * 256) {
    const int m = static_cast<int>(g / GPR);
    const int n = static_cast<int>(g - static_cast<long long>(m) * GPR) * 8;
    const float* src = p.ws + static_cast<size_t>(m) * p.N + n;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < p.splits; ++s) {
      const float4 a = ldf4(src + s * slab), b = ldf4(src + s * slab + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    epilogue8(p, m, n, v);
  }
}

// ------------------------------------------------------------------------------------------------
// v3 main loop: operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging,
// no ds_write), STAGES-deep ring with a counted `s_waitcnt vmcnt(N)` and a raw s_barrier per K-step,
// so STAGES-1 K-steps stay in flight across the barrier.  The DMA writes 1 KiB per wave-instruction
// lane-linearly (8 rows x 128 B), so the (row>>1)&7 chunk swizzle goes on the per-lane SOURCE
// address.  Padding pixels and M tails read a zero page instead of being predicated.
// MODE 0: dense rows (1x1/s1 conv, GEMM), K % 64 == 0.  MODE 3: patchify conv (stride == kernel, no
// padding, KW * Cin % 64 == 0: a K-step is a contiguous piece of one input row of the patch).
// MODE 2: implicit conv with Cin % 64 == 0
// (one 64-channel K-step never straddles a filter tap, so the tap is wave-uniform per K-step).
// ------------------------------------------------------------------------------------------------
// s_waitcnt with only the vector-memory counter constrained (gfx9 simm16: vmcnt = bits 3:0 + 15:14,
// expcnt 6:4 and lgkmcnt 11:8 left at their maxima).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Wait until at most j*G of this wave's DMA instructions are outstanding, j <= J (j wave-uniform).
template <int G, int J>
__device__ __forceinline__ void wait_stages(int j) {
  if constexpr (J == 0) {
    wait_vmcnt<0>();
  } else {
    if (j >= J) wait_vmcnt<G * J>();
    else wait_stages<G, J - 1>(j);
  }
}

__device__ __forceinline__ void glds16(const uint16_t* g, uint16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// 8 bf16 (one MFMA operand fragment, 8 consecutive channels) -> act(v * s + h), re-rounded to bf16.
__device__ __forceinline__ bf16x8 bn_act8(bf16x8 f, float4 s0, float4 s1, float4 h0, float4 h1, int relu) {
  const uint4 q = __builtin_bit_cast(uint4, f);
  float v[8];
  unpack2(q.x, v[0], v[1]);
  unpack2(q.y, v[2], v[3]);
  unpack2(q.z, v[4], v[5]);
  unpack2(q.w, v[6], v[7]);
  const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    v[t] = fmaf(v[t], sc[t], sh[t]);
    if (relu) v[t] = fmaxf(v[t], 0.f);
  }
  return __builtin_bit_cast(bf16x8, make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])));
}

constexpr int kBnlMaxK = 2048;  // pre-activation on load: channels staged in LDS

// SPLIT (fp32 mode): each stage holds [A_hi][B_hi][A_lo][B_lo]; the lo tiles are DMA'd from the
// planes wplane / xplane elements after the hi ones (zero-page rows stay zero-page), and every
// fragment pair takes three MFMAs (hi*hi + lo*hi + hi*lo).
// SK: the stream-K form (ConvArgs::sk > 0), a separate instantiation so that the plain kernels keep
// their register allocation (the segment walk around the body cost ~50 VGPRs in the same kernel).
template <int BM, int BN, int MODE, int STAGES, bool BNL = false, bool SPLIT = false, int BKS = BK, bool SK = false>
__global__ __launch_bounds__(256) void conv_glds_kernel(const ConvArgs p, const int kt_per_split) {
  static_assert(BKS == 64 || BKS == 32, "K-step width");
  constexpr int CPR = BKS / 8;        // 16-byte chunks per LDS row
  constexpr int RPI = 512 / BKS;      // rows per 1 KiB DMA wave-instruction
  constexpr int KSUB = BKS / 32;      // MFMA K=32 substeps per K-step
  constexpr int KR = BK / BKS;        // K-steps per 64-wide split-K unit
  auto sw = [](int row, int chunk) { return row * BKS + ((chunk ^ ((row >> 1) & (CPR - 1))) << 3); };
  constexpr int NP = SPLIT ? 2 : 1;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_ELEMS = BN * BKS, B_ELEMS = BM * BKS, PLANE = A_ELEMS + B_ELEMS, STAGE = NP * PLANE;
  constexpr int GA = BN / 4 / RPI, GB = BM / 4 / RPI, G = NP * (GA + GB);  // DMA instructions per wave per stage
  // epilogue: the f32 tile, plus (fp32: ConvArgs::row_parts readers) the BM (mean, rstd) row cache
  constexpr int EPI_ELEMS = BM * BN * 2 + (SPLIT ? BM * 4 : 0);
  constexpr int LDS_ELEMS = STAGES * STAGE > EPI_ELEMS ? STAGES * STAGE : EPI_ELEMS;
  // One LDS array: the stage ring / epilogue tile, then (BNL) the channel table.  No separate
  // dummy arrays: a 1-stage split 64x64 block is exactly 32 KiB.
  constexpr int BNL_ELEMS = BNL ? 2 * 2 * kBnlMaxK : 0;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS + BNL_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int nk_total = p.Kpad / BKS;
  // One output tile's K-steps [kt_begin, kt_end): the whole kernel for a plain / split-K launch,
  // one segment of the block's range for a stream-K launch (nsplit, sk, sk_first: tile_epilogue).
  auto run = [&](int tile_m, int tile_n, int split, int tile, int kt_begin, int kt_end, int nsplit, StreamK sk,
                 int sk_first) {
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = kt_end - kt_begin;
  // pre-activation on load: this slice's per-channel scale/shift in LDS (K = channels for 1x1)
  float* bnl = reinterpret_cast<float*>(lds + LDS_ELEMS);  // BNL only: [scale | shift] x kBnlMaxK
  if constexpr (BNL) {
    for (int i = tid; i < nk * BKS; i += 256) {
      bnl[i] = p.in_scale[kt_begin * BKS + i];
      bnl[kBnlMaxK + i] = p.in_shift[kt_begin * BKS + i];
    }
    // visible to every wave after the main loop's first barrier
  }

  // Per-lane DMA sources.  Wave `wave` fills rows [wave*R/4, (wave+1)*R/4) of each operand, 8 rows
  // per instruction (16 for 32-wide K-steps); lane L -> row L / CPR of that group, physical chunk L % CPR.
  const uint16_t* asrc[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = wave * (BN / 4) + i * RPI + lane / CPR;
    const int c = (lane % CPR) ^ ((r >> 1) & (CPR - 1));
    asrc[i] = p.w + static_cast<size_t>(n0 + r) * p.Kpad + c * 8;
  }
  // MODE 0: each lane's row pointer, M-tail rows pointed into the zero page (which holds a whole
  // K row), so a K-step is one pointer add.  MODE 2: image base + channel chunk and the output
  // pixel's top-left input coordinate; taps advance incrementally (no divisions in the loop).
  const uint16_t* bsrc[GB];
  int bih[GB], biw[GB];
  bool bval[GB];
  long long bdel[GB];  // SPLIT, MODE 0: distance to the lo plane (0 for zero-page tail rows)
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = wave * (BM / 4) + i * RPI + lane / CPR;
    const int c = (lane % CPR) ^ ((r >> 1) & (CPR - 1));
    const int m = m0 + r;
    bval[i] = m < p.M;
    bdel[i] = bval[i] ? p.xplane : 0;
    const int mm = bval[i] ? m : 0;
    if (MODE == 0) {
      bsrc[i] = (bval[i] ? p.x + static_cast<size_t>(mm) * p.Cin : p.zeros) + c * 8;
      bih[i] = biw[i] = 0;
    } else if (MODE == 3) {  // patchify: the patch's top-left input pixel (tail rows: the zero page)
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int rr = mm - b * hw;
      const int oh = rr / p.Wo;
      const int ow = rr - oh * p.Wo;
      bsrc[i] = (bval[i] ? p.x + ((static_cast<size_t>(b) * p.H + oh * p.stride) * p.W + ow * p.stride) * p.Cin : p.zeros) +
                c * 8;
      bih[i] = biw[i] = 0;
    } else {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw;
      const int rr = mm - b * hw;
      const int oh = rr / p.Wo;
      const int ow = rr - oh * p.Wo;
      bih[i] = bval[i] ? oh * p.stride - p.pad_h : -(1 << 20);  // tail rows never pass the bounds test
      biw[i] = ow * p.stride - p.pad_w;
      bsrc[i] = p.x + static_cast<size_t>(b) * p.H * p.W * p.Cin + c * 8;
    }
  }
  // uniform state of the next K-step to issue (MODE 2: channel offset within the tap, tap x/y)
  int nx_k0 = kt_begin * BKS;
  int nx_ci0 = 0, nx_kx = 0, nx_ky = 0;
  if (MODE == 2) {
    const int cpt = p.Cin / BKS;  // K-steps per filter tap
    const int tap = kt_begin / cpt;
    nx_ci0 = (kt_begin - tap * cpt) * BKS;
    nx_ky = tap / p.KW;
    nx_kx = tap - nx_ky * p.KW;
  }

  // DMA the K-step at the current state into stage `buf` and advance the state.
  auto issue = [&](int buf) {
    uint16_t* A = lds + buf * STAGE;
    uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int i = 0; i < GA; ++i) glds16(asrc[i] + nx_k0, A + (wave * (BN / 4) + i * RPI) * BKS);
    if constexpr (SPLIT) {
#pragma unroll
      for (int i = 0; i < GA; ++i) glds16(asrc[i] + p.wplane + nx_k0, A + PLANE + (wave * (BN / 4) + i * RPI) * BKS);
    }
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        glds16(bsrc[i] + nx_k0, Bt + (wave * (BM / 4) + i * RPI) * BKS);
        if constexpr (SPLIT) glds16(bsrc[i] + bdel[i] + nx_k0, Bt + PLANE + (wave * (BM / 4) + i * RPI) * BKS);
      }
    } else if (MODE == 3) {
      // K order (ky, kx, c): a K-step is a contiguous piece of one kernel row of the patch, i.e. of
      // one input row (stride == kernel, no padding)
      const int rowlen = p.KW * p.Cin;
      const int ky = nx_k0 / rowlen;
      const long long d = static_cast<long long>(ky) * p.W * p.Cin + (nx_k0 - ky * rowlen);
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const uint16_t* src = bval[i] ? bsrc[i] + d : bsrc[i];
        glds16(src, Bt + (wave * (BM / 4) + i * RPI) * BKS);
        if constexpr (SPLIT) glds16(src + bdel[i], Bt + PLANE + (wave * (BM / 4) + i * RPI) * BKS);
      }
    } else {
      const int dy = nx_ky * p.dil, dx = nx_kx * p.dil;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int ih = bih[i] + dy;
        const int iw = biw[i] + dx;
        const bool v = static_cast<unsigned>(ih) < static_cast<unsigned>(p.H) &&
                       static_cast<unsigned>(iw) < static_cast<unsigned>(p.W);
        const uint16_t* src = v ? bsrc[i] + ((ih * p.W + iw) * p.Cin + nx_ci0) : p.zeros;
        glds16(src, Bt + (wave * (BM / 4) + i * RPI) * BKS);
        if constexpr (SPLIT) glds16(v ? src + p.xplane : p.zeros, Bt + PLANE + (wave * (BM / 4) + i * RPI) * BKS);
      }
      nx_ci0 += BKS;
      if (nx_ci0 == p.Cin) {
        nx_ci0 = 0;
        if (++nx_kx == p.KW) {
          nx_kx = 0;
          ++nx_ky;
        }
      }
    }
    nx_k0 += BKS;
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One K-step's MFMAs on the stage at A (K-step t of this slice, for the BNL channel table).
  auto compute = [&](const uint16_t* A, int t) {
    const uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int s = 0; s < KSUB; ++s) {
      const int chunk = s * 4 + (lane >> 4);
      bf16x8 af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + sw(wn * WN + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + sw(wm * WM + j * 16 + (lane & 15), chunk));
      if constexpr (SPLIT) {
        bf16x8 afl[TN], bfl[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i)
          afl[i] = *reinterpret_cast<const bf16x8*>(A + PLANE + sw(wn * WN + i * 16 + (lane & 15), chunk));
#pragma unroll
        for (int j = 0; j < TM; ++j)
          bfl[j] = *reinterpret_cast<const bf16x8*>(Bt + PLANE + sw(wm * WM + j * 16 + (lane & 15), chunk));
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
          }
      }
      if constexpr (BNL) {
        const float* sc = bnl + t * BKS + chunk * 8;
        const float4 s0 = *reinterpret_cast<const float4*>(sc), s1 = *reinterpret_cast<const float4*>(sc + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(sc + kBnlMaxK);
        const float4 h1 = *reinterpret_cast<const float4*>(sc + kBnlMaxK + 4);
#pragma unroll
        for (int j = 0; j < TM; ++j) bfr[j] = bn_act8(bfr[j], s0, s1, h0, h1, p.in_relu);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // row_parts reader (fp32 only): the rows' statistics groups are loaded ahead of the first
  // K-step's DMA and merged while it is in flight
  RowParts<BM> rp;
  float2 rms = make_float2(0.f, 0.f);
  const bool rp_on = SPLIT && p.row_parts;
  if (rp_on) rp.issue(p, m0, tid);

  if constexpr (STAGES == 1) {
    // No ring: load, wait, compute, once per K-step.  Meant for nk == 1 (K <= 64: the expand /
    // reduce convs of stage 1), where a ring buys nothing and a 1-stage LDS footprint lets 2-4x
    // more blocks share a CU to hide the load and epilogue latency.
    // (the first K-step's DMA issued ahead of the loop, so that the row_parts merge runs under it
    // outside the loop -- merged inside it, at t == 0, the 64-row tiles' statistics came out wrong)
    const bool dma = p.probe != 1, mfma = p.probe != 2;  // ConvArgs::probe (measurement only)
    if (nk > 0 && dma) issue(0);
    if (rp_on) rms = rp.merge(p);
    for (int t = 0; t < nk; ++t) {
      if (t) {
        __syncthreads();  // everyone done reading the previous K-step
        if (dma) issue(0);
      }
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (mfma) compute(lds, t);
    }
  } else {
    const bool dma = p.probe != 1, mfma = p.probe != 2;
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk && dma) issue(s);
    if (rp_on) rms = rp.merge(p);
    int rd = 0, wr = STAGES - 1;  // ring indices of the stage read this step / the stage issued next
    for (int t = 0; t < nk; ++t) {
      // Stage t has landed for this wave once at most min(STAGES-2, nk-1-t) younger stages (G DMA
      // instructions each) are outstanding.
      wait_stages<G, STAGES - 2>(nk - 1 - t);
      __builtin_amdgcn_s_barrier();  // ... and for every wave; also: everyone is done reading stage t-1
      asm volatile("" ::: "memory");
      if (t + STAGES - 1 < nk && dma) issue(wr);
      wr = wr + 1 == STAGES ? 0 : wr + 1;
      const uint16_t* A = lds + rd * STAGE;
      rd = rd + 1 == STAGES ? 0 : rd + 1;
      if (mfma) compute(A, t);
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // all operand reads done before the epilogue reuses the LDS
  tile_epilogue<BM, BN>(p, acc, lds, m0, n0, wm, wn, lane, tid, tile, split, LinearRows{0, 0}, rms,
                        epi_flag_off(LDS_ELEMS, EPI_ELEMS), nsplit, sk, sk_first);
  };

  if constexpr (SK) {
    // Stream-K (ConvArgs::sk): the grid's P blocks split the T x nk_total (tile, K-step) iterations
    // evenly; block id (XCD-remapped, so consecutive ranges -- a tile's contributors -- share an XCD)
    // walks its range tile by tile: a tile inside the range runs whole with the direct epilogue, a
    // cut one leaves a partial for the tile's last arriving contributor (tile_epilogue).  (One call
    // site of `run`, so the body is inlined once.)
    const int ntn = (p.N + BN - 1) / BN;
    const int Ml = p.live ? min(p.M, static_cast<int>(*p.live) * p.Ho * p.Wo) : p.M;
    const int ntm = (Ml + BM - 1) / BM;
    StreamK sk;
    sk.nk = nk_total;
    sk.I = static_cast<long long>(ntm) * ntn * nk_total;
    sk.P = static_cast<int>(gridDim.x);
    const int nb = sk.P, b = blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7;
    const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
    long long it = sk.start(id);
    const long long end = sk.start(id + 1);
    for (bool first_seg = true; it < end; first_seg = false) {
      const int tile = static_cast<int>(it / nk_total);
      const long long tb = static_cast<long long>(tile) * nk_total, te = tb + nk_total;
      const int kt_begin = static_cast<int>(it - tb);
      const int kt_end = static_cast<int>((end < te ? end : te) - tb);
      const int first = sk.owner(tb), last = sk.owner(te - 1);
      int tile_m, tile_n;
      tile_mn(p, ntm, ntn, tile, tile_m, tile_n);
      it += kt_end - kt_begin;
      if (!first_seg) __syncthreads();  // every wave done with the previous segment's LDS
      run(tile_m, tile_n, first == last ? -1 : id, tile, kt_begin, kt_end, last - first + 1, sk, first);
    }
  } else {
    int tile_m, tile_n, split, tile;
    if (!block_coords(p, BM, BN, tile_m, tile_n, split, tile)) return;  // whole block, before any barrier
    // kt_per_split counts 64-wide K-steps; split < 0: a whole tile of a tail split-K launch
    const int kt_begin = split < 0 ? 0 : split * kt_per_split * KR;
    const int kt_end = split < 0 ? nk_total : min(nk_total, kt_begin + kt_per_split * KR);
    run(tile_m, tile_n, split, tile, kt_begin, kt_end, -1, StreamK{}, 0);
  }
}

// ------------------------------------------------------------------------------------------------
// Spatially tiled 3x3 / stride 1 / pad 1 conv (Cin % 64 == 0), 64 output channels x an 8x8 pixel
// tile per block.  The implicit-GEMM loop above reads one 64-channel row per output pixel per
// filter tap, i.e. every input pixel ~9 times per N-tile; here a block stages the 10x10 input patch
// of its tile once per 64-channel slice and serves all 9 taps from it (tap (dy, dx) = the patch
// window shifted by (dy, dx)), so a slice costs one patch + 9 weight K-steps (~19 KB/tap in fp32
// split mode instead of 32 KB).  One stage, no ring (the loop the tuner prefers at these sizes).
// Patch LDS layout: pixel q = row * 10 + col, 128 B per pixel, 16-B chunk c stored at
// c ^ g(col) ^ h(row): tables found by exhaustive search so that every ds_read_b128 lane group of
// every (tap, fragment, K-half) hits 16 distinct bank slots.
// Split-K runs over channel slices (kt_per_split counts slices here).
constexpr uint32_t kPatchSwzCol = 0x37b77b77u, kPatchSwzRow = 0x1d5c7555u;
__device__ __forceinline__ int patch_swz(int row, int col) {
  return static_cast<int>(((kPatchSwzCol >> (3 * col)) ^ (kPatchSwzRow >> (3 * row))) & 7u);
}

struct SpatialRows {  // tile row r (8x8 pixel tile, raster) -> output pixel, -1 outside the image
  int b, ty0, tx0, Ho, Wo;
  __device__ __forceinline__ int operator()(int r) const {
    const int oy = ty0 + (r >> 3), ox = tx0 + (r & 7);
    return oy < Ho && ox < Wo ? (b * Ho + oy) * Wo + ox : -1;
  }
};

template <bool SPLIT>
__global__ __launch_bounds__(256) void conv3x3_spatial_kernel(const ConvArgs p, const int sl_per_split) {
  constexpr int BM = 64, BN = 64, NP = SPLIT ? 2 : 1;
  constexpr int PW = 10, NPIX = 100, PINSTR = 13;          // patch pixels; 1 KiB (8-pixel) DMA pieces
  constexpr int PPLANE = PINSTR * 8 * 64, APLANE = BN * BK;  // elements per plane
  constexpr int PATCH = NP * PPLANE, WTS = NP * APLANE;
  constexpr int LDS_ELEMS = PATCH + WTS > BM * BN * 2 ? PATCH + WTS : BM * BN * 2;
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];
  uint16_t* patch = lds;
  uint16_t* A = lds + PATCH;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  // block -> (image tile, N-tile, channel-slice range), XCD-aware as block_coords
  const int tiles_x = (p.Wo + 7) >> 3, tiles_y = (p.Ho + 7) >> 3, tpi = tiles_x * tiles_y;
  const int Bl = p.live ? min(p.B, static_cast<int>(*p.live)) : p.B;
  const int ntm = Bl * tpi, ntn = (p.N + BN - 1) / BN, S = gridDim.y;
  const int nwg = min(static_cast<int>(gridDim.x * gridDim.y), ntm * ntn * S);
  const int bid = blockIdx.x + blockIdx.y * gridDim.x;
  if (bid >= nwg) return;  // whole block, before any barrier
  const int q8 = nwg >> 3, r8 = nwg & 7, x8 = bid & 7;
  const int id = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + (bid >> 3);
  const int tile = id / S, split = id - tile * S;
  int tile_m, tile_n;
  if (p.order == 1 || (p.order == 0 && static_cast<long long>(p.N) * p.K <= static_cast<long long>(p.B) * p.H * p.W * p.Cin)) {
    tile_m = tile / ntn;
    tile_n = tile - tile_m * ntn;
  } else {
    tile_n = tile / ntm;
    tile_m = tile - tile_n * ntm;
  }
  const int b = tile_m / tpi, tt = tile_m - b * tpi;
  const int ty0 = (tt / tiles_x) * 8, tx0 = (tt - (tt / tiles_x) * tiles_x) * 8;
  const int n0 = tile_n * BN;
  const int nsl = p.Cin / BK;
  const int cs0 = split * sl_per_split, cs1 = min(nsl, cs0 + sl_per_split);

  // patch DMA sources: piece I = wave + 4i (< 13), lane -> pixel I*8 + lane/8, physical chunk lane%8
  const uint16_t* psrc[4];
  bool pval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int I = wave + 4 * i;
    const int q = I * 8 + (lane >> 3);
    const int py = q / PW, px = q - (q / PW) * PW;
    const int iy = ty0 - 1 + py, ix = tx0 - 1 + px;
    pval[i] = I < PINSTR && q < NPIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    const int c = (lane & 7) ^ (q < NPIX ? patch_swz(py, px) : 0);
    psrc[i] = pval[i] ? p.x + ((static_cast<size_t>(b) * p.H + iy) * p.W + ix) * p.Cin + c * 8 : p.zeros;
  }
  // weight DMA sources: rows wave*16 + i*8 + lane/8 of this N-tile
  const uint16_t* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wave * (BN / 4) + i * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    asrc[i] = p.w + static_cast<size_t>(n0 + r) * p.Kpad + c * 8;
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cs = cs0; cs < cs1; ++cs) {
    for (int tap = 0; tap < 9; ++tap) {
      if (cs != cs0 || tap) __syncthreads();  // every wave done reading the patch / weights
      if (tap == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int I = wave + 4 * i;
          if (I >= PINSTR) break;  // wave-uniform
          const uint16_t* src = psrc[i] + (pval[i] ? cs * BK : 0);
          glds16(src, patch + I * 512);
          if constexpr (SPLIT) glds16(pval[i] ? src + p.xplane : p.zeros, patch + PPLANE + I * 512);
        }
      }
      const int k0 = tap * p.Cin + cs * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        glds16(asrc[i] + k0, A + (wave * (BN / 4) + i * 8) * BK);
        if constexpr (SPLIT) glds16(asrc[i] + p.wplane + k0, A + APLANE + (wave * (BN / 4) + i * 8) * BK);
      }
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int dy = tap / 3, dx = tap - dy * 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int chunk = s * 4 + (lane >> 4);
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(A + swz(wn * 32 + i * 16 + (lane & 15), chunk));
        int boff[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int pix = j * 16 + (lane & 15);
          const int row = wm * 4 + (pix >> 3) + dy, col = (pix & 7) + dx;
          boff[j] = (row * PW + col) * BK + ((chunk ^ patch_swz(row, col)) << 3);
          bfr[j] = *reinterpret_cast<const bf16x8*>(patch + boff[j]);
        }
        if constexpr (SPLIT) {
          bf16x8 afl[2], bfl[2];
#pragma unroll
          for (int i = 0; i < 2; ++i)
            afl[i] = *reinterpret_cast<const bf16x8*>(A + APLANE + swz(wn * 32 + i * 16 + (lane & 15), chunk));
#pragma unroll
          for (int j = 0; j < 2; ++j) bfl[j] = *reinterpret_cast<const bf16x8*>(patch + PPLANE + boff[j]);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // all operand reads done before the epilogue reuses the LDS
  tile_epilogue<BM, BN>(p, acc, lds, 0, n0, wm, wn, lane, tid, tile, split, SpatialRows{b, ty0, tx0, p.Ho, p.Wo},
                        float2{0.f, 0.f}, epi_flag_off(LDS_ELEMS, BM * BN * 2));
}

template <int BM, int BN, int STAGES, int BKS = BK>
bool launch_glds(int mode, dim3 grid, hipStream_t s, const ConvArgs& b, int kt_per) {
  const bool mode0 = mode == 0;
  if (mode == 3) {  // patchify convs (ViT patch embedding): 1- and 2-stage loops only
    if constexpr (STAGES <= 2) {
      if (b.split) {
        if constexpr (STAGES * (BM + BN) * BKS * 4 <= 160 * 1024)
          hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 3, STAGES, false, true, BKS>), grid, dim3(256), 0, s, b, kt_per);
        else
          return false;
      } else if (!b.in_scale) {
        hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 3, STAGES, false, false, BKS>), grid, dim3(256), 0, s, b, kt_per);
      } else {
        return false;
      }
      return true;
    } else {
      return false;
    }
  }
  if (b.sk > 0) {  // stream-K: 1- and 2-stage loops, no pre-activation on load
    if constexpr (STAGES <= 2 && BKS == BK) {
      if (b.in_scale) return false;
      if (b.split) {
        if constexpr (STAGES * (BM + BN) * BKS * 4 <= 160 * 1024) {
          if (mode0) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 0, STAGES, false, true, BKS, true>), grid, dim3(256), 0, s, b, kt_per);
          else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 2, STAGES, false, true, BKS, true>), grid, dim3(256), 0, s, b, kt_per);
        } else {
          return false;
        }
      } else if (mode0) {
        hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 0, STAGES, false, false, BKS, true>), grid, dim3(256), 0, s, b, kt_per);
      } else {
        hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 2, STAGES, false, false, BKS, true>), grid, dim3(256), 0, s, b, kt_per);
      }
      return true;
    } else {
      return false;
    }
  }
  if (b.split) {  // only ring depths whose doubled stages fit the LDS are instantiated
    if constexpr (STAGES * (BM + BN) * BKS * 4 <= 160 * 1024) {
      if (mode0) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 0, STAGES, false, true, BKS>), grid, dim3(256), 0, s, b, kt_per);
      else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 2, STAGES, false, true, BKS>), grid, dim3(256), 0, s, b, kt_per);
    }
  } else if (b.in_scale) {
    if (mode0) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 0, STAGES, true, false, BKS>), grid, dim3(256), 0, s, b, kt_per);
    else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 2, STAGES, true, false, BKS>), grid, dim3(256), 0, s, b, kt_per);
  } else if (mode0) {
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 0, STAGES, false, false, BKS>), grid, dim3(256), 0, s, b, kt_per);
  } else {
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, 2, STAGES, false, false, BKS>), grid, dim3(256), 0, s, b, kt_per);
  }
  return true;
}

template <int BM, int BN>
hipError_t launch_cfg(const ConvArgs& a, hipStream_t s, int variant) {
  const bool dense1x1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad_h == 0 && a.pad_w == 0 && a.H == a.Ho &&
                        a.W == a.Wo;
  const int vec = a.Cin % 8 == 0 ? 8 : 4;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int nk = a.Kpad / BK;
  const int splits = std::max(1, std::min(a.splits, nk));
  const int kt_per = (nk + splits - 1) / splits;
  const int eff = (nk + kt_per - 1) / kt_per;  // no empty slices
  ConvArgs b = a;
  b.splits = eff;
  if (a.split) {  // plane distances of the split activations (weights: set by the planner)
    b.xplane = static_cast<long long>(a.B) * a.H * a.W * a.Cin;
    b.oplane = static_cast<long long>(a.M) * a.N;
    if (a.wplane <= 0 || a.in_scale) return hipErrorInvalidValue;
  } else {
    b.xplane = b.oplane = 0;
  }
  // fused split-K reduction needs a zeroed counter per output tile
  const bool fused = eff > 1 && a.counters && tiles <= a.counters_n;
  if (!fused) b.counters = nullptr;
  if (a.sk > 0) {
    // stream-K: LDS-DMA loops only, in-kernel reduction only (a counter per tile), P blocks
    if (variant < 1 || variant > 5 || !a.counters || tiles > a.counters_n || !a.ws || a.N % 8 || a.tail > 0 ||
        a.in_scale || a.row_parts || a.stats_out)
      return hipErrorInvalidValue;
    b.counters = a.counters;
    b.splits = 1;
  }
  // LayerNorm statistics (ConvArgs::stats_out / row_parts): rows GEMMs, not the spatially tiled 3x3
  if ((a.stats_out || a.row_parts) && variant == 6) return hipErrorInvalidValue;
  dim3 grid(tiles, eff);
  if (a.sk > 0) grid = dim3(a.sk, 1);
  if (a.tail > 0) {
    // tail split-K: 1-D grid sized for the worst live batch (the whole-tile count steps down at
    // every multiple of `tail`, so fewer live tiles can need more blocks)
    if (!fused || variant == 0 || variant >= 6) return hipErrorInvalidValue;
    const int ntn = (a.N + BN - 1) / BN, ntm = (a.M + BM - 1) / BM;
    int g = 0;
    for (int m = 1; m <= ntm; ++m) {
      const int T = m * ntn, Tw = T > a.tail ? T - T % a.tail : T;
      g = std::max(g, Tw + (T - Tw) * eff);
    }
    grid = dim3(g, 1);
  }
  if (a.in_scale) {  // pre-activation on load: 1x1 convs in the LDS-DMA loop only
    if (a.KH != 1 || a.KW != 1 || a.pad_h || a.pad_w || a.K != a.Cin || a.K > kBnlMaxK || a.Cin % BK || !a.in_shift)
      return hipErrorInvalidValue;
    if (variant == 0) variant = 1;  // the register-staged loop has no pre-activation: 2-stage ring
  }
  if (variant == 6) {  // spatially tiled 3x3/s1/p1 (64x64 tile only): split-K over channel slices
    if constexpr (BM == 64 && BN == 64) {
      if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.dil != 1 || a.pad_h != 1 || a.pad_w != 1 || a.H != a.Ho ||
          a.W != a.Wo || a.Cin % BK || a.K != 9 * a.Cin || a.Kpad != a.K || a.N % 8 || !a.zeros || a.in_scale)
        return hipErrorInvalidValue;
      const int nsl = a.Cin / BK;
      const int sp = std::max(1, std::min(a.splits, nsl));
      const int per = (nsl + sp - 1) / sp, effs = (nsl + per - 1) / per;
      const int stiles = a.B * ((a.Ho + 7) / 8) * ((a.Wo + 7) / 8) * ((a.N + 63) / 64);
      ConvArgs c = b;
      c.splits = effs;
      const bool sfused = effs > 1 && a.counters && stiles <= a.counters_n;
      if (!sfused) c.counters = nullptr;
      if (c.split) hipLaunchKernelGGL(conv3x3_spatial_kernel<true>, dim3(stiles, effs), dim3(256), 0, s, c, per);
      else hipLaunchKernelGGL(conv3x3_spatial_kernel<false>, dim3(stiles, effs), dim3(256), 0, s, c, per);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess || effs == 1 || sfused) return e;
      const long long groups = static_cast<long long>(c.M) * (c.N / 8);
      hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(static_cast<int>(std::min<long long>((groups + 255) / 256, 8192))),
                         dim3(256), 0, s, c);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  if (variant > 0) {  // LDS-DMA pipeline: needs whole 64-wide K-steps of real data
    const bool mode0 = dense1x1 && a.K % BK == 0 && a.Cin == a.K;
    const bool mode2 = !dense1x1 && a.Cin % BK == 0;
    // patchify (stride == kernel, no padding, a kernel row = whole 64-wide K-steps): dense row pieces
    const bool mode3 = !dense1x1 && !mode2 && a.KH == a.stride && a.KW == a.stride && a.stride > 1 && a.dil == 1 &&
                       a.pad_h == 0 && a.pad_w == 0 && (a.KW * a.Cin) % BK == 0 && a.K == a.KH * a.KW * a.Cin &&
                       a.Kpad == a.K && a.Ho == (a.H - a.KH) / a.stride + 1 && a.Wo == (a.W - a.KW) / a.stride + 1;
    if (!a.zeros || !(mode0 || mode2 || mode3)) return hipErrorInvalidValue;
    const int mode = mode0 ? 0 : mode2 ? 2 : 3;
    // ring depth per variant: 2, 3, 4, 6 stages (6 only where it fits the 160 KiB LDS); variant 5 =
    // one stage, no ring.  (Measured and dropped: rings of 32-wide K-steps, conv_glds_kernel<...,
    // BKS = 32>, at the 1-stage footprint, and a 1-stage loop that also touched the next K-step's
    // lines toward L2 with 4-byte LDS-DMA loads: both slower, profiles/r2_feed_calibration.md.)
    constexpr int kStageBytes = (BM + BN) * BK * 2;
    if (a.in_scale && variant == 4) return hipErrorInvalidValue;  // 6 stages + the channel table exceed the LDS
    // split stages are twice as large: 128x128 fits 2 stages, 64-wide tiles 3-4 (160 KiB LDS)
    const int np = a.split ? 2 : 1;
    const int stages = variant == 1 ? 2 : variant == 2 ? 3 : variant == 3 ? 4 : variant == 4 ? 6 : 1;
    if (stages * kStageBytes * np > 160 * 1024) return hipErrorInvalidValue;
    bool ok = true;
    switch (variant) {
      case 1: ok = launch_glds<BM, BN, 2>(mode, grid, s, b, kt_per); break;
      case 2: ok = launch_glds<BM, BN, 3>(mode, grid, s, b, kt_per); break;
      case 3: ok = launch_glds<BM, BN, 4>(mode, grid, s, b, kt_per); break;
      case 5: ok = launch_glds<BM, BN, 1>(mode, grid, s, b, kt_per); break;
      default:
        if constexpr (6 * kStageBytes <= 160 * 1024) ok = launch_glds<BM, BN, 6>(mode, grid, s, b, kt_per);
        else return hipErrorInvalidValue;
    }
    if (!ok) return hipErrorInvalidValue;
  } else if (a.split) {
    if (dense1x1 && vec == 8) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 0, 8, true>), grid, dim3(256), 0, s, b, kt_per);
    else if (vec == 8) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 8, true>), grid, dim3(256), 0, s, b, kt_per);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 4, true>), grid, dim3(256), 0, s, b, kt_per);
  } else if (dense1x1 && vec == 8) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 0, 8>), grid, dim3(256), 0, s, b, kt_per);
  } else if (vec == 8) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 8>), grid, dim3(256), 0, s, b, kt_per);
  } else {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 1, 4>), grid, dim3(256), 0, s, b, kt_per);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || eff == 1 || fused || a.sk > 0) return e;
  const long long groups = static_cast<long long>(b.M) * (b.N / 8);
  const int g = static_cast<int>(std::min<long long>((groups + 255) / 256, 8192));
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(g), dim3(256), 0, s, b);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Wide-tile GEMM for the fp32 (split) rows GEMMs of transformers (MODE 0 only: dense rows, K % 64
// == 0).  256 pixels x BN = 128 channels per block, 512 threads = 8 waves in a 4 (pixels) x 2
// (channels) grid, each wave a 64 x 64 output, so two waves share every SIMD and hide each other's
// LDS reads under their MFMAs (the 4-wave 128x128 kernel has one).  32-wide K-steps (hi + lo planes
// of both operands = 48 KiB per stage) in a 3-deep LDS-DMA ring (144 KiB, one block per CU): two
// K-steps stay in flight across every barrier (counted vmcnt, raw s_barrier, as conv_glds_kernel).
// Per K-step a wave issues 16 ds_read_b128 for 48 MFMAs (1 : 3); the 256-row tile halves the weight
// bytes per output row against the 128-row tiles.
template <int BN>
__global__ __launch_bounds__(512) void gemm_wide_kernel(const ConvArgs p, const int kt_per_split) {
  constexpr int BM = 256, BKS = 32, NT = 512, WAVES_M = 4, WAVES_N = 2, STAGES = 3;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int CPR = BKS / 8, RPI = 512 / BKS;  // 16-B chunks per LDS row; rows per 1 KiB DMA instruction
  constexpr int A_ELEMS = BN * BKS, B_ELEMS = BM * BKS, PLANE = A_ELEMS + B_ELEMS, STAGE = 2 * PLANE;
  constexpr int GA = BN / 8 / RPI, GB = BM / 8 / RPI;  // DMA instructions per wave per plane
  constexpr int G = 2 * (GA + GB);
  static_assert(GA >= 1 && GB >= 1, "8 waves x 16 rows per DMA instruction");
  constexpr int EPI_ELEMS = BM * BN * 2 + BM * 4;  // f32 staging tile + row_parts row cache
  constexpr int LDS_ELEMS = STAGES * STAGE > EPI_ELEMS ? STAGES * STAGE : EPI_ELEMS;
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];
  auto sw = [](int row, int chunk) { return row * BKS + ((chunk ^ ((row >> 1) & (CPR - 1))) << 3); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  int tile_m, tile_n, split, tile;
  if (!block_coords(p, BM, BN, tile_m, tile_n, split, tile)) return;  // whole block, before any barrier
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk_total = p.Kpad / BKS;
  const int kt_begin = split * kt_per_split * 2;  // kt_per_split counts 64-wide K-steps
  const int kt_end = min(nk_total, kt_begin + kt_per_split * 2);
  const int nk = kt_end - kt_begin;

  // per-lane DMA sources (lane L -> row L / CPR of its 16-row group, physical chunk L % CPR; the
  // swizzle goes on the source address); M-tail rows read the zero page
  const uint16_t* asrc[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = wave * (BN / 8) + i * RPI + lane / CPR;
    const int c = (lane % CPR) ^ ((r >> 1) & (CPR - 1));
    asrc[i] = p.w + static_cast<size_t>(n0 + r) * p.Kpad + c * 8;
  }
  const uint16_t* bsrc[GB];
  long long bdel[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = wave * (BM / 8) + i * RPI + lane / CPR;
    const int c = (lane % CPR) ^ ((r >> 1) & (CPR - 1));
    const bool v = m0 + r < p.M;
    bsrc[i] = (v ? p.x + static_cast<size_t>(m0 + r) * p.Cin : p.zeros) + c * 8;
    bdel[i] = v ? p.xplane : 0;
  }
  int nx_k0 = kt_begin * BKS;
  auto issue = [&](int buf) {
    uint16_t* A = lds + buf * STAGE;
    uint16_t* Bt = A + A_ELEMS;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      glds16(asrc[i] + nx_k0, A + (wave * (BN / 8) + i * RPI) * BKS);
      glds16(asrc[i] + p.wplane + nx_k0, A + PLANE + (wave * (BN / 8) + i * RPI) * BKS);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      glds16(bsrc[i] + nx_k0, Bt + (wave * (BM / 8) + i * RPI) * BKS);
      glds16(bsrc[i] + bdel[i] + nx_k0, Bt + PLANE + (wave * (BM / 8) + i * RPI) * BKS);
    }
    nx_k0 += BKS;
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const uint16_t* A) {
    const uint16_t* Bt = A + A_ELEMS;
    const int chunk = lane >> 4;
    bf16x8 af[TN], afl[TN], bfr[TM], bfl[TM];
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int o = sw(wn * WN + i * 16 + (lane & 15), chunk);
      af[i] = *reinterpret_cast<const bf16x8*>(A + o);
      afl[i] = *reinterpret_cast<const bf16x8*>(A + PLANE + o);
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int o = sw(wm * WM + j * 16 + (lane & 15), chunk);
      bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + o);
      bfl[j] = *reinterpret_cast<const bf16x8*>(Bt + PLANE + o);
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
  };

  RowParts<BM, NT> rp;  // row_parts reader: loads ahead of the prologue DMA, merged under it
  float2 rms = make_float2(0.f, 0.f);
  if (p.row_parts) rp.issue(p, m0, tid);
  const bool dma = p.probe != 1, mfma = p.probe != 2;  // ConvArgs::probe (measurement only)
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk && dma) issue(s);
  if (p.row_parts) rms = rp.merge(p);
  int rd = 0, wr = STAGES - 1;
  for (int t = 0; t < nk; ++t) {
    wait_stages<G, STAGES - 2>(nk - 1 - t);  // stage t landed for this wave ...
    __builtin_amdgcn_s_barrier();             // ... and every wave; all done reading stage t - 1
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk && dma) issue(wr);
    wr = wr + 1 == STAGES ? 0 : wr + 1;
    const uint16_t* A = lds + rd * STAGE;
    rd = rd + 1 == STAGES ? 0 : rd + 1;
    if (mfma) compute(A);
  }
  wait_vmcnt<0>();
  __syncthreads();  // all operand reads done before the epilogue reuses the LDS
  tile_epilogue<BM, BN, LinearRows, NT, WAVES_M>(p, acc, lds, m0, n0, wm, wn, lane, tid, tile, split,
                                                 LinearRows{0, 0}, rms);
}

// 256 x 128 wide tile (gemm_wide_kernel): fp32 dense-rows GEMMs only.
inline hipError_t launch_wide(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 256, BN = 128;
  const bool dense = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad_h == 0 && a.pad_w == 0 && a.H == a.Ho &&
                     a.W == a.Wo && a.K % BK == 0 && a.Cin == a.K && a.Kpad == a.K;
  if (!dense || !a.split || a.in_scale || !a.zeros || a.wplane <= 0 || a.N % 8) return hipErrorInvalidValue;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int nk = a.Kpad / BK;
  const int splits = std::max(1, std::min(a.splits, nk));
  const int kt_per = (nk + splits - 1) / splits;
  const int eff = (nk + kt_per - 1) / kt_per;
  ConvArgs b = a;
  b.splits = eff;
  b.xplane = static_cast<long long>(a.B) * a.H * a.W * a.Cin;
  b.oplane = static_cast<long long>(a.M) * a.N;
  const bool fused = eff > 1 && a.counters && tiles <= a.counters_n;
  if (!fused) b.counters = nullptr;
  hipLaunchKernelGGL(gemm_wide_kernel<BN>, dim3(tiles, eff), dim3(512), 0, s, b, kt_per);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || eff == 1 || fused || a.sk > 0) return e;
  const long long groups = static_cast<long long>(b.M) * (b.N / 8);
  const int g = static_cast<int>(std::min<long long>((groups + 255) / 256, 8192));
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(g), dim3(256), 0, s, b);
  return hipGetLastError();
}

}  // namespace

// One launcher per tile shape, defined in conv_tile_<BM>x<BN>.hip.
hipError_t launch_tile_128x128(const ConvArgs& a, hipStream_t s, int variant);
hipError_t launch_tile_128x64(const ConvArgs& a, hipStream_t s, int variant);
hipError_t launch_tile_64x128(const ConvArgs& a, hipStream_t s, int variant);
hipError_t launch_tile_64x64(const ConvArgs& a, hipStream_t s, int variant);
// conv_tile_wide.hip: variant 7 (256-row, 8-wave tiles)
hipError_t launch_tile_wide(const ConvArgs& a, hipStream_t s, int tile);
// conv_skinny.hip: variant 8 (<= 32 dense rows, 16 channels per block, K split over 8 waves)
hipError_t launch_tile_skinny(const ConvArgs& a, hipStream_t s, int tile);
// conv_quad.hip: variant 9 (four 8x8 sub-tiles x 64 channels per block, 3x3 only)
hipError_t launch_tile_quad(const ConvArgs& a, hipStream_t s, int tile);

}  // namespace igemm
}  // namespace kern
}  // namespace die
