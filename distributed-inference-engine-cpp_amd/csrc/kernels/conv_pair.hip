// Back-to-back 1x1 GEMM pair (ResNet-v2 bottleneck boundary) in one launch, gfx950 MFMA.
//
// In a pre-activation bottleneck the expand conv of unit u (+ shortcut) produces x_{u+1}, whose
// BN+ReLU a_{u+1} is the input of unit u+1's reduce conv.  Two launches write a_{u+1} ([M][N1],
// 4 bytes per value in fp32 mode) and read it back: at batch 20 in stage 1 that is 64 MB each way,
// and the expand conv ran at the HBM roofline for it (profiles/r3_pmc_resnet50_fp32_b20.md rows
// 5/8/11).  Here one block owns BM = 64 pixel rows and walks N1 in 64-channel chunks:
//   1. expand chunk: acc1[64 px][64 ch] = Y · W1c  (Y = the block's [64][K1] input, staged once)
//   2. epilogue from registers: + bias1 + residual -> x_{u+1} (16-byte stores),
//      a = act2(v * s2 + h2) -> bf16 (split: hi/lo) straight into an LDS K-step tile
//   3. reduce: acc2[64 px][N2] += A · W2[:, chunk]   (one 64-wide K-step per chunk)
// and finally stores act(acc2 + bias2).  a_{u+1} never leaves the CU.
//
// The GEMMs run transposed (A operand = weights [N][K], B = pixels [M][K]) on
// v_mfma_f32_16x16x32_bf16, so a lane's accumulator holds 4 consecutive output channels of one
// pixel.  The weight rows of every 32-row block are permuted on the host (pair_permute_row) so the
// two fragments of a wave's 32 channels give each lane 8 CONSECUTIVE channels: the residual loads,
// x_{u+1} stores, the LDS writes of `a` and the output stores are all 16-byte vectors, with no
// LDS staging pass and no extra barrier.
//
// Operands reach LDS by LDS-DMA (global_load_lds_dwordx4, rows of 128 B with the (row>>1)&7 chunk
// swizzle applied on the per-lane source address, as in conv_igemm_impl.h).  The next chunk's W1
// slice is DMA'd during this chunk's reduce MFMAs and its W2 slice during the next expand, with one
// counted `s_waitcnt vmcnt` per chunk.  (Measured and dropped: a double-buffered W2 slice with the
// residual prefetched a chunk ahead -- equal at batch 20, 4-8 % slower at 32: gpurun_out/r4_pair2.)  Split (fp32) mode: every operand is a hi/lo plane pair, three MFMAs per
// fragment pair (hi*hi + lo*hi + hi*lo), as everywhere else in the engine (common.h).
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

constexpr int BM = 64;  // pixel rows per block
constexpr int BK = 64;  // K-step (one LDS row = 128 bytes)
int g_pair_shared_w = -2;  // set_pair_shared_w (host side, read at launch)

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void glds16(const uint16_t* g, uint16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

__device__ __forceinline__ void mfma3(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                      const bf16x8& bl, bool split) {
  if (split) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// K1: expand input channels; N2: reduce output channels.  256 threads = 4 waves in a 2 x 2 grid
// (wm: 32-pixel half, wn: 32-channel half of a 64-channel expand chunk / N2/2 reduce channels).
// WS (PairArgs::shared_w): the W1 chunk and the W2 slice share one LDS buffer, loaded in turn --
// W2 slice ci during the epilogue of chunk ci, W1 chunk ci+1 during the next chunk's residual
// load -- so a block needs less LDS and two blocks fit a CU; the x / a stores then move behind the
// barrier that publishes the A tile (a counted wait for the W2 slice must not also wait for them).
template <int K1, int N2, bool SPLIT, bool WS = false>
__global__ __launch_bounds__(256) void conv_pair_kernel(const PairArgs p) {
  constexpr int NP = SPLIT ? 2 : 1;
  constexpr int KS1 = K1 / BK;                 // K-steps of the expand GEMM
  constexpr int PL = BM * BK;                  // elements of one [64][64] plane tile
  constexpr int Y_EL = KS1 * NP * PL;          // [KS1][NP][64 px][64]
  constexpr int W1_EL = KS1 * NP * PL;         // [KS1][NP][64 ch][64]
  constexpr int W2_EL = NP * N2 * BK;          // [NP][N2][64]
  constexpr int A_EL = NP * PL;                // [NP][64 px][64]
  constexpr int GW2 = NP * (N2 / 8) / 4;      // W2 DMA instructions per wave
  constexpr int NF2 = N2 / 32;                 // reduce fragments (16 channels) per wave
  constexpr int W_EL = WS ? (W1_EL > W2_EL ? W1_EL : W2_EL) : W1_EL + W2_EL;
  __shared__ __attribute__((aligned(16))) uint16_t lds[Y_EL + W_EL + A_EL];
  uint16_t* const Ys = lds;
  uint16_t* const W1s = lds + Y_EL;
  uint16_t* const W2s = WS ? W1s : W1s + W1_EL;
  uint16_t* const As = W1s + W_EL;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int l16 = lane & 15, g = lane >> 4;
  const int Ml = p.live ? min(p.M, static_cast<int>(*p.live) * p.rows_per_sample) : p.M;
  const int m0 = blockIdx.x * BM;
  if (m0 >= Ml) return;  // whole block, before any barrier
  const long long xplane = static_cast<long long>(p.M) * K1;
  const long long rplane = static_cast<long long>(p.M) * p.N1;
  const long long oplane = static_cast<long long>(p.M) * N2;
  const int NC = p.N1 / BK;

  // ---- DMA sources: instruction i of this wave fills rows (wave + 4i) * 8 .. +7 of a 64-row tile
  // (N2-row tile for W2); lane L -> row +L/8, physical chunk L%8 = logical chunk ^ ((row>>1)&7).
  auto lrow = [&](int i) { return (wave + 4 * i) * 8 + (lane >> 3); };
  auto lchunk = [&](int r) { return (lane & 7) ^ ((r >> 1) & 7); };

  auto issue_y = [&]() {
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int i = 0; i < BM / 32; ++i) {
        const int r = lrow(i), m = m0 + r;
        const uint16_t* src = m < p.M ? p.x + static_cast<size_t>(m) * K1 + ks * BK + lchunk(r) * 8 : p.zeros;
        uint16_t* dst = Ys + ks * NP * PL + (wave + 4 * i) * 8 * BK;
        glds16(src, dst);
        if constexpr (SPLIT) glds16(m < p.M ? src + xplane : p.zeros, dst + PL);
      }
  };
  auto issue_w1 = [&](int ci) {
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int i = 0; i < BM / 32; ++i) {
        const int r = lrow(i);
        const uint16_t* src = p.w1 + static_cast<size_t>(ci * BK + r) * K1 + ks * BK + lchunk(r) * 8;
        uint16_t* dst = W1s + ks * NP * PL + (wave + 4 * i) * 8 * BK;
        glds16(src, dst);
        if constexpr (SPLIT) glds16(src + p.wplane1, dst + PL);
      }
  };
  auto issue_w2 = [&](int ci) {
#pragma unroll
    for (int i = 0; i < N2 / 32; ++i) {
      const int r = lrow(i);
      const uint16_t* src = p.w2 + static_cast<size_t>(r) * p.N1 + ci * BK + lchunk(r) * 8;
      uint16_t* dst = W2s + (wave + 4 * i) * 8 * BK;
      glds16(src, dst);
      if constexpr (SPLIT) glds16(src + p.wplane2, dst + N2 * BK);
    }
  };

  // this lane's two pixels (fragments j = 0, 1) and 8-channel group within a 32-channel block
  int pix[2];
  bool pv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    pix[j] = m0 + wm * 32 + j * 16 + l16;
    pv[j] = pix[j] < p.M;
  }
  const int cg = wn * 32 + 8 * g;  // channel offset within a 64-channel chunk

  f32x4 acc2[NF2][2];
#pragma unroll
  for (int i = 0; i < NF2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // residual of a chunk (clamped rows keep the instruction count wave-uniform)
  uint4 rr[2][NP];
  auto load_res = [&](int ci) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const size_t o = static_cast<size_t>(pv[j] ? pix[j] : p.M - 1) * p.N1 + ci * BK + cg;
      rr[j][0] = *reinterpret_cast<const uint4*>(p.res + o);
      if constexpr (SPLIT) rr[j][1] = *reinterpret_cast<const uint4*>(p.res + rplane + o);
    }
  };

  // Issue order per chunk ci (vector-memory ops of this wave, oldest first): after B1 of ci-1: W1
  // slice ci | after B2 of ci-1: W2 slice ci | top of ci: residual ci.  So "W1 slice ci landed" at
  // the top = at most (W2 slice + residual) younger operations outstanding; the x stores of ci-1
  // are older still.  W2 slice ci has landed once the epilogue's wait for the residual (younger)
  // returns, before B1.  (Empty asm statements with a memory clobber pin the issue order.)
  // The reduce epilogue's bias, loaded once up front (loaded at the end, its wait also drained the
  // last chunk's x / a stores: vmcnt counts loads and stores in issue order).
  // (without WS only: with WS the registers are at the 2-waves-per-SIMD limit)
  float bb2[NF2 / 2][8];
  auto load_bias2 = [&](int q) {
    const int n = wn * (N2 / 2) + q * 32 + 8 * g;
    const float4 b0 = *reinterpret_cast<const float4*>(p.bias2 + n);
    const float4 b1 = *reinterpret_cast<const float4*>(p.bias2 + n + 4);
    bb2[q][0] = b0.x, bb2[q][1] = b0.y, bb2[q][2] = b0.z, bb2[q][3] = b0.w;
    bb2[q][4] = b1.x, bb2[q][5] = b1.y, bb2[q][6] = b1.z, bb2[q][7] = b1.w;
  };
  if constexpr (!WS) {
#pragma unroll
    for (int q = 0; q < NF2 / 2; ++q) load_bias2(q);
  }
  issue_y();
  issue_w1(0);
  if constexpr (!WS) issue_w2(0);
  for (int ci = 0; ci < NC; ++ci) {
    asm volatile("" ::: "memory");
    load_res(ci);
    // Chunk ci's expand-epilogue parameters.  Loaded in the epilogue (after issue_w2), their wait
    // also waited for the W2 slice issued just before them, vmcnt counting in issue order.  Without
    // WS they ride with the residual (6 loads, the youngest); with WS (whose registers are at the
    // 2-waves-per-SIMD limit during the expand MFMAs) they are issued after the expand, before the
    // W2 slice.
    const int c0 = ci * BK + cg;  // this lane's 8 logical channels
    float4 b0, b1, s0, s1, h0, h1;
    auto load_par = [&]() {
      b0 = *reinterpret_cast<const float4*>(p.bias1 + c0);
      b1 = *reinterpret_cast<const float4*>(p.bias1 + c0 + 4);
      s0 = *reinterpret_cast<const float4*>(p.scale2 + c0);
      s1 = *reinterpret_cast<const float4*>(p.scale2 + c0 + 4);
      h0 = *reinterpret_cast<const float4*>(p.shift2 + c0);
      h1 = *reinterpret_cast<const float4*>(p.shift2 + c0 + 4);
    };
    if constexpr (!WS) load_par();
    asm volatile("" ::: "memory");
    // outstanding after the wait: the residual (and, without WS, the parameters and the W2 slice
    // issued before them)
    wait_vmcnt<(WS ? 0 : GW2 + 6) + 2 * NP>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    // ---- 1. expand chunk ----
    f32x4 acc1[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = s * 4 + g;
        bf16x8 af[NP][2], bf[NP][2];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            af[pl][i] = *reinterpret_cast<const bf16x8*>(W1s + (ks * NP + pl) * PL + swz(wn * 32 + i * 16 + l16, ch));
            bf[pl][i] = *reinterpret_cast<const bf16x8*>(Ys + (ks * NP + pl) * PL + swz(wm * 32 + i * 16 + l16, ch));
          }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) mfma3(acc1[i][j], af[0][i], af[NP - 1][i], bf[0][j], bf[NP - 1][j], SPLIT);
      }

    if constexpr (WS) {
      __syncthreads();  // every wave done with the W1 chunk: the buffer takes the W2 slice
      load_par();
      asm volatile("" ::: "memory");
      issue_w2(ci);
      asm volatile("" ::: "memory");
      wait_vmcnt<GW2>();  // the residual (issued before the W2 slice) has landed
    }

    // ---- 2. epilogue: x_{u+1} and the pre-activation tile ----
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float hh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float vv[WS ? 2 : 1][8], uu[WS ? 2 : 1][8];  // WS: x_{u+1} and a of both pixels, stored after the barrier
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float* const v = vv[WS ? j : 0];
      float r[8];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[t] = acc1[0][j][t];
        v[t + 4] = acc1[1][j][t];
      }
      unpack8(rr[j][0], r);
      if constexpr (SPLIT) {
        float rl[8];
        unpack8(rr[j][1], rl);
#pragma unroll
        for (int t = 0; t < 8; ++t) r[t] += rl[t];
      }
      // x_{u+1} = v rounded exactly as the expand conv's epilogue rounds it: (acc + bias) + (hi + lo)
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = (v[t] + bb[t]) + r[t];
      if (!WS && p.xout && pv[j]) store8v(p.xout + static_cast<size_t>(pix[j]) * p.N1 + c0, rplane, SPLIT, v);
      float* const u = uu[WS ? j : 0];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        u[t] = v[t] * ss[t] + hh[t];
        if (p.relu2) u[t] = fmaxf(u[t], 0.f);
      }
      if (!WS && p.aout && pv[j]) store8v(p.aout + static_cast<size_t>(pix[j]) * p.N1 + c0, rplane, SPLIT, u);
      const int row = wm * 32 + j * 16 + l16;
      uint4 hi, lo;
      if constexpr (SPLIT) {
        split8(u, hi, lo);
        *reinterpret_cast<uint4*>(As + PL + swz(row, cg >> 3)) = lo;
      } else {
        hi = make_uint4(pack2(u[0], u[1]), pack2(u[2], u[3]), pack2(u[4], u[5]), pack2(u[6], u[7]));
      }
      *reinterpret_cast<uint4*>(As + swz(row, cg >> 3)) = hi;
    }
    if constexpr (WS) {
      wait_vmcnt<0>();  // the W2 slice has landed (no stores issued since it)
      __syncthreads();  // A tile and W2 slice visible to every wave
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (p.xout && pv[j]) store8v(p.xout + static_cast<size_t>(pix[j]) * p.N1 + c0, rplane, SPLIT, vv[WS ? j : 0]);
        if (p.aout && pv[j]) store8v(p.aout + static_cast<size_t>(pix[j]) * p.N1 + c0, rplane, SPLIT, uu[WS ? j : 0]);
      }
    } else {
      __syncthreads();  // A tile visible; every wave done with W1 slice ci (and W2 slice ci landed)
      if (ci + 1 < NC) issue_w1(ci + 1);
    }

    // ---- 3. reduce: one K-step ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + g;
      bf16x8 af[NP][NF2], bf[NP][2];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
#pragma unroll
        for (int i = 0; i < NF2; ++i)
          af[pl][i] = *reinterpret_cast<const bf16x8*>(W2s + pl * N2 * BK + swz(wn * (N2 / 2) + i * 16 + l16, ch));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[pl][j] = *reinterpret_cast<const bf16x8*>(As + pl * PL + swz(wm * 32 + j * 16 + l16, ch));
      }
#pragma unroll
      for (int i = 0; i < NF2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma3(acc2[i][j], af[0][i], af[NP - 1][i], bf[0][j], bf[NP - 1][j], SPLIT);
    }
    __syncthreads();  // every wave done with W2 slice ci and the A tile
    if constexpr (WS) {
      if (ci + 1 < NC) issue_w1(ci + 1);
    } else {
      if (ci + 1 < NC) issue_w2(ci + 1);
    }
  }

  // ---- reduce epilogue: + bias2, act, 16-byte stores of 8 consecutive channels ----
#pragma unroll
  for (int q = 0; q < NF2 / 2; ++q) {
    const int n = wn * (N2 / 2) + q * 32 + 8 * g;
    if constexpr (WS) load_bias2(q);
    const float* bb = bb2[q];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!pv[j]) continue;
      float v[8];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[t] = acc2[2 * q][j][t] + bb[t];
        v[t + 4] = acc2[2 * q + 1][j][t] + bb[t + 4];
      }
      if (p.relu) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = fmaxf(v[t], 0.f);
      }
      store8v(p.out + static_cast<size_t>(pix[j]) * N2 + n, oplane, SPLIT, v);
    }
  }
}

// LDS bytes of one block (bf16 elements: Y + W1 chunk + W2 slice + A tile, or Y + shared W + A)
template <int K1, int N2>
constexpr int pair_lds_bytes(bool split, bool ws) {
  const int np = split ? 2 : 1, w1 = (K1 / BK) * np * BM * BK, w2 = np * N2 * BK;
  return 2 * ((K1 / BK) * np * BM * BK + (ws ? (w1 > w2 ? w1 : w2) : w1 + w2) + np * BM * BK);
}

template <int K1, int N2>
void launch_pair(const PairArgs& a, hipStream_t s) {
  const int blocks = (a.M + BM - 1) / BM;
  const dim3 grid(blocks);
  // shared W: only where it turns one block per CU into two (160 KiB of LDS per CU) and the grid
  // needs more than one block per CU (256 CUs) -- below that the overlapped W loads are faster
  constexpr int kCuLds = 160 * 1024, kCus = 256;
  const bool helps = pair_lds_bytes<K1, N2>(a.split, false) > kCuLds / 2 && pair_lds_bytes<K1, N2>(a.split, true) <= kCuLds / 2;
  const int mode = g_pair_shared_w >= -1 ? g_pair_shared_w : a.shared_w;
  const bool ws = mode == 1 || (mode < 0 && helps && blocks > kCus);
  if (a.split) {
    if (ws) hipLaunchKernelGGL((conv_pair_kernel<K1, N2, true, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_pair_kernel<K1, N2, true>), grid, dim3(256), 0, s, a);
  } else {
    if (ws) hipLaunchKernelGGL((conv_pair_kernel<K1, N2, false, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_pair_kernel<K1, N2, false>), grid, dim3(256), 0, s, a);
  }
}

}  // namespace

void set_pair_shared_w(int v) { g_pair_shared_w = v; }

// N2 = 256 (the stage-2 -> stage-3 boundary of ResNet-v2): the W2 slice is 64 KiB in split mode,
// 144 KiB of LDS in all at K1 = 128.
bool conv_pair_supported(int K1, int N1, int N2) {
  return (K1 == 64 || K1 == 128) && (N2 == 64 || N2 == 128 || N2 == 256) && N1 % BK == 0 && N1 >= BK;
}

hipError_t conv_pair(const PairArgs& a, hipStream_t s) {
  if (!conv_pair_supported(a.K1, a.N1, a.N2) || a.M <= 0) return hipErrorInvalidValue;
  if (!a.x || !a.w1 || !a.bias1 || !a.res || !a.scale2 || !a.shift2 || !a.w2 || !a.bias2 || !a.out || !a.zeros)
    return hipErrorInvalidValue;
  if (a.split && (a.wplane1 <= 0 || a.wplane2 <= 0)) return hipErrorInvalidValue;
  if (a.live && a.rows_per_sample <= 0) return hipErrorInvalidValue;
  if (a.K1 == 64) {
    if (a.N2 == 64) launch_pair<64, 64>(a, s);
    else if (a.N2 == 128) launch_pair<64, 128>(a, s);
    else launch_pair<64, 256>(a, s);
  } else {
    if (a.N2 == 64) launch_pair<128, 64>(a, s);
    else if (a.N2 == 128) launch_pair<128, 128>(a, s);
    else launch_pair<128, 256>(a, s);
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
