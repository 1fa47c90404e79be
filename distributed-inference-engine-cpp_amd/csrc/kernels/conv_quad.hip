// Four-tile 3x3 conv: variant 9 of the conv config space (cfg 39 = tile 3 + 4 * 9), for the late
// ResNet stages at the serving batch (14x14 and 7x7 maps, 256-512 channels).
//
// Why (profiles/r6_conv3x3_quad.md): the spatial kernel (variant 6) owns an 8x8-pixel x 64-channel
// tile, so every 64 pixels re-read the whole 3x3 weight slab of their 64 output channels -- at
// B = 24 a stage-3 3x3 moves ~230 MB of weights for 5 MB of activations, and each of its four waves
// reads 8 LDS fragments for 12 MFMAs.  Here ONE block owns four 8x8 sub-tiles (a whole 14x14 image,
// or four 7x7 images) x 64 output channels; its 8 waves (two per SIMD, so one wave's LDS reads and
// waits hide under the other's MFMAs) each compute half a sub-tile (32 pixels x 64 channels):
//   * the weights of a tap (64 channels x 64 K, 16 KiB in fp32 split mode) are loaded once for 256
//     pixels instead of 64 -- 4x fewer weight bytes per output;
//   * per 32-deep K substep a wave reads 12 fragments (4 weight + 2 pixel, hi and lo) for 24 MFMAs
//     (was 8 for 12);
//   * the weights of the next two taps stream into a 3-deep ring under this tap's MFMAs (one barrier
//     per tap, counted vmcnt; the spatial kernel waited for every tap's DMA with nothing in flight --
//     a 2-deep ring measured 38.7 us on the stage-3 3x3 at B = 24, against 32.2 for the spatial
//     kernel: one tap of MFMAs (0.64 us) does not cover a loaded weight fetch).
// Patch LDS layout and swizzle are the spatial kernel's (patch_swz): sub-tile w's 10x10 input patch
// of the current 64-channel slice sits at patch + w * SUB, 128 B per pixel, and the rows a wave reads
// per fragment are the same pairs {0,1} .. {6,7} (+ dy) the swizzle tables were searched for.
// LDS: 4 x 26 KiB patches + 3 x 16 KiB weights = 152 KiB (one block per CU; split mode).  Split-K
// over channel slices with the shared fused reduction (tile_epilogue, 256-row tile, 4 waves on M).
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {
namespace {

constexpr int kQuadSub = 4;  // 8x8 sub-tiles per block

// tile row r (sub-tile r / 64, raster pixel r % 64) -> output pixel, -1 outside the image / batch
struct QuadRows {
  int st0, nst, tiles_x, tpi, Ho, Wo;
  __device__ __forceinline__ int operator()(int r) const {
    const int st = st0 + (r >> 6);
    if (st >= nst) return -1;
    const int b = st / tpi, tt = st - b * tpi;
    const int oy = (tt / tiles_x) * 8 + ((r >> 3) & 7), ox = (tt - (tt / tiles_x) * tiles_x) * 8 + (r & 7);
    return oy < Ho && ox < Wo ? (b * Ho + oy) * Wo + ox : -1;
  }
};

constexpr int kQuadThreads = 512;  // 8 waves: wave w = half (w & 1) of sub-tile w >> 1

template <bool SPLIT>
__global__ __launch_bounds__(kQuadThreads) void conv3x3_quad_kernel(const ConvArgs p, const int sl_per_split) {
  constexpr int BM = 64 * kQuadSub, BN = 64, NP = SPLIT ? 2 : 1;
  constexpr int PW = 10, NPIX = 100, PINSTR = 13;            // patch pixels; 1 KiB (8-pixel) DMA pieces
  constexpr int PPLANE = PINSTR * 8 * 64, APLANE = BN * BK;  // elements per plane
  constexpr int SUB = NP * PPLANE;                           // one sub-tile's patch (both planes)
  constexpr int PATCH = kQuadSub * SUB, WBUF = NP * APLANE;
  constexpr int EPI = BM * BN * 2;                           // f32 staging tile (bf16 elements)
  constexpr int NWB = 3;                                     // weight ring depth (taps)
  constexpr int GW = NP;                                     // weight DMA instructions per wave per tap
  constexpr int LDS_ELEMS = PATCH + NWB * WBUF > EPI + 2 ? PATCH + NWB * WBUF : EPI + 2;
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_ELEMS];
  uint16_t* const patch = lds;
  uint16_t* const wb = lds + PATCH;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = wave >> 1, half = wave & 1;
  // block -> (group of 4 sub-tiles, N-tile, channel-slice range), XCD-aware as block_coords
  const int tiles_x = (p.Wo + 7) >> 3, tiles_y = (p.Ho + 7) >> 3, tpi = tiles_x * tiles_y;
  const int Bl = p.live ? min(p.B, static_cast<int>(*p.live)) : p.B;
  const int nst = Bl * tpi;  // live sub-tiles
  const int ntm = (nst + kQuadSub - 1) / kQuadSub, ntn = (p.N + BN - 1) / BN, S = gridDim.y;
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
  const int n0 = tile_n * BN;
  const int nsl = p.Cin / BK;
  const int cs0 = split * sl_per_split, cs1 = min(nsl, cs0 + sl_per_split);

  // this wave's sub-tile: its 10x10 patch, piece I (0..12) = pixels I*8 .. I*8+7, lane -> pixel
  // I*8 + lane/8, physical chunk lane%8; the sub-tile's two waves load the even / odd pieces.
  // Offsets: elements from the tensor base (+ the swizzled chunk), -1 = zero page.
  constexpr int NPC = (PINSTR + 1) / 2;  // pieces per wave (the odd half has one fewer)
  const int st = tile_m * kQuadSub + sub;
  const bool st_ok = st < nst;
  const int sb = st_ok ? st / tpi : 0, stt = st_ok ? st - sb * tpi : 0;
  const int ty0 = (stt / tiles_x) * 8, tx0 = (stt - (stt / tiles_x) * tiles_x) * 8;
  int poff[NPC];
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int I = 2 * i + half;
    const int q = I * 8 + (lane >> 3);
    const int py = q / PW, px = q - (q / PW) * PW;
    const int iy = ty0 - 1 + py, ix = tx0 - 1 + px;
    const bool v = st_ok && q < NPIX && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    const int c = (lane & 7) ^ (q < NPIX ? patch_swz(py, px) : 0);
    poff[i] = v ? ((sb * p.H + iy) * p.W + ix) * p.Cin + c * 8 : -1;
  }
  uint16_t* const mypatch = patch + sub * SUB;
  // weight DMA source: rows wave*8 + lane/8 of this N-tile (one 1 KiB piece per plane per wave)
  const int wr = wave * 8 + (lane >> 3);
  const uint16_t* const asrc = p.w + static_cast<size_t>(n0 + wr) * p.Kpad + (((lane & 7) ^ ((wr >> 1) & 7)) * 8);
  const bool dma = p.probe != 1, mfma = p.probe != 2;  // ConvArgs::probe (measurement only)
  auto issue_w = [&](int cs, int tap, int buf) {
    if (!dma) return;
    const int k0 = tap * p.Cin + cs * BK;
    uint16_t* dst = wb + buf * WBUF + wave * 8 * BK;
    glds16(asrc + k0, dst);
    if constexpr (SPLIT) glds16(asrc + p.wplane + k0, dst + APLANE);
  };
  auto issue_patch = [&](int cs) {
    if (!dma) return;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int I = 2 * i + half;
      if (I >= PINSTR) break;  // wave-uniform
      const bool v = poff[i] >= 0;
      const uint16_t* src = v ? p.x + poff[i] + cs * BK : p.zeros;
      glds16(src, mypatch + I * 512);
      if constexpr (SPLIT) glds16(v ? src + p.xplane : p.zeros, mypatch + PPLANE + I * 512);
    }
  };

  f32x4 acc[4][2];  // [16-channel fragment][16-pixel fragment] of the wave's 32 pixels x 64 channels
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cs = cs0; cs < cs1; ++cs) {
    if (cs != cs0) __syncthreads();  // every wave done with the previous slice's patch and weights
    issue_patch(cs);
    issue_w(cs, 0, 0);
    issue_w(cs, 1, 1);
    for (int tap = 0; tap < 9; ++tap) {
      // this tap's weights (and, at tap 0, the patch) have landed for this wave -- only the next
      // tap's weights may still be in flight; the barrier makes them visible to all and retires
      // every wave's reads of the ring slot issued into next (read at tap - 1)
      if (tap < 8) wait_vmcnt<GW>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (tap < 7) issue_w(cs, tap + 2, (tap + 2) % NWB);  // two taps ahead, under this tap's MFMAs
      const uint16_t* A = wb + (tap % NWB) * WBUF;
      const int dy = tap / 3, dx = tap - dy * 3;
#pragma unroll
      for (int s = 0; s < 2 && mfma; ++s) {
        const int chunk = s * 4 + (lane >> 4);
        bf16x8 af[4], bfr[2];
        int boff[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(A + swz(i * 16 + (lane & 15), chunk));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int pix = (half * 2 + j) * 16 + (lane & 15);
          const int row = (pix >> 3) + dy, col = (pix & 7) + dx;
          boff[j] = (row * PW + col) * BK + ((chunk ^ patch_swz(row, col)) << 3);
          bfr[j] = *reinterpret_cast<const bf16x8*>(mypatch + boff[j]);
        }
        if constexpr (SPLIT) {
          bf16x8 afl[4], bfl[2];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            afl[i] = *reinterpret_cast<const bf16x8*>(A + APLANE + swz(i * 16 + (lane & 15), chunk));
#pragma unroll
          for (int j = 0; j < 2; ++j) bfl[j] = *reinterpret_cast<const bf16x8*>(mypatch + PPLANE + boff[j]);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // all operand reads done before the epilogue reuses the LDS
  tile_epilogue<BM, BN, QuadRows, kQuadThreads, 8>(p, acc, lds, 0, n0, wave, 0, lane, tid, tile, split,
                                          QuadRows{tile_m * kQuadSub, nst, tiles_x, tpi, p.Ho, p.Wo},
                                          float2{0.f, 0.f}, epi_flag_off(LDS_ELEMS, EPI));
}

}  // namespace

// cfg 39 (tile 3 + 4 * 9): 3x3 / stride 1 / pad 1, Cin % 64 == 0; split-K over 64-channel slices.
hipError_t launch_tile_quad(const ConvArgs& a, hipStream_t s, int tile) {
  if (tile != TILE_64x64) return hipErrorInvalidValue;
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.dil != 1 || a.pad_h != 1 || a.pad_w != 1 || a.H != a.Ho ||
      a.W != a.Wo || a.Cin % BK || a.K != 9 * a.Cin || a.Kpad != a.K || a.N % 8 || !a.zeros || a.in_scale ||
      a.row_stats || a.row_parts || a.stats_out || a.sk || a.tail)
    return hipErrorInvalidValue;
  if (a.split && a.wplane <= 0) return hipErrorInvalidValue;
  ConvArgs c = a;
  c.xplane = a.split ? static_cast<long long>(a.B) * a.H * a.W * a.Cin : 0;
  c.oplane = a.split ? static_cast<long long>(a.M) * a.N : 0;
  const int nsl = a.Cin / BK;
  const int sp = std::max(1, std::min(a.splits, nsl));
  const int per = (nsl + sp - 1) / sp, effs = (nsl + per - 1) / per;
  const int tpi = ((a.Ho + 7) / 8) * ((a.Wo + 7) / 8);
  const int qtiles = ((a.B * tpi + kQuadSub - 1) / kQuadSub) * ((a.N + 63) / 64);
  c.splits = effs;
  const bool fused = effs > 1 && a.counters && qtiles <= a.counters_n;
  if (!fused) c.counters = nullptr;
  if (c.split) hipLaunchKernelGGL(conv3x3_quad_kernel<true>, dim3(qtiles, effs), dim3(kQuadThreads), 0, s, c, per);
  else hipLaunchKernelGGL(conv3x3_quad_kernel<false>, dim3(qtiles, effs), dim3(kQuadThreads), 0, s, c, per);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || effs == 1 || fused) return e;
  const long long groups = static_cast<long long>(c.M) * (c.N / 8);
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(static_cast<int>(std::min<long long>((groups + 255) / 256, 8192))),
                     dim3(256), 0, s, c);
  return hipGetLastError();
}

}  // namespace igemm
}  // namespace kern
}  // namespace die
