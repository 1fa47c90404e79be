// Implicit-GEMM convolution / GEMM for gfx950 on MFMA (v_mfma_f32_16x16x32_bf16).
//
// Replaces the Conv / FusedConv / Gemm kernels ONNX Runtime would run for the reference
// (src/inference_engine.cpp:114-121,176-183 -> [ext] ORT CUDA EP).  Design (CDNA4-first):
//  * NHWC bf16 activations, weights pre-packed as [Npad][Kpad] bf16 with k = (ky, kx, ci), so both
//    MFMA operands are K-contiguous and a BK=64 K-step of the activation tile is a plain 128-byte
//    row per output pixel (padding pixels -> zeros, predicated loads).
//  * The GEMM is computed transposed (A = weights, B = pixels): each 16x16 accumulator holds
//    4 consecutive output channels of one pixel per lane.
//  * 256-thread blocks = 4 wave64s in a 2x2 grid; BMxBN in {128,64}^2; 64-wide K-steps double-
//    buffered in LDS with the next tile's global loads issued before the MFMAs of the current one
//    (async-STAGE split) and ONE barrier per K-step.
//  * LDS rows are 128 B; the 16-byte chunk index is XOR-swizzled with (row>>1)&7, which makes the
//    ds_read_b128 fragment reads of both operands bank-conflict-free for the gfx950 b128 lane
//    groups ({0-3,12-15,20-27}, ...).
//  * Epilogue staged through LDS (f32 tile, XOR-swizzled 16-B chunks), then every thread owns 8
//    consecutive channels of one pixel: 16-byte coalesced residual loads and output stores (a wave
//    writes whole 256-B row segments).  Fused: + bias (folded BatchNorm), + residual, ReLU, bf16
//    and/or f32 store, and a second output act(v*scale2+shift2) (the next pre-activation unit's
//    BN+ReLU), which removes every standalone BatchNormalization / Relu / Add of ResNet-v2.
//  * Split-K for layers with few output tiles (late stages, the FC head): K slices write f32
//    partials with the same coalesced path; splitk_epilogue sums them and applies the epilogue.
//  * The kernels live in conv_igemm_impl.h; conv_tile_<BM>x<BN>.hip instantiate one tile shape
//    each (parallel build).  This file holds the heuristics and the dispatcher.
#include "conv_igemm_impl.h"

namespace die {
namespace kern {

constexpr int BK = 64;  // K-step (conv_igemm_impl.h)

void tile_dims(int cfg, int& bm, int& bn) {
  switch (cfg % NUM_TILES) {
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
  return TILE_128x128;  // few tiles: big tiles + split-K (choose_splits)
}

int choose_splits(int M, int N, int K, int cfg) {
  if (N % 8) return 1;
  int bm, bn;
  tile_dims(cfg, bm, bn);
  const long tiles = static_cast<long>((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int nk = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < 384 && s < 16 && nk / (2 * s) >= 4 &&
         splitk_workspace_bytes(M, N, 2 * s) <= (64u << 20))
    s *= 2;
  return s;
}

size_t splitk_workspace_bytes(int M, int N, int splits) {
  return splits > 1 ? static_cast<size_t>(splits) * M * N * sizeof(float) : 0;
}

hipError_t conv_igemm(const ConvArgs& a, int cfg, hipStream_t s) {
  if (a.Cin % 4 != 0 || a.Kpad % BK != 0 || a.K > a.Kpad) return hipErrorInvalidValue;
  if (!a.out && !a.out_f32 && !a.out2) return hipErrorInvalidValue;
  if (a.out2 && (!a.scale2 || !a.shift2)) return hipErrorInvalidValue;
  if ((a.row_stats || a.row_parts) && !a.col_sum) return hipErrorInvalidValue;
  // epilogue statistics: whole 64-column groups in one 8-lane DPP group; readers: the fp32 (split)
  // kernels' LDS-staged epilogue (the launcher also rules out the two-kernel split-K form)
  if (a.stats_out && a.N % 64 != 0) return hipErrorInvalidValue;
  if (a.row_parts && (a.row_stats || !a.split || a.N % 8 != 0 || a.K % 64 != 0)) return hipErrorInvalidValue;
  if (a.splits > 1 && (a.N % 8 != 0 || !a.ws)) return hipErrorInvalidValue;
  // tail split-K: the LDS-DMA loops (variants 1-5) with the in-kernel reduction only
  if (a.tail < 0 || (a.tail > 0 && (a.splits < 2 || !a.counters))) return hipErrorInvalidValue;
  if (cfg < 0 || cfg >= NUM_CFGS) return hipErrorInvalidValue;
  const int variant = cfg / NUM_TILES;
  if (a.tail > 0 && (variant == 0 || variant >= 6)) return hipErrorInvalidValue;
  if (a.sk < 0 || (a.sk > 0 && (variant == 0 || variant >= 6))) return hipErrorInvalidValue;  // stream-K: LDS-DMA loops
  if (variant == 7) return igemm::launch_tile_wide(a, s, cfg % NUM_TILES);
  if (variant == 8) return igemm::launch_tile_skinny(a, s, cfg % NUM_TILES);
  if (variant == 9) return igemm::launch_tile_quad(a, s, cfg % NUM_TILES);
  switch (cfg % NUM_TILES) {
    case TILE_128x128: return igemm::launch_tile_128x128(a, s, variant);
    case TILE_128x64: return igemm::launch_tile_128x64(a, s, variant);
    case TILE_64x128: return igemm::launch_tile_64x128(a, s, variant);
    default: return igemm::launch_tile_64x64(a, s, variant);
  }
}

}  // namespace kern
}  // namespace die
