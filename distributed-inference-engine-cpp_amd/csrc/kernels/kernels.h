// Host-side launch API of the hand-written gfx950 kernels.  Every launcher is asynchronous on the
// given stream and capture-safe (no allocation, no synchronisation), so the engine can record a
// whole forward pass into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace die {
namespace kern {

// Implicit-GEMM convolution / GEMM on MFMA (bf16 in, f32 accumulate), NHWC activations.
//   out[m, n] = epilogue( sum_k X[m, k] * W[n, k] )      m = (b, oh, ow), k = (ky, kx, ci)
// W is [Npad][Kpad] bf16 (K contiguous, zero padded to the tile multiples).
// Epilogue (all optional): + bias[n]; + res[m, n]; relu; store out (bf16) or out_f32 (f32);
//   second output out2 = act2(v * scale2[n] + shift2[n])  (pre-activation BN of the next unit).
struct ConvArgs {
  const uint16_t* x = nullptr;
  const uint16_t* w = nullptr;
  int B = 1, H = 1, W = 1, Cin = 1;       // input NHWC (Cin = storage channels)
  int Ho = 1, Wo = 1, N = 1;              // output spatial and channels
  int KH = 1, KW = 1, stride = 1, pad_h = 0, pad_w = 0, dil = 1;
  int K = 1, Kpad = 64;                   // K = KH*KW*Cin
  int M = 1;                              // B*Ho*Wo
  const float* bias = nullptr;
  const uint16_t* res = nullptr;          // [M][N] bf16
  int relu = 0;
  uint16_t* out = nullptr;                // [M][N] bf16
  float* out_f32 = nullptr;               // [M][N] f32 (instead of / in addition to out)
  const float* scale2 = nullptr;
  const float* shift2 = nullptr;
  int relu2 = 0;
  uint16_t* out2 = nullptr;
  // split-K: `splits` slices of K write f32 partials to ws[split][M][N]; a second kernel sums them
  // and applies the epilogue.  splits == 1 -> epilogue fused in the GEMM kernel.
  int splits = 1;
  float* ws = nullptr;
  // optional: counters_n zero-initialised ints -> the last split block of each tile reduces the
  // partials and runs the epilogue itself (no second kernel); they return to zero after use.
  int* counters = nullptr;
  int counters_n = 0;
  // Zero page (device), >= Kpad + 64 bf16 elements: source of the LDS-DMA loads for padding pixels
  // and M-tail rows (a tail row reads a whole K row from it).
  const uint16_t* zeros = nullptr;
  // Live batch (device scalar, nullable): a hipGraph captured for a batch bucket runs the batches
  // that round up to it; only the first *live samples are real, so output tiles that hold padding
  // samples only are skipped (their rows stay undefined; every op is per-sample).
  const long long* live = nullptr;
  // Pre-activation on load (1x1 convs, K = Cin <= 2048, LDS-DMA loop): the input operand is
  // act(x * in_scale[c] + in_shift[c]) of the stored x (ResNet-v2's BN+ReLU of the unit input is
  // applied here instead of being stored a second time by the producing conv).
  const float* in_scale = nullptr;
  const float* in_shift = nullptr;
  int in_relu = 0;
  // relu == 3: Clip(clip_lo, clip_hi) (ReLU6 = Clip(0, 6)) instead of ReLU / GELU
  float clip_lo = 0.f, clip_hi = 0.f;
  // LayerNorm folded into the GEMM (rows GEMMs): x is the LayerNorm INPUT, the weights carry gamma,
  // and before the bias v = rstd[m] * (v - mean[m] * col_sum[n]); row_stats = [M][2] (mean, rstd)
  // from layernorm_rows' stats mode, col_sum[n] = sum_k of the (gamma-scaled) weight row n.
  const float* row_stats = nullptr;
  const float* col_sum = nullptr;
  // LayerNorm statistics produced by the epilogue of the GEMM that writes the LayerNorm's input (ViT:
  // the attention-out / MLP2 GEMMs with the residual add; N % 64 == 0): stats_out = [M][N/64] float2
  // (mean, M2) of every row's 64-column groups of the output.  A folded reader (fp32 mode) takes
  // row_parts (that buffer, [M][K/64]) instead of row_stats: each block fetches its rows' groups at
  // its start (in flight with the first operand loads), merges them in a fixed order (Chan et al.)
  // into mean and rstd = 1/sqrt(M2/K + ln_eps), and keeps them in LDS for the epilogue.  No
  // standalone statistics pass over the rows.
  float* stats_out = nullptr;
  const float* row_parts = nullptr;
  float ln_eps = 0.f;
  // fp32 mode (common.h "split" tensors): x, res, out and out2 are split (hi, lo) bf16 planes and w
  // holds the weights' hi plane followed by their lo plane `wplane` elements later.  The planes of
  // the activations follow from the shapes (x: B*H*W*Cin, res/out/out2: M*N; the launcher fills
  // xplane/oplane).  out_f32 and the split-K workspace stay plain fp32.
  int split = 0;
  long long wplane = 0;
  long long xplane = 0, oplane = 0;
  // Tile order of the XCD-aware block mapping (autotuned): 0 = heuristic (replicate the smaller
  // operand on every XCD), 1 = N-fastest (an XCD owns a range of pixel rows, reads all weights),
  // 2 = M-fastest (an XCD owns a range of output channels, reads all activations), 3 / 4 = N in 2 / 4
  // panels, panel-major (an XCD's range reads one panel of the weights).
  int order = 0;
  // Measurement only (tools/gemm_sweep.py --probe; gemm_wide_kernel and conv_glds_kernel): 1 = no
  // operand DMA (MFMAs on whatever the LDS holds), 2 = no MFMAs (DMA + waits + barriers only).  The
  // outputs are garbage; the engine never sets it.
  int probe = 0;
  // Tail split-K (LDS-DMA loops, fused split-K only): with T output tiles, the first T - T % tail
  // tiles run whole (no split-K, direct epilogue) and only the last partial round's tiles are cut
  // into `splits` K-slices, reduced in-kernel.  A grid of 257-300 tiles then costs one round plus
  // a sliver instead of two rounds on the busiest CUs (tail = 256: one tile per CU per round).  0 =
  // uniform split-K.
  int tail = 0;
  // Stream-K (LDS-DMA loops, variants 1-5; needs counters >= tiles and ws >= streamk_workspace_bytes):
  // sk = P > 0 launches exactly P blocks that split the T x K-steps iterations of all tiles evenly
  // (P = 256: one block per CU) instead of one block per (tile, split) -- a grid of 296 tiles then
  // costs 1.16 tiles per CU, not two on the busiest CUs.  Cut tiles are reduced in-kernel by their
  // last arriving contributor, in block order (bitwise repeatable for a given P).
  int sk = 0;
};

// Split-K workspace of a stream-K launch (ConvArgs::sk = P blocks, BM x BN tiles): two partial
// slabs per block.
inline size_t streamk_workspace_bytes(int P, int bm, int bn) { return static_cast<size_t>(P) * 2 * bm * bn * sizeof(float); }

// A launch config = tile + NUM_TILES * variant; variant 0 = register-staged main loop (any shape),
// 1..4 = LDS-DMA ring of 2, 3, 4, 6 stages (variants 1-4: 1x1 with K % 64 == 0, or Cin % 64 == 0;
// 6 stages only where they fit the LDS; they return hipErrorInvalidValue otherwise so a tuner can
// skip them).  The deep rings keep more K-steps in flight for the latency-bound small-M layers.
// Variant 5 = the LDS-DMA loop with ONE stage (no ring): for K <= 64 layers, where the smaller LDS
// footprint fits more blocks per CU.  Variant 6 = spatially tiled 3x3/s1/p1 kernel (8x8 pixels x 64
// channels per block, input patch staged once per 64-channel slice; 64x64 tile config only).
// Variant 7 = the 8-wave wide-tile GEMM (fp32 dense rows only): tile 0 -> 256 pixels x 128 channels
// (conv_igemm_impl.h gemm_wide_kernel); the other tiles of variant 7 are not instantiated.
// Variant 8 = the skinny dense GEMM (<= 32 rows, e.g. a classifier head at the serving batch):
// tile 0 only (conv_skinny.hip), 16 channels per block, K split over 8 waves, no split-K.
// Variant 9 = the four-tile 3x3 kernel (conv_quad.hip): four 8x8 sub-tiles x 64 channels per block,
// one sub-tile per wave, the tap's weights loaded once for 256 pixels (3x3/s1/p1, Cin % 64 == 0;
// tile 3 only, cfg 39).
enum TileCfg { TILE_128x128 = 0, TILE_128x64 = 1, TILE_64x128 = 2, TILE_64x64 = 3, NUM_TILES = 4, NUM_CFGS = 40 };
// BM (pixels) x BN (channels) of a config.
void tile_dims(int cfg, int& bm, int& bn);
// Heuristic (tile, splits) choice for a problem shape (used when not autotuned).
int choose_tile(int M, int N, int K);
int choose_splits(int M, int N, int K, int tile_cfg);
// Bytes of split-K workspace a launch needs.
size_t splitk_workspace_bytes(int M, int N, int splits);
// Launch (vectorisation picked from Cin: 8 channels per 16-B load when Cin % 8 == 0, else 4).
// Returns hipSuccess or hipErrorInvalidValue for an unsupported configuration (checked on the host
// before any launch).
hipError_t conv_igemm(const ConvArgs& a, int tile_cfg, hipStream_t s);

// `split` (launchers below): every bf16 tensor argument is a split tensor (common.h) whose lo plane
// follows its hi plane by the tensor's element count at batch B (views: rows * pitch).
// fp32 NCHW -> (x * scale[c] + shift[c]) -> bf16 NHWC with Cp >= C channels (pad channels = 0).
hipError_t input_prep(const float* x, const float* scale, const float* shift, uint16_t* out, int B, int C, int H,
                      int W, int Cp, hipStream_t s, int split = 0);
// `live` (nullable device scalar, kernels below and ConvArgs::live): only the first *live of the B
// samples are computed; the rest of the outputs are left as they are.
// NHWC bf16 max / average pooling (C % 8 == 0).
hipError_t pool2d(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh,
                  int sw, int ph, int pw, int is_max, int count_include_pad, hipStream_t s,
                  const long long* live = nullptr, const float* scale = nullptr, const float* shift = nullptr,
                  int act = 0, int split = 0);
// [B, HW, C] bf16 -> [B, C] (mean over HW), optional y = relu(x*scale+shift) before averaging;
// writes bf16 `out` and/or f32 `out_f32`.
// mode: 0 mean (GlobalAveragePool / ReduceMean), 1 sum (ReduceSum), 2 max (GlobalMaxPool / ReduceMax).
hipError_t global_avgpool(const uint16_t* x, uint16_t* out, float* out_f32, const float* scale, const float* shift,
                          int relu, int B, int HW, int C, hipStream_t s, const long long* live = nullptr,
                          int split = 0, int mode = 0);
// Global pool (mode as above) fused with the fully-connected layer that reads it (misc.hip
// gap_fc_kernel): x [B, HW, C] -> out f32 [B][N] = act(pool(x) . w[n] + bias[n]); w = [>= N][Kpad]
// GEMM weights (split: lo plane at +wplane).  Partials [C/cs][B][N] f32 go through `ws` (ws_bytes),
// one counter per group of 128 classes (counters_n available, left at 0).  gap_fc_slice: the
// channel slice the launcher uses for this shape (0 = unsupported: C % 8, workspace too small).
int gap_fc_slice(int C, int B, int N, size_t ws_bytes);
void set_gap_fc_stop(int v);  // measurement only (tools/gap_fc_bench.py): phase at which blocks return
constexpr size_t kSplitKWorkspaceBytes = size_t(64) << 20;  // the engine's split-K / GAP_FC workspace
hipError_t gap_fc(const uint16_t* x, int B, int HW, int C, int mode, const uint16_t* w, long long wplane, int Kpad,
                  const float* bias, int N, int act, float* out, float* ws, size_t ws_bytes, int* counters,
                  int counters_n, hipStream_t s, const long long* live = nullptr, int split = 0);
// Elementwise over [M][C] bf16: y = act(x * scale[c] + shift[c] (+ z))   (scale/shift/z optional;
// act 1 = ReLU, 3 = Clip(clip_lo, clip_hi))
hipError_t affine_act(const uint16_t* x, const uint16_t* z, const float* scale, const float* shift, int act,
                      uint16_t* y, long long M, int C, hipStream_t s, const long long* live = nullptr,
                      long long rows_per_sample = 0, int split = 0, float clip_lo = 0.f, float clip_hi = 0.f);

// Grouped / depthwise convolution, NHWC, fp32 weights [Cout][KH][KW][Cin/groups] (gconv.hip).
struct GConvArgs {
  const uint16_t* x = nullptr;
  const float* w = nullptr;
  const float* bias = nullptr;
  const uint16_t* res = nullptr;  // added after the activation (inverted-residual blocks)
  uint16_t* out = nullptr;
  float* out_f32 = nullptr;
  int B = 1, H = 1, W = 1, Cin = 1, Ho = 1, Wo = 1, Cout = 8, groups = 1;
  int KH = 1, KW = 1, stride = 1, pad_h = 0, pad_w = 0, dil = 1;
  int act = 0;  // 0 none, 1 ReLU, 3 Clip(clip_lo, clip_hi)
  float clip_lo = 0.f, clip_hi = 0.f;
  int split = 0;
  const long long* live = nullptr;
};
hipError_t grouped_conv(const GConvArgs& a, hipStream_t s);

// Softmax over the last axis of [rows][C] (one wave per row, fp32 math); writes bf16/split `y`
// (row pitch ld) and/or f32 `y_f32` (dense [rows][C]).  ld = stored row pitch of x and y (0 = C).
hipError_t softmax_rows(const uint16_t* x, uint16_t* y, float* y_f32, long long rows, int C, hipStream_t s,
                        int split = 0, int ld = 0);

// ---- generic kernels (generic.hip): the planner's general path ----
// fp32 [R][F] -> bf16 / split rows [R][Fp] (Fp % 8 == 0, pad columns zero): rank-2/3 graph inputs.
hipError_t rows_prep(const float* x, uint16_t* y, long long R, int F, int Fp, hipStream_t s, int split = 0);
// input_prep for any channel count: fp32 NCHW -> affine -> NHWC with Cp % 8 == 0 stored channels.
hipError_t input_prep_wide(const float* x, const float* scale, const float* shift, uint16_t* out, int B, int C, int H,
                           int W, int Cp, hipStream_t s, int split = 0);
// y[r][coly + j] = x[r][colx + j], j < ncols, over R rows (concat / slice along the channel axis).
// xplane / yplane: lo-plane distances of split tensors (elements).
hipError_t copy_cols(const uint16_t* x, long long xplane, int ldx, int colx, uint16_t* y, long long yplane, int ldy,
                     int coly, long long R, int ncols, hipStream_t s, int split = 0);
// out = act(x op y) over [R][C] rows; ymode 0: y same shape; 1: y one row per sample (broadcast over
// its rows_per_sample rows).  op 0 add, 1 sub, 2 mul, 3 div, 4 max, 5 min, 6-10 x > / < / == / >= / <= y (1 or 0).
// act codes as unary_rows.
// Cl (0 = C): logical channels; the pad columns [Cl, C) are written 0, whatever the op gives for
// them (Div of two zero pads is NaN, and NaN * 0 would poison the next GEMM's every output).
hipError_t binary_rows(const uint16_t* x, const uint16_t* y, uint16_t* out, long long R, int C, long long rows_per_sample,
                       int ymode, int op, int act, float a, float b, hipStream_t s, const long long* live = nullptr,
                       int split = 0, int Cl = 0);
// y = act(x * scale[c] + shift[c]) (scale/shift nullable); act 0 none, 1 ReLU, 2 GELU (erf),
// 3 Clip(a, b), 4 sigmoid, 5 tanh, 6 leaky ReLU (slope a), 7 exp, 8 abs, 9 sqrt, 10 neg,
// 11 reciprocal, 12 log, 13 erf, 14 pow(x, a), 15 HardSigmoid(alpha a, beta b), 16 HardSwish,
// 17 softplus, 18-22 v > / < / == / >= / <= a (1 or 0), 23 Not (v == 0), 24 v != 0 (Cast to bool).
// Cl (0 = C): logical channels; pad columns [Cl, C) are written 0.
hipError_t unary_rows(const uint16_t* x, const float* scale, const float* shift, uint16_t* y, long long R, int C,
                      int act, float a, float b, hipStream_t s, const long long* live = nullptr,
                      long long rows_per_sample = 0, int split = 0, int Cl = 0);
// NHWC zero padding: y [B][Ho][Wo][C] = x [B][H][W][C] placed at (t, l), zeros around (C % 8 == 0).
// Strides sy, sx > 1 insert zeros between input pixels (ConvTranspose lowered to a stride-1 conv).
hipError_t pad_nhwc(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, int t, int l,
                    hipStream_t s, int split = 0, int sy = 1, int sx = 1);
// Batched MatMul of two row activations (kernels/bmm.hip): C[b] (M x ldc) = A[b] (M x lda, first K
// columns) * B[b] (K x ldb, first N columns); output columns [N, ldc) written 0.
hipError_t bmm_rows(const uint16_t* A, const uint16_t* Bm, uint16_t* C, int batch, int M, int N, int K, int lda, int ldb,
                    int ldc, hipStream_t s, const long long* live = nullptr, int split = 0);
// out = cond != 0 ? a : b over rows [R][C] (a / b null: the scalars av / bv); pad columns written 0.
hipError_t where_rows(const uint16_t* c, const uint16_t* a, const uint16_t* b, float av, float bv, uint16_t* out,
                      long long R, int C, hipStream_t s, const long long* live = nullptr, long long rows_per_sample = 1,
                      int split = 0, int Cl = 0);
// ONNX Resize / Upsample of an NHWC image.  coord: 0 half_pixel, 1 asymmetric, 2 align_corners,
// 3 pytorch_half_pixel, 4 tf_half_pixel_for_nn; mode 0 nearest (nearest: 0 round_prefer_floor,
// 1 round_prefer_ceil, 2 floor, 3 ceil), 1 linear.  scale_*: output / input (the op's scales).
hipError_t resize_nhwc(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, float scale_h,
                       float scale_w, int coord, int mode, int nearest, hipStream_t s, const long long* live = nullptr,
                       int split = 0);
// f32 [R][C] from bf16 / split rows of pitch ld >= C (graph outputs with padded columns).
hipError_t rows_to_f32(const uint16_t* x, float* y, long long R, int C, int ld, hipStream_t s, int split = 0);
// f32 NCHW [B][C][H][W] from bf16 NHWC with Cs >= C stored channels.
hipError_t nhwc_to_nchw_f32_strided(const uint16_t* x, float* y, int B, int H, int W, int C, int Cs, hipStream_t s,
                                    int split = 0);
// bf16 NHWC [B,H,W,C] -> f32 NCHW [B,C,H,W]
hipError_t nhwc_to_nchw_f32(const uint16_t* x, float* y, int B, int H, int W, int C, hipStream_t s, int split = 0);
// f32 -> bf16 / bf16 -> f32 copies
hipError_t f32_to_bf16(const float* x, uint16_t* y, long long n, hipStream_t s);
hipError_t bf16_to_f32(const uint16_t* x, float* y, long long n, hipStream_t s, int split = 0);

// Back-to-back 1x1 GEMM pair of a ResNet-v2 bottleneck boundary (conv_pair.hip), one launch:
//   v   = x · W1ᵀ + bias1 + res                 (unit u's expand conv + shortcut; [M][N1])
//   xout = v                                    (the raw sum: unit u+1's residual; optional)
//   a   = act2(v * scale2 + shift2)             (unit u+1's pre-activation BN+ReLU; never stored)
//   out = act(a · W2ᵀ + bias2)                  (unit u+1's reduce conv; [M][N2])
// `a` is produced 64 channels at a time in LDS and consumed there as one K-step of the second
// GEMM, so the [M][N1] pre-activation tensor never goes to memory.  Weights [N][K] bf16 (split:
// hi plane then lo plane, w*plane elements apart) with the rows of every 32-row block PERMUTED
// (pair_permute_row): each lane's two accumulator fragments then hold 8 consecutive channels,
// stored as 16-byte vectors without an LDS staging pass.  K1 in {64, 128}, N2 in {64, 128},
// N1 % 64 == 0, rows of x/res/xout/out dense (ld = K1 / N1 / N1 / N2).
struct PairArgs {
  const uint16_t* x = nullptr;
  const uint16_t* w1 = nullptr;
  const float* bias1 = nullptr;
  const uint16_t* res = nullptr;
  uint16_t* xout = nullptr;
  // the pre-activation a = act2(x * scale2 + shift2) [M][N1], stored too when other ops read it
  // (a stage boundary whose projection shortcut also reads a); nullptr: a stays in LDS only
  uint16_t* aout = nullptr;
  const float* scale2 = nullptr;
  const float* shift2 = nullptr;
  int relu2 = 1;
  const uint16_t* w2 = nullptr;
  const float* bias2 = nullptr;
  int relu = 1;
  uint16_t* out = nullptr;
  int M = 0, K1 = 64, N1 = 256, N2 = 64;
  int rows_per_sample = 1;            // for `live`
  const long long* live = nullptr;
  const uint16_t* zeros = nullptr;    // zero page >= K1 + 64 elements (M-tail rows)
  int split = 0;
  long long wplane1 = 0, wplane2 = 0;
  // One LDS buffer for the W1 chunk and the W2 slice (used in turn, not overlapped): 80 KiB per
  // block instead of 112 / 96 at K1 = 128 in fp32, so two blocks share a CU.  -1 = when the grid
  // exceeds one block per CU (M / 64 > 256, e.g. stage 2 above batch 20), 0 = never, 1 = always.
  int shared_w = -1;
};
// Physical row of logical output channel n in a pair weight matrix (a permutation inside each
// block of 32 rows; the inverse maps physical -> logical).
inline int pair_permute_row(int n) {
  const int b = n & ~31, r = n & 31;  // logical r = 8g + 4h + t  ->  physical 16h + 4g + t
  const int g = r >> 3, h = (r >> 2) & 1, t = r & 3;
  return b + 16 * h + 4 * g + t;
}
bool conv_pair_supported(int K1, int N1, int N2);
// Measurement switch (process-wide, read at launch): >= -1 overrides every launch's
// PairArgs::shared_w (-1 auto, 0 never, 1 always); -2 (default) leaves it to the caller.
void set_pair_shared_w(int v);
hipError_t conv_pair(const PairArgs& a, hipStream_t s);

// 7x7 / stride 2 / pad 3 conv, 4 input channels (NHWC, 3 real + 1 zero), 64 output channels:
// w = [64][224] bf16 with k = ky*32 + kx*4 + c (kx padded to 8), out = act(conv + bias) NHWC bf16.
// split: x/out are split tensors and w holds the hi plane [64][224] followed by the lo plane.
hipError_t conv_stem7x7(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* out, int B, int H, int W,
                        int Ho, int Wo, int relu, hipStream_t s, const long long* live = nullptr, int split = 0);
// Persistent stem that reads the graph input directly: x fp32 NCHW [B][C][H][W], C <= 4, with the
// input's pending per-channel affine (in_scale/in_shift, nullable) applied on load -- replaces
// input_prep + conv_stem7x7.  max_blocks <= 0: two blocks per CU.
// Stem 7x7/2 (NCHW fp32 input, fused input BN) + 3x3/2 pad-1 max pool + per-channel affine (+ ReLU if
// pact == 1) of the pooled value, one kernel (stem.hip).  Weight rows permuted by pair_permute_row;
// bias / pscale / pshift in logical channel order.  out: [B][Hp][Wp][64].
bool stem_pool_supported(int H, int W, int Hs, int Ws, int Hp, int Wp, int split);
size_t stem_pool_lds_bytes(int Ws, int split);
hipError_t conv_stem_pool_nchw(const float* x, int C, const float* in_scale, const float* in_shift, const uint16_t* w,
                               const float* bias, int relu, const float* pscale, const float* pshift, int pact,
                               uint16_t* out, int B, int H, int W, int Hs, int Ws, int Hp, int Wp, hipStream_t s,
                               const long long* live = nullptr, int split = 0, int target_blocks = 0);
hipError_t conv_stem7x7_nchw(const float* x, int C, const float* in_scale, const float* in_shift, const uint16_t* w,
                             const float* bias, uint16_t* out, int B, int H, int W, int Ho, int Wo, int relu,
                             hipStream_t s, const long long* live = nullptr, int split = 0, int max_blocks = 0);

// Evict the L2s: stream-read `bytes` (> 8 x 4 MiB) of a scratch buffer (autotuning in the cache
// state a layer sees inside a forward: L2 cold, Infinity Cache warm).
hipError_t l2_scrub(const void* buf, size_t bytes, float* sink, hipStream_t s);

// dst[0..n) = src[0..n) in one small block (src may be host-coherent pinned memory).
hipError_t copy_i64(const long long* src, long long* dst, int n, hipStream_t s);

// ---- device JSON decode (decode.hip) ----
// Sample b's number-list text lives at text + offs[b] (offs == nullptr: text + b * text_cap;
// text_cap % 4096 == 0) with lens[b] <= text_cap bytes (-1 = not a text sample: skipped).  Writes
// out[b][0..numel) (values, zero padded), status[b] (0 ok, bit 0 = needs host parse, 2 = more than
// numel values) and ntok[b].
size_t decode_scratch_bytes(int max_batch, size_t text_cap);
// packed/poffs (optional): sample b's lens[b] characters are 4-bit packed (core/textpack.h) at
// packed + poffs[b] (8-byte aligned, in a slot of text_cap / 2 bytes) and expanded in registers as
// the decode kernels load them; poffs[b] < 0 (or packed == nullptr) reads raw text at text + offs[b].
// Measurement switch (process-wide): 0 = packed launches decode on the symbol (nibble) kernels
// (default), 1 = the character kernels for every launch (the round-4 path).
void set_decode_variant(int v);
hipError_t decode_json_numbers(const unsigned char* text, const long long* offs, size_t text_cap,
                               const long long* lens, int B, float* out, long long numel, int* status, int* ntok,
                               void* scratch, hipStream_t s, const unsigned char* packed = nullptr,
                               const long long* poffs = nullptr);

// ---- transformer (transformer.hip) ----
// LayerNorm over the last dim of bf16 rows [rows][C] (C % 8 == 0: the stored pitch), fp32
// statistics over the first Cl columns (0 = C; pad columns written 0); any C (> 2048: a block per row).
// true when the streaming attention kernel is built in (any sequence length; else S <= 256)
// Streaming attention variant (measurement switch, process-wide): 0 = K/V staged one tile ahead
// (default), 1 = two tiles ahead, 2 = 0 with the natural (not XCD-aware) block mapping, 3 = 0 with
// contiguous pair ranges per XCD.
void set_attention_variant(int v);
bool attention_any_length();
// Head dim / sequence length the attention launcher takes (streaming kernel: head dim 32, 64, 80,
// 96 or 128, any length; the whole-K/V kernel: 64 and <= 256 tokens).
bool attention_supported(int D, int S);
// variant (measurement): 0 = the default choice, 1 = 16 lanes x 6 chunks per row (C <= 768: 4 rows
// per wave, twice the loads in flight per lane), 2 = the block-per-row kernel.
// LayerNorm row order (measurement switch, process-wide, read at launch): 1 = XCD-affine (rows read
// on the XCD whose GEMM tiles wrote them), 0 (default) = natural block order -- the ViT forward A/B
// was inside the run-to-run noise (profiles/r4_attention_xcd_map.md).
void set_layernorm_xcd(int v);
// stats != nullptr: statistics mode -- (mean, rstd) of each row to stats[2 row], 2 row + 1 and y is
// not written (the normalisation is folded into the consuming GEMM: ConvArgs::row_stats).
hipError_t layernorm_rows(const uint16_t* x, uint16_t* y, const float* gamma, const float* beta, float eps,
                          long long rows, int C, hipStream_t s, int split = 0, int Cl = 0, int variant = 0,
                          float* stats = nullptr);
// out[b,0,:] = cls + pos[0]; out[b,1+s,:] = patches[b,s,:] + pos[1+s]   (cls/pos optional, f32)
// stats (nullable, C % 64 == 0): also the rows' LayerNorm statistics partials, [B*(S0+1)][C/64] float2
// (mean, M2) as ConvArgs::stats_out writes them
hipError_t tokens_assemble(const uint16_t* patches, const float* cls, const float* pos, uint16_t* out, int B, int S0,
                           int C, hipStream_t s, int split = 0, float* stats = nullptr);
// y[b,:] = x[b, idx, :]   (x is [B][S][C])
hipError_t gather_rows(const uint16_t* x, uint16_t* y, int B, int S, int idx, int C, hipStream_t s, int split = 0);
// Multi-head attention: out[b,s,h*D:(h+1)*D] = softmax(scale * Q_h K_h^T) V_h with Q/K/V rows
// [B*S][ld*] (head h at columns h*D).  D and S as attention_supported() takes them (split: q/k/v/out
// planes are B*S*ld of their pitch).
hipError_t attention(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* out, int B, int S, int H,
                     int D, int ldq, int ldk, int ldv, int ldo, float scale, hipStream_t s, int split = 0);

}  // namespace kern
}  // namespace die
