// Lowering of an ONNX graph to a fused, NHWC/bf16 device program for gfx950.
//
// Passes (one walk over the topologically sorted nodes, with lookahead):
//  * BatchNormalization directly on the graph input -> folded into the input-prep kernel that also
//    converts NCHW fp32 -> NHWC bf16 (it cannot be folded into the stem weights exactly, because the
//    stem's zero padding is applied after the BN);
//  * Conv -> BatchNormalization -> Relu  -> one conv with folded weights/bias and ReLU epilogue;
//  * Conv -> Add(other) [-> Relu]        -> residual epilogue (other operand already computed);
//  * value -> BatchNormalization [-> Relu] consumed next to the value itself (pre-activation units)
//    -> the producing conv's second output (dual store), so ResNet-v2 has no standalone BN/ReLU/Add;
//  * Gemm / MatMul(2-D initializer) -> the same MFMA kernel as a 1x1 conv over rows;
//  * GlobalAveragePool / MaxPool / AveragePool -> NHWC kernels; Flatten of 1x1 maps -> view.
//  * transformers (ViT): the patch Conv's Reshape/Transpose, the heads Reshape/Transpose, the
//    MatMul -> Div -> Softmax -> MatMul chain and the shape-computation subgraph are all lazy views;
//    the chain materialises as one fused attention kernel when the context is merged back into rows.
//    Sibling Q/K/V MatMuls become one GEMM (N = 3*D); MatMul -> Add(bias) -> erf-GELU and
//    MatMul -> Add(bias) -> Add(residual) fold into the GEMM epilogue; cls Expand/Concat + position
//    Add -> one token-assembly kernel; LayerNormalization and Gather(token) -> row kernels.
// Anything else falls back to standalone affine/add/relu kernels, or is rejected with a clear
// error (the CPU executor still runs such models).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.h"
#include "../onnx/onnx_model.h"

namespace die {

struct PlanBuf {
  size_t bytes_per_sample = 0;  // scaled by the batch size at allocation time
  size_t offset = 0;            // arena offset (max batch), assigned by the planner
  int first_use = -1, last_use = -1;
};

struct PlanOp {
  enum Kind {
    INPUT_PREP, CONV, POOL, GAP, AFFINE, TO_NCHW_F32, BF16_TO_F32,
    LAYERNORM, TOKENS, GATHER_ROWS, ATTENTION, STEM, GCONV, SOFTMAX,
    // general path (kernels/generic.hip)
    ROWS_PREP,  // rank-2/3 graph input: f32 [rows][C] -> bf16 rows [rows][Cp]
    COPY_COLS,  // out[:, col[1] + j] = in[:, col[0] + j], j < C (concat / slice); pitches ld[0], ld[1]
    BINARY,     // out = act(in (op gidx) in2); S = 0: same shape, 1: in2 = one row per sample
    UNARY,      // out = act(in * scale + shift) with any activation code
    // ResNet-v2 bottleneck boundary in one launch (kernels/conv_pair.hip): a dual-store 1x1 expand
    // conv fused with the 1x1 reduce conv that is the sole reader of its pre-activation output
    CONV_PAIR,
    PAD,     // NHWC zero padding (ONNX Pad not folded into a conv): out [Ho][Wo] = in [H][W] at (ph, pw),
             // stride sh, sw (zero insertion: ConvTranspose lowered to a stride-1 conv)
    WHERE,   // out = in != 0 ? in2 : in3 (in2 / in3 = -1: the scalars clip_lo / clip_hi)
    RESIZE,  // NHWC Resize: in [H][W] -> out [Ho][Wo]; act = mode, gidx = coord, is_max = nearest mode,
             // clip_lo / clip_hi = scales (output / input)
    BMM,     // batched MatMul of two row activations: out [S][Cp pitch C] = in [S][gidx of ld[0]] x
             // in2 [gidx][ld[1]]; Cp = logical N
    GAP_FC   // global pool (gidx = mode) of in [H*W][C] + the 1x1 GEMM that is its only reader, in one
             // launch: out_f32 [Cp] = act(pool . w + bias); conv describes the GEMM (Kpad, wplane)
  } kind;
  std::string name;
  // buffers (-1 = none).  -2 = the graph input (f32 NCHW), -3 = the graph output (f32).
  int in = -1, in2 = -1, in3 = -1, out = -1, out2 = -1, out_f32 = -1;
  int out3 = -1;  // CONV_PAIR: the pre-activation `a` when ops other than the fused reduce conv read it
  // parameter offsets (bytes) into the device parameter blob
  size_t w_off = 0, bias_off = SIZE_MAX, s2_off = SIZE_MAX, b2_off = SIZE_MAX, scale_off = SIZE_MAX,
         shift_off = SIZE_MAX;
  // conv geometry (per sample; ConvArgs B/M are set at launch)
  kern::ConvArgs conv;
  int tile_bmax = 0;
  // generic geometry
  int C = 0, H = 0, W = 0, Ho = 0, Wo = 0, Cp = 0;
  int kh = 0, kw = 0, sh = 1, sw = 1, ph = 0, pw = 0, is_max = 0, cip = 0, act = 0;
  // stored row pitch when it differs from the logical channel count C (padded channels; 0 = C):
  // BF16_TO_F32 / TO_NCHW_F32 drop the pad columns, SOFTMAX reads and writes rows of this pitch
  int ld_store = 0;
  int groups = 1;                      // GCONV
  float clip_lo = 0.f, clip_hi = 0.f;  // act == 3 (Clip) of AFFINE / GCONV
  long long rows_per_sample = 0;  // AFFINE / LAYERNORM: rows of C per sample
  // transformer ops: sequence length, heads, head dim, column offsets / pitches of in/in2/in3
  int S = 0, nh = 0, hd = 0, gidx = 0;
  int col[3] = {0, 0, 0}, ld[3] = {0, 0, 0};
  float fscale = 1.f, eps = 0.f;
  double flops_per_sample = 0;
  // Side branch: this op may run on a second stream, concurrently with the ops after it, until
  // op `join` (its first consumer) waits for it.  The arena keeps its inputs live until `join`.
  int join = -1;
  // CONV: pre-activation on load (ConvArgs::in_scale/in_shift/in_relu), parameter offsets
  size_t in_scale_off = SIZE_MAX, in_shift_off = SIZE_MAX;
  int in_relu = 0;
  // CONV_PAIR: in = expand input [M][K1], in2 = residual, out = raw sum x (-1: not stored), out2 =
  // reduce output [M][n2]; conv/w_off/bias_off/s2_off/b2_off describe the expand conv and the BN of
  // the pre-activation, w2_off/bias2_off/w2plane/pair_relu the reduce conv.  Both weight matrices
  // have their rows permuted by kern::pair_permute_row.
  size_t w2_off = 0, bias2_off = SIZE_MAX;
  long long w2plane = 0;
  int n2 = 0, pair_relu = 0;
  // LayerNorm folded into its GEMM readers (EngineOptions::fold_layernorm): the LAYERNORM op has
  // stats_only = 1 and out = a [rows][2] f32 (mean, rstd) buffer; each reading CONV has in = the
  // LayerNorm's input, in3 = that statistics buffer, gamma folded into its weights, beta into its
  // bias and colsum_off = the per-column sums of its weights (ConvArgs::row_stats / col_sum).
  int stats_only = 0;
  size_t colsum_off = SIZE_MAX;
  // LayerNorm statistics from the producer's epilogue (stats_from_producer): the CONV that writes a
  // statistics-only LayerNorm's input also writes out_stats = the [M][N/64] (mean, M2) column-group
  // partials (ConvArgs::stats_out), the LayerNorm op is gone, and its folded readers have
  // in3 = out_stats, in3_parts = 1 (ConvArgs::row_parts) and eps = the LayerNorm's epsilon.
  int out_stats = -1;
  int in3_parts = 0;
};

struct Plan {
  std::vector<PlanOp> ops;
  std::vector<PlanBuf> bufs;
  std::vector<uint8_t> params;  // host copy of the packed device parameters
  size_t arena_bytes_per_sample = 0;  // sum of per-sample sizes at the chosen offsets (scaled by Bmax)
  size_t arena_bytes = 0;             // for max_batch
  std::vector<int64_t> input_shape;   // [1, C, H, W]
  std::vector<int64_t> output_shape;  // [1, ...]
  size_t input_numel = 0, output_numel = 0;
  double flops_per_sample = 0;
  // fp32 mode: every activation buffer holds split (hi, lo) bf16 planes (kernels/common.h), GEMM
  // weights are packed as hi + lo planes, and every kernel runs its split variant.
  bool split = false;
  std::string summary() const;
};

// Thrown by build_plan for a graph with nodes the HIP planner cannot lower (what() lists them all):
// the engine factory's cue for the hybrid HIP + CPU partition (engine.cpp create_engine).
struct PlanUnsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Build the plan for batches up to max_batch.  Throws PlanUnsupported on unsupported graphs, listing EVERY node
// the engine cannot lower (not only the first).  side_branches: mark independent convs to run on
// a second stream (PlanOp::join; extends their inputs' lifetimes).  split: fp32 mode (Plan::split).
// fuse_pairs: lower expand -> reduce 1x1 conv pairs to CONV_PAIR ops (EngineOptions::fuse_pairs).
// fuse_stem_pool: stem conv + max pool in one STEM op (EngineOptions::fuse_stem_pool).
// fuse_gap_fc: global pool + the FC head reading it in one GAP_FC op (EngineOptions::fuse_gap_fc).
// fold_layernorm: LayerNorms read only by GEMMs become statistics ops (EngineOptions::fold_layernorm).
// ln_stats_epilogue: ... and those statistics come from the epilogue of the GEMM producing the
// LayerNorm's input where one does (EngineOptions::ln_stats_epilogue).
Plan build_plan(const onnx::Model& m, int max_batch, bool side_branches = false, bool split = false,
                bool bn_on_load = false, bool fuse_pairs = true, bool fuse_stem_pool = true, bool fuse_gap_fc = false,
                bool fold_layernorm = true, bool ln_stats_epilogue = true);

// Load-time support report: which nodes the HIP planner cannot lower, and why.  `blocked` counts
// nodes not tried because an input came from an unsupported node.
struct PlanReport {
  bool supported = true;
  struct Item {
    std::string node, op, error;
  };
  std::vector<Item> unsupported;
  int blocked = 0;
  std::string text() const;  // one line per unsupported node
};
PlanReport plan_report(const onnx::Model& m, int max_batch = 8, bool split = false);

}  // namespace die
