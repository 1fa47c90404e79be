#include "hip_plan.h"

#include <algorithm>
#include <array>
#include <climits>
#include <cmath>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>

namespace die {

using onnx::Node;

namespace {

constexpr int kBufGraphIn = -2;
constexpr int kBufGraphOut = -3;

uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u) return static_cast<uint16_t>(u >> 16);  // inf/nan
  u += 0x7FFFu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

float from_bf16(uint16_t h) {
  const uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

constexpr int64_t kBatchDim = INT64_MIN;  // symbolic batch size inside SHAPE values

// A planner value.  Besides materialised tensors (NHWC images, bf16/f32 rows) the planner keeps
// lazy views that only become kernels when consumed in a supported way.
struct Val {
  enum Kind {
    GRAPH_IN,    // f32 NCHW graph input
    NHWC,        // bf16 [B][H][W][C]
    ROWS_BF16,   // bf16 rows: logical [B, H*W, C] (rank 3) or [B, C] (rank 2, H*W == 1)
    ROWS_F32,    // f32 rows (graph output)
    NCHW_FLAT,   // Reshape(NHWC, [0, C, -1]) : logical [B, C, H*W] over an NHWC buffer
    HEADS,       // Reshape(rows, [0, 0, nh, hd]) (+ Transposes): base [B, S, nh, hd], logical = perm
    ATTN,        // attention chain: stage 0 = Q K^T, 1 = softmax, 2 = (P V) with logical perm
    SHAPE,       // int64 shape-computation value (ints known unless `known` is false)
    BCAST_INIT,  // Expand(initializer, shape) -> [B, 1, C]
    TOKCAT,      // Concat([cls, patch rows], axis=1)
    UNKNOWN      // produced by a node the planner could not lower (support report)
  } kind = NHWC;
  int C = 0, H = 1, W = 1;
  // Stored vs logical channels: rows / NHWC pixels are stored with C channels (a multiple of 8:
  // 16-byte vectors, MFMA K/N steps); `cl` is the model's channel count when that is smaller (pad
  // channels hold finite values that every consumer ignores: zero weights, dropped on output).
  int cl = 0;
  // ROWS_BF16 from Flatten/Reshape of an NHWC map with H*W > 1: ONNX order is (c, h, w), the buffer
  // holds (h, w, c); a Gemm/MatMul consumer permutes its weight rows instead of the data.
  int flat_hw = 0, flat_c = 0;
  int buf = -1;
  int rank = 0;         // ROWS: 2 or 3
  int ld = 0, col = 0;  // ROWS/HEADS: row pitch (0 -> C) and column offset, in elements
  bool has_affine = false;
  std::vector<float> asc, ash;
  // HEADS / ATTN
  int nh = 0, hd = 0;
  std::array<int, 4> perm{{0, 1, 2, 3}};
  int q = -1, k = -1, v = -1, stage = 0;
  float scale = 1.f;
  // SHAPE / BCAST_INIT / TOKCAT
  std::vector<int64_t> ints;
  bool known = true;
  std::string init_name;
  int patches = -1;
  int pitch() const { return ld ? ld : C; }
  int logical() const { return cl ? cl : C; }
  bool padded() const { return cl && cl != C; }
};

int round8(int c) { return (c + 7) / 8 * 8; }

class Planner {
 public:
  Planner(const onnx::Model& m, int max_batch, bool side_branches, bool split, bool bn_on_load, bool fuse_pairs = true,
          bool fuse_stem_pool = true, bool fuse_gap_fc = false, bool fold_layernorm = true,
          bool ln_stats_epilogue = true)
      : m_(m), max_batch_(max_batch), side_branches_(side_branches), split_(split), bn_on_load_(bn_on_load),
        fuse_pairs_(fuse_pairs), fuse_stem_pool_(fuse_stem_pool), fuse_gap_fc_(fuse_gap_fc),
        fold_layernorm_(fold_layernorm), ln_stats_epilogue_(ln_stats_epilogue) {}

  // Every node is tried; a node that cannot be lowered is recorded (with its error) and its
  // outputs become UNKNOWN, so the walk goes on and the report lists every unsupported node.
  PlanReport report_;

  Plan run() {
    if (m_.inputs.empty() || m_.outputs.empty()) throw std::runtime_error("model needs an input and an output");
    for (size_t i = 0; i < m_.nodes.size(); ++i)
      for (auto& in : m_.nodes[i].inputs) consumers_[in].push_back(static_cast<int>(i));
    for (auto& o : m_.outputs) graph_outputs_.insert(o.name);
    plan_.split = split_;
    define_graph_input();

    done_.assign(m_.nodes.size(), false);
    for (size_t i = 0; i < m_.nodes.size(); ++i) {
      if (done_[i]) continue;
      done_[i] = true;
      const Node& n = m_.nodes[i];
      bool blocked = false;
      for (const auto& in : n.inputs) {
        auto it = vid_.find(in);
        if (it != vid_.end() && vals_[it->second].kind == Val::UNKNOWN) blocked = true;
      }
      if (blocked) {
        report_.blocked++;
        mark_unknown(n);
        continue;
      }
      try {
        lower(static_cast<int>(i));
      } catch (const std::exception& e) {
        report_.supported = false;
        report_.unsupported.push_back(PlanReport::Item{n.name, n.op_type, e.what()});
        mark_unknown(n);
      }
    }
    if (!report_.supported) throw PlanUnsupported("HIP engine cannot lower this graph:\n" + report_.text());
    finalize_output();
    fuse_pool_affine();
    if (fuse_stem_pool_) fuse_stem_pool();
    if (fuse_pairs_) fuse_conv_pairs();
    if (fuse_gap_fc_) fuse_gap_fc();
    // fp32 (split) mode only: in bf16 the weights re-rounded with gamma folded in and the mean
    // subtracted after a bf16-input GEMM cost ViT-B/16 ~3 % of its rel-L2 budget
    if (fold_layernorm_ && split_) fold_layernorm();
    if (fold_layernorm_ && split_ && ln_stats_epilogue_) stats_from_producer();
    if (bn_on_load_ && !split_) preact_on_load();  // measured slower (profiles/r1_preact_on_load.md)
    if (side_branches_) mark_side_branches();
    assign_arena();
    return std::move(plan_);
  }

 private:
  // ---- helpers --------------------------------------------------------------------------------
  const onnx::Tensor& init(const std::string& name, const Node& n) const {
    auto it = m_.initializers.find(name);
    if (it == m_.initializers.end())
      throw std::runtime_error(n.op_type + " " + n.name + ": input " + name + " must be an initializer");
    return it->second;
  }
  bool is_init(const std::string& name) const { return m_.initializers.count(name) != 0; }
  Val& val(const std::string& name, const Node& n) {
    auto it = vid_.find(name);
    if (it == vid_.end()) throw std::runtime_error(n.op_type + " " + n.name + ": unknown input value " + name);
    return vals_[it->second];
  }
  void define(const std::string& name, const Val& v) {
    vid_[name] = static_cast<int>(vals_.size());
    vals_.push_back(v);
  }
  int sole_consumer(const std::string& name) const {
    if (graph_outputs_.count(name)) return -1;
    auto it = consumers_.find(name);
    if (it == consumers_.end() || it->second.size() != 1) return -1;
    return done_[it->second[0]] ? -1 : it->second[0];
  }
  std::vector<int> consumers(const std::string& name) const {
    auto it = consumers_.find(name);
    return it == consumers_.end() ? std::vector<int>{} : it->second;
  }
  // An activation buffer of `bytes_per_sample` bf16 bytes (fp32 mode: hi and lo planes, twice that).
  int new_buf(size_t bytes_per_sample) {
    PlanBuf b;
    b.bytes_per_sample = bytes_per_sample * (split_ ? 2 : 1);
    plan_.bufs.push_back(b);
    return static_cast<int>(plan_.bufs.size()) - 1;
  }
  size_t push_f32(const std::vector<float>& v) {
    size_t off = round_up(plan_.params.size(), 256);
    plan_.params.resize(off + round_up(v.size(), 128) * 4, 0);
    std::memcpy(plan_.params.data() + off, v.data(), v.size() * 4);
    return off;
  }
  size_t push_bf16(const std::vector<uint16_t>& v) {
    size_t off = round_up(plan_.params.size(), 256);
    plan_.params.resize(off + v.size() * 2);
    std::memcpy(plan_.params.data() + off, v.data(), v.size() * 2);
    return off;
  }
  // GEMM weights given in fp32: bf16, or (fp32 mode) the hi plane followed by the lo plane
  // (lo = bf16(w - hi)); `wplane` receives the plane distance in elements (0 when not split).
  size_t push_weights(const std::vector<float>& w, long long& wplane) {
    std::vector<uint16_t> q(w.size() * (split_ ? 2 : 1));
    for (size_t i = 0; i < w.size(); ++i) {
      q[i] = to_bf16(w[i]);
      if (split_) {
        uint32_t u = static_cast<uint32_t>(q[i]) << 16;
        float hi;
        std::memcpy(&hi, &u, 4);
        q[w.size() + i] = to_bf16(w[i] - hi);
      }
    }
    wplane = split_ ? static_cast<long long>(w.size()) : 0;
    return push_bf16(q);
  }
  void add_op(PlanOp op) { plan_.ops.push_back(std::move(op)); }

  void mark_unknown(const Node& n) {
    Val u;
    u.kind = Val::UNKNOWN;
    for (const auto& o : n.outputs)
      if (!vid_.count(o)) define(o, u);
  }

  // Graph input 0 (the reference binds input 0 of any model, src/inference_engine.cpp:35-52):
  //  * rank 4 [N, C, H, W]: an image (lazy: folded into the stem or an input-prep pass);
  //  * rank 2 [N, F] / rank 3 [N, S, F]: rows -> one ROWS_PREP pass (f32 -> bf16 / split, F padded
  //    to a multiple of 8).
  void define_graph_input() {
    const auto& vi = m_.inputs[0];
    const size_t r = vi.dims.size();
    for (size_t k = 1; k < r; ++k)
      if (vi.dims[k] <= 0) throw std::runtime_error("input dims must be static except the batch");
    if (r == 4) {
      Val in;
      in.kind = Val::GRAPH_IN;
      in.C = static_cast<int>(vi.dims[1]);
      in.H = static_cast<int>(vi.dims[2]);
      in.W = static_cast<int>(vi.dims[3]);
      in.buf = kBufGraphIn;
      define(vi.name, in);
      plan_.input_shape = {1, in.C, in.H, in.W};
      plan_.input_numel = static_cast<size_t>(in.C) * in.H * in.W;
      return;
    }
    if (r != 2 && r != 3)
      throw std::runtime_error("HIP engine takes a rank-2, -3 or -4 input, got rank " + std::to_string(r));
    const int S = r == 3 ? static_cast<int>(vi.dims[1]) : 1;
    const int F = static_cast<int>(vi.dims[r - 1]);
    PlanOp p;
    p.kind = PlanOp::ROWS_PREP;
    p.name = "rows_prep";
    p.in = kBufGraphIn;
    p.C = F;
    p.Cp = round8(F);
    p.rows_per_sample = S;
    p.out = new_buf(static_cast<size_t>(S) * p.Cp * 2);
    Val v;
    v.kind = Val::ROWS_BF16;
    v.C = p.Cp;
    v.cl = p.Cp != F ? F : 0;
    v.H = S;
    v.rank = static_cast<int>(r);
    v.buf = p.out;
    add_op(std::move(p));
    define(vi.name, v);
    plan_.input_shape = r == 3 ? std::vector<int64_t>{1, S, F} : std::vector<int64_t>{1, F};
    plan_.input_numel = static_cast<size_t>(S) * F;
  }

  // BN parameters -> per-channel (scale, shift).
  void bn_affine(const Node& bn, std::vector<float>& sc, std::vector<float>& sh) {
    const auto& g = init(bn.in(1), bn).f;
    const auto& b = init(bn.in(2), bn).f;
    const auto& mu = init(bn.in(3), bn).f;
    const auto& var = init(bn.in(4), bn).f;
    const float eps = bn.get_float("epsilon", 1e-5f);
    sc.resize(g.size());
    sh.resize(g.size());
    for (size_t c = 0; c < g.size(); ++c) {
      sc[c] = g[c] / std::sqrt(var[c] + eps);
      sh[c] = b[c] - mu[c] * sc[c];
    }
  }

  // ---- lowering ---------------------------------------------------------------------------------
  void lower(int idx) {
    const Node& n = m_.nodes[idx];
    const std::string& op = n.op_type;
    if (lower_shape_op(idx)) return;
    if (op == "Conv") return n.get_int("group", 1) != 1 ? lower_gconv(idx) : lower_conv(idx);
    if (op == "Gemm" || (op == "MatMul" && is_init(n.in(1)))) return lower_gemm(idx);
    if (op == "MatMul") return lower_attn_matmul(idx);
    if (op == "BatchNormalization") return lower_bn(idx);
    if (op == "Relu") return lower_relu(idx);
    if (op == "Add") return lower_add(idx);
    if (op == "MaxPool" || op == "AveragePool") return lower_pool(idx);
    if (op == "GlobalAveragePool") return lower_gap(idx);
    if (op == "Reshape") return lower_reshape(idx);
    if (op == "Flatten" || op == "Squeeze") return lower_flatten(idx);
    if (op == "Transpose") return lower_transpose(idx);
    if (op == "Div" || op == "Mul" || op == "Sub") return lower_scale(idx);
    if (op == "Softmax") return lower_softmax(idx);
    if (op == "Clip") return lower_clip(idx);
    if (op == "ReduceMean") return lower_reduce_mean(idx);
    if (op == "ReduceSum" || op == "ReduceMax") {
      if (lower_spatial_reduce(idx, op == "ReduceSum" ? 1 : 2)) return;
      throw std::runtime_error(op + " " + n.name + ": only reductions over the spatial axes of an image or the token axis of rows");
    }
    if (op == "GlobalMaxPool") return lower_gap(idx, 2);
    if (op == "Max" || op == "Min") {
      if (n.inputs.size() == 2 && lower_binary_acts(n)) return;
      throw std::runtime_error(op + " " + n.name + ": only two activations of one shape (or a per-sample broadcast)");
    }
    if (op == "Pad") return lower_pad(idx);
    if (op == "ZeroInsert" && n.domain == "die") return lower_pad(idx);  // ConvTranspose rewrite (rewrite_for_device)
    if (op == "Greater" || op == "Less" || op == "Equal" || op == "GreaterOrEqual" || op == "LessOrEqual")
      return lower_compare(idx);
    if (op == "And" || op == "Or") {
      if (lower_binary_acts(n)) return;
      throw std::runtime_error(op + " " + n.name + ": only two boolean activations of one shape");
    }
    if (op == "Not") return emit_unary(n, materialize_in(n.in(0), n), 23, 0.f, 0.f, n.outputs[0]);
    if (op == "Where") return lower_where(idx);
    if (op == "Cast") return lower_cast(idx);
    if (op == "Resize" || op == "Upsample") return lower_resize(idx);
    if (op == "Split") return lower_split(idx);
    if (op == "Slice") return lower_slice(idx);
    if (op == "LayerNormalization") return lower_layernorm(idx);
    if (op == "Gather") return lower_gather(idx);
    if (op == "Concat") return lower_concat(idx);
    if (op == "Sigmoid" || op == "Tanh" || op == "LeakyRelu" || op == "Gelu" || op == "Exp" || op == "Abs" ||
        op == "Sqrt" || op == "Neg" || op == "Reciprocal" || op == "Log" || op == "Erf" || op == "Pow" ||
        op == "HardSigmoid" || op == "HardSwish" || op == "Softplus")
      return lower_unary(idx);
    if (op == "Identity" || op == "Dropout") {
      Val v = val(n.in(0), n);
      define(n.outputs[0], v);
      return;
    }
    throw std::runtime_error("HIP engine: unsupported op " + op + " (" + n.name + ")");
  }

  int ensure_nhwc_input(Val& x, const std::string& name) {
    // Graph input -> input-prep kernel (applies any pending BN affine), memoised per value.
    auto it = prepped_.find(name);
    if (it != prepped_.end()) return it->second;
    PlanOp p;
    p.kind = PlanOp::INPUT_PREP;
    p.name = "input_prep";
    p.in = kBufGraphIn;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.Cp = x.C <= 4 ? 4 : round8(x.C);  // > 8 channels: input_prep_wide
    if (x.has_affine) {
      p.scale_off = push_f32(x.asc);
      p.shift_off = push_f32(x.ash);
    }
    p.out = new_buf(static_cast<size_t>(p.Cp) * x.H * x.W * 2);
    const int buf = p.out;
    add_op(std::move(p));
    prepped_[name] = buf;
    return buf;
  }

  // An image graph input (lazy: f32 NCHW plus any pending BN affine) consumed by something other
  // than a conv's input load -- a ReLU, a pool, the residual operand of an Add: the input-prep
  // pass materialises it as an NHWC tensor once (per value: the raw input and its BN'd form are
  // two values) and every later reader sees that.  Hybrid HIP + CPU segments start at such inputs
  // (engine/hybrid_engine.cpp: a ResNet segment begins at a unit's raw sum x).
  Val materialize_in(const std::string& name, const Node& n) {
    Val v = val(name, n);
    if (v.kind != Val::GRAPH_IN) return v;
    const int buf = ensure_nhwc_input(v, name);
    Val o = v;
    o.kind = Val::NHWC;
    o.C = v.C <= 4 ? 4 : round8(v.C);
    o.cl = o.C != v.C ? v.C : 0;
    o.buf = buf;
    o.has_affine = false;
    o.asc.clear();
    o.ash.clear();
    define(name, o);
    return o;
  }

  void lower_conv(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = val(n.in(0), n);
    const auto& wt = init(n.in(1), n);
    if (wt.dims.size() != 4) throw std::runtime_error("Conv " + n.name + ": only 2-D convs are supported");
    if (n.get_int("group", 1) != 1) throw std::runtime_error("Conv " + n.name + ": grouped convs are not supported yet");
    const int Cout = static_cast<int>(wt.dims[0]), Cin = static_cast<int>(wt.dims[1]);
    const int KH = static_cast<int>(wt.dims[2]), KW = static_cast<int>(wt.dims[3]);
    auto st = n.get_ints("strides", {1, 1});
    auto dl = n.get_ints("dilations", {1, 1});
    auto pads = conv_pads(n);
    if (st[0] != st[1] || dl[0] != dl[1]) throw std::runtime_error("Conv " + n.name + ": anisotropic stride/dilation");
    const std::string ap = n.get_string("auto_pad", "NOTSET");
    int in_buf;
    int Cstore;
    // A ResNet-style stem on the graph input reads the fp32 NCHW input itself (input_prep fused into
    // its patch loader); the prep pass is only planned if this conv turns out not to be that stem.
    bool deferred_prep = false;
    if (x.kind == Val::GRAPH_IN) {
      deferred_prep = KH == 7 && KW == 7 && x.C <= 4;
      in_buf = deferred_prep ? -2 : ensure_nhwc_input(x, n.in(0));
      Cstore = x.C <= 4 ? 4 : round8(x.C);
    } else if (x.kind == Val::NHWC) {
      in_buf = x.buf;
      Cstore = x.C;  // stored channels (pad channels get zero weights)
    } else {
      throw std::runtime_error("Conv " + n.name + ": input must be an image tensor");
    }
    if (Cin != (x.kind == Val::GRAPH_IN ? x.C : x.logical())) throw std::runtime_error("Conv " + n.name + ": channel mismatch");
    if (ap == "SAME_UPPER" || ap == "SAME_LOWER") {
      for (int d = 0; d < 2; ++d) {
        const int in = d ? x.W : x.H, k = d ? KW : KH;
        const int out = (in + static_cast<int>(st[0]) - 1) / static_cast<int>(st[0]);
        const int total = std::max(0, (out - 1) * static_cast<int>(st[0]) + (k - 1) * static_cast<int>(dl[0]) + 1 - in);
        const int lo = ap == "SAME_UPPER" ? total / 2 : total - total / 2;
        pads[d] = lo;
        pads[d + 2] = total - lo;
      }
    } else if (ap == "VALID") {
      pads = {0, 0, 0, 0};
    }
    // pads = [top, left, bottom, right]: the kernels offset by top/left and bound-check the input,
    // so asymmetric padding (TF-style SAME exports) only changes the output size
    const int s = static_cast<int>(st[0]), d = static_cast<int>(dl[0]);
    const int Ho = (x.H + static_cast<int>(pads[0] + pads[2]) - d * (KH - 1) - 1) / s + 1;
    const int Wo = (x.W + static_cast<int>(pads[1] + pads[3]) - d * (KW - 1) - 1) / s + 1;
    // Cout % 8 != 0: computed and stored with Cp channels (zero weights and bias: pad channels are
    // act(0)), the Val remembers the logical count
    const int Cp = round8(Cout);

    // --- fusion lookahead ---
    std::vector<float> scale(Cp, 1.f), shift(Cp, 0.f);
    if (!n.in(2).empty()) {
      const auto& b = init(n.in(2), n).f;
      for (int c = 0; c < Cout; ++c) shift[c] = b[c];
    }
    std::string cur = n.outputs[0];
    int c1 = sole_consumer(cur);
    if (c1 >= 0 && m_.nodes[c1].op_type == "BatchNormalization") {
      std::vector<float> sc, sh;
      bn_affine(m_.nodes[c1], sc, sh);
      for (int c = 0; c < Cout; ++c) {
        scale[c] = sc[c];
        shift[c] = shift[c] * sc[c] + sh[c];
      }
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    }
    int relu = 0, res_buf = -1;
    float clip_lo = 0.f, clip_hi = 0.f;
    std::string res_name;
    c1 = sole_consumer(cur);
    if (c1 >= 0 && m_.nodes[c1].op_type == "Relu") {
      relu = 1;
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    } else if (c1 >= 0 && m_.nodes[c1].op_type == "Clip" && clip_bounds(m_.nodes[c1], clip_lo, clip_hi)) {
      relu = 3;  // Clip epilogue (ReLU6)
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    } else if (c1 >= 0 && m_.nodes[c1].op_type == "Add") {
      const Node& add = m_.nodes[c1];
      const std::string other = add.in(0) == cur ? add.in(1) : add.in(0);
      if (vid_.count(other) && vals_[vid_.at(other)].kind == Val::GRAPH_IN) materialize_in(other, add);
      auto it = vid_.find(other);
      if (it != vid_.end() && vals_[it->second].kind == Val::NHWC && vals_[it->second].C == Cp &&
          vals_[it->second].logical() == Cout && vals_[it->second].H == Ho && vals_[it->second].W == Wo &&
          add.in(0) != add.in(1)) {
        res_buf = vals_[it->second].buf;
        res_name = other;
        done_[c1] = true;
        cur = add.outputs[0];
        const int c2 = sole_consumer(cur);
        if (c2 >= 0 && m_.nodes[c2].op_type == "Relu") {
          relu = 1;
          done_[c2] = true;
          cur = m_.nodes[c2].outputs[0];
        }
      }
    }
    // dual store: a BN (+ReLU) consumer of `cur`
    std::string out2_name;
    std::vector<float> s2, b2;
    int relu2 = 0;
    int bn2 = -1;
    for (int ci : consumers(cur)) {
      if (!done_[ci] && m_.nodes[ci].op_type == "BatchNormalization" && m_.nodes[ci].in(0) == cur) {
        bn2 = ci;
        break;
      }
    }
    if (bn2 >= 0) {
      bn_affine(m_.nodes[bn2], s2, b2);
      s2.resize(Cp, 1.f);
      b2.resize(Cp, 0.f);
      done_[bn2] = true;
      out2_name = m_.nodes[bn2].outputs[0];
      const int c3 = sole_consumer(out2_name);
      if (c3 >= 0 && m_.nodes[c3].op_type == "Relu") {
        relu2 = 1;
        done_[c3] = true;
        out2_name = m_.nodes[c3].outputs[0];
      }
    }
    bool need_out1 = graph_outputs_.count(cur) != 0 || bn2 < 0;
    for (int ci : consumers(cur))
      if (ci != bn2) need_out1 = true;

    // --- weights: [Npad][Kpad] bf16, k = (ky*KW + kx)*Cstore + ci ---
    const int K = KH * KW * Cstore;
    const int Kpad = static_cast<int>(round_up(K, 64));
    const int Npad = static_cast<int>(round_up(Cp, 128));
    std::vector<float> wp(static_cast<size_t>(Npad) * Kpad, 0.f);
    for (int co = 0; co < Cout; ++co)
      for (int ci = 0; ci < Cin; ++ci)
        for (int ky = 0; ky < KH; ++ky)
          for (int kx = 0; kx < KW; ++kx) {
            const float w = wt.f[((static_cast<size_t>(co) * Cin + ci) * KH + ky) * KW + kx] * scale[co];
            wp[static_cast<size_t>(co) * Kpad + (ky * KW + kx) * Cstore + ci] = w;
          }

    PlanOp p;
    p.kind = PlanOp::CONV;
    p.name = n.name;
    p.in = in_buf;
    p.in2 = res_buf;
    // ResNet stem (7x7/2, pad 3, 4 stored input channels, 64 outputs, plain epilogue): LDS-patch kernel
    const bool stem = KH == 7 && KW == 7 && s == 2 && d == 1 && pads[0] == 3 && pads[1] == 3 && pads[2] == 3 &&
                      pads[3] == 3 && Cstore == 4 && Cout == 64 && res_buf < 0 && bn2 < 0 && need_out1 &&
                      relu != 3 && !graph_outputs_.count(cur);
    if (deferred_prep && !stem) {
      in_buf = ensure_nhwc_input(x, n.in(0));
      p.in = in_buf;
    }
    if (stem) {
      p.kind = PlanOp::STEM;
      if (in_buf == -2) {  // fused input prep: channel count and the input's pending affine
        p.C = x.C;
        if (x.has_affine) {
          p.scale_off = push_f32(x.asc);
          p.shift_off = push_f32(x.ash);
        }
      }
      std::vector<float> ws(64 * 224, 0.f);
      for (int co = 0; co < Cout; ++co)
        for (int ci = 0; ci < Cin; ++ci)
          for (int ky = 0; ky < 7; ++ky)
            for (int kx = 0; kx < 7; ++kx)
              ws[co * 224 + ky * 32 + kx * 4 + ci] = wt.f[((static_cast<size_t>(co) * Cin + ci) * KH + ky) * KW + kx] * scale[co];
      wp.swap(ws);
    }
    p.w_off = push_weights(wp, p.conv.wplane);
    p.conv.split = split_;
    p.bias_off = push_f32(shift);
    auto& a = p.conv;
    a.H = x.H;
    a.W = x.W;
    a.Cin = Cstore;
    a.Ho = Ho;
    a.Wo = Wo;
    a.N = Cp;
    a.KH = KH;
    a.KW = KW;
    a.stride = s;
    a.pad_h = static_cast<int>(pads[0]);
    a.pad_w = static_cast<int>(pads[1]);
    a.dil = d;
    a.K = K;
    a.Kpad = Kpad;
    a.relu = relu;
    a.relu2 = relu2;
    a.clip_lo = clip_lo;
    a.clip_hi = clip_hi;
    p.flops_per_sample = 2.0 * Ho * Wo * Cout * (KH * KW * Cin);
    p.tile_bmax = kern::choose_tile(max_batch_ * Ho * Wo, Cp, K);
    const size_t out_bytes = static_cast<size_t>(Ho) * Wo * Cp * 2;
    Val o;
    o.kind = Val::NHWC;
    o.C = Cp;
    o.cl = Cp != Cout ? Cout : 0;
    o.H = Ho;
    o.W = Wo;
    if (need_out1) {
      p.out = new_buf(out_bytes);
      o.buf = p.out;
      define(cur, o);
    }
    if (bn2 >= 0) {
      p.s2_off = push_f32(s2);
      p.b2_off = push_f32(b2);
      p.out2 = new_buf(out_bytes);
      Val o2 = o;
      o2.buf = p.out2;
      define(out2_name, o2);
    }
    add_op(std::move(p));
  }

  // ---- GEMM over rows ---------------------------------------------------------------------------
  bool scalar_is(const std::string& name, float want) const {
    auto it = m_.initializers.find(name);
    if (it == m_.initializers.end() || it->second.f.size() != 1) return false;
    return std::fabs(it->second.f[0] - want) <= 1e-3f * std::fabs(want);
  }
  static const std::string& other_input(const Node& nd, const std::string& x) { return nd.in(0) == x ? nd.in(1) : nd.in(0); }

  // erf-GELU as exported by torch: x/sqrt2 -> Erf -> +1 -> (x * .) -> (* 0.5), or 0.5x * (1 + erf).
  bool match_gelu(const std::string& v, std::vector<int>& used, std::string& out) const {
    if (graph_outputs_.count(v)) return false;
    const auto cs = consumers(v);
    if (cs.size() != 2) return false;
    int dv = -1, mu = -1;
    for (int c : cs) {
      if (done_[c]) return false;
      const Node& nd = m_.nodes[c];
      if (nd.op_type == "Div" && nd.in(0) == v && scalar_is(nd.in(1), 1.41421356f)) dv = c;
      else if (nd.op_type == "Mul" && scalar_is(other_input(nd, v), 0.70710678f)) dv = c;
      else if (nd.op_type == "Mul") mu = c;
      else return false;
    }
    if (dv < 0 || mu < 0) return false;
    const int er = sole_consumer(m_.nodes[dv].outputs[0]);
    if (er < 0 || m_.nodes[er].op_type != "Erf") return false;
    const int ad = sole_consumer(m_.nodes[er].outputs[0]);
    if (ad < 0 || m_.nodes[ad].op_type != "Add" || !scalar_is(other_input(m_.nodes[ad], m_.nodes[er].outputs[0]), 1.f))
      return false;
    const std::string& a = m_.nodes[ad].outputs[0];
    const Node& M = m_.nodes[mu];
    const std::string& mo = other_input(M, v);
    if (mo == a) {
      const int hf = sole_consumer(M.outputs[0]);
      if (hf < 0 || m_.nodes[hf].op_type != "Mul" || !scalar_is(other_input(m_.nodes[hf], M.outputs[0]), 0.5f)) return false;
      used = {dv, er, ad, mu, hf};
      out = m_.nodes[hf].outputs[0];
      return true;
    }
    if (scalar_is(mo, 0.5f)) {
      const int fin = sole_consumer(a);
      if (fin < 0 || fin != sole_consumer(M.outputs[0]) || m_.nodes[fin].op_type != "Mul") return false;
      used = {dv, er, ad, mu, fin};
      out = m_.nodes[fin].outputs[0];
      return true;
    }
    return false;
  }

  struct GemmTail {
    std::vector<float> bias;  // from a following Add(initializer), empty if none
    int act = 0;              // 1 relu, 2 gelu
    std::string res;          // residual operand (rows)
    std::string out;
    std::vector<int> used;
  };
  // Epilogue fusion lookahead for a MatMul/Gemm producing `N` columns over `rows` rows per sample.
  GemmTail gemm_tail(const Node& n, int N, int rows, bool is_gemm, int N_logical) const {
    GemmTail t;
    t.out = n.outputs[0];
    int c1 = sole_consumer(t.out);
    if (!is_gemm && c1 >= 0 && m_.nodes[c1].op_type == "Add" && is_init(other_input(m_.nodes[c1], t.out))) {
      const auto& c = m_.initializers.at(other_input(m_.nodes[c1], t.out)).f;
      if (c.size() == static_cast<size_t>(N_logical) || c.size() == 1) {
        t.bias.assign(N, 0.f);
        for (int j = 0; j < N_logical; ++j) t.bias[j] = c[c.size() == 1 ? 0 : j];
        t.used.push_back(c1);
        t.out = m_.nodes[c1].outputs[0];
        c1 = sole_consumer(t.out);
      }
    }
    std::vector<int> gu;
    std::string g;
    if (c1 >= 0 && m_.nodes[c1].op_type == "Relu") {
      t.act = 1;
      t.used.push_back(c1);
      t.out = m_.nodes[c1].outputs[0];
    } else if (match_gelu(t.out, gu, g)) {
      t.act = 2;
      t.used.insert(t.used.end(), gu.begin(), gu.end());
      t.out = g;
    } else if (c1 >= 0 && m_.nodes[c1].op_type == "Add") {
      const Node& add = m_.nodes[c1];
      const std::string& other = other_input(add, t.out);
      auto it = vid_.find(other);
      if (it != vid_.end() && add.in(0) != add.in(1)) {
        const Val& r = vals_[it->second];
        if (r.kind == Val::ROWS_BF16 && r.C == N && r.logical() == N_logical && r.H * r.W == rows &&
            r.pitch() == r.C && r.col == 0) {
          t.res = other;
          t.used.push_back(c1);
          t.out = add.outputs[0];
          const int c2 = sole_consumer(t.out);
          if (c2 >= 0 && m_.nodes[c2].op_type == "Relu") {
            t.act = 1;
            t.used.push_back(c2);
            t.out = m_.nodes[c2].outputs[0];
          }
        }
      }
    }
    return t;
  }

  // Sibling MatMuls of one input that each only add a bias and feed a Reshape (Q/K/V projections)
  // -> one GEMM with concatenated weights.  Returns the group (just {idx} when not applicable).
  std::vector<int> qkv_group(int idx, const std::string& xname, int K) const {
    std::vector<int> g;
    bool self = false;
    for (int c : consumers(xname)) {
      if (c != idx && done_[c]) continue;
      const Node& nd = m_.nodes[c];
      if (nd.op_type != "MatMul" || nd.in(0) != xname || !is_init(nd.in(1))) continue;
      const auto& w = m_.initializers.at(nd.in(1));
      if (w.dims.size() != 2 || w.dims[0] != K || w.dims[1] % 8) continue;
      const int a = sole_consumer(nd.outputs[0]);
      if (a < 0 || m_.nodes[a].op_type != "Add" || !is_init(other_input(m_.nodes[a], nd.outputs[0]))) continue;
      if (m_.initializers.at(other_input(m_.nodes[a], nd.outputs[0])).f.size() != static_cast<size_t>(w.dims[1])) continue;
      const int r = sole_consumer(m_.nodes[a].outputs[0]);
      if (r < 0 || m_.nodes[r].op_type != "Reshape") continue;
      g.push_back(c);
      self |= c == idx;
    }
    if (!self || g.size() < 2) return {idx};
    return g;
  }

  void lower_gemm(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    const bool gemm = n.op_type == "Gemm";
    int rows = 1, rank = 2;
    if (x.kind == Val::ROWS_BF16) {
      rows = x.H * x.W;
      rank = x.rank ? x.rank : (rows == 1 ? 2 : 3);
    } else if (!(x.kind == Val::NHWC && x.H == 1 && x.W == 1)) {
      throw std::runtime_error(n.op_type + " " + n.name + ": input must be a [batch, (tokens,) features] matrix");
    }
    if (x.pitch() != x.C || x.col) throw std::runtime_error(n.op_type + " " + n.name + ": strided input rows");
    if (gemm && rank != 2) throw std::runtime_error("Gemm " + n.name + ": input must be 2-D");
    const auto& wt = init(n.in(1), n);
    if (wt.dims.size() != 2) throw std::runtime_error(n.op_type + " " + n.name + ": weight must be 2-D");
    if (gemm && n.get_int("transA", 0)) throw std::runtime_error("Gemm " + n.name + ": transA is not supported");
    const bool tb = gemm && n.get_int("transB", 0);
    const float alpha = gemm ? n.get_float("alpha", 1.f) : 1.f;
    const float beta = gemm ? n.get_float("beta", 1.f) : 1.f;
    // K: the model's inner dimension; Ks: the stored row length (pads / NHWC-flatten order)
    const int K = static_cast<int>(tb ? wt.dims[1] : wt.dims[0]);
    const int Ks = x.C;
    const int hw = x.flat_hw;  // Flatten of an NHWC map: logical k = c*hw + p sits at p*Cs + c
    const int Kl = hw ? x.flat_c * hw : x.logical();
    if (K != Kl) throw std::runtime_error(n.op_type + " " + n.name + ": inner dimension mismatch");
    auto kstore = [&](int k) { return hw ? (k % hw) * (Ks / hw) + k / hw : k; };

    const std::vector<int> group = gemm ? std::vector<int>{idx} : qkv_group(idx, n.in(0), K);
    // columns of each member
    std::vector<int> Ns, offs;
    int Ntot = 0;
    for (int gi : group) {
      const auto& w = init(m_.nodes[gi].in(1), m_.nodes[gi]);
      const int Nj = static_cast<int>(tb ? w.dims[0] : w.dims[1]);
      offs.push_back(Ntot);
      Ns.push_back(Nj);
      Ntot += Nj;
    }
    const int Np = group.size() > 1 ? Ntot : round8(Ntot);  // stored columns (QKV members are % 8 already)
    const int Kpad = static_cast<int>(round_up(Ks, 64));
    const int Npad = static_cast<int>(round_up(Np, 128));
    std::vector<float> wp(static_cast<size_t>(Npad) * Kpad, 0.f);
    std::vector<float> bias(Np, 0.f);
    for (size_t g = 0; g < group.size(); ++g) {
      const Node& nd = m_.nodes[group[g]];
      const auto& w = init(nd.in(1), nd);
      const int Nj = Ns[g];
      for (int j = 0; j < Nj; ++j)
        for (int k = 0; k < K; ++k) {
          const float v = tb ? w.f[static_cast<size_t>(j) * K + k] : w.f[static_cast<size_t>(k) * Nj + j];
          wp[static_cast<size_t>(offs[g] + j) * Kpad + kstore(k)] = alpha * v;
        }
      if (gemm && !nd.in(2).empty()) {
        const auto& c = init(nd.in(2), nd).f;
        for (int j = 0; j < Nj; ++j) bias[offs[g] + j] = beta * c[c.size() == 1 ? 0 : j % c.size()];
      }
    }
    PlanOp p;
    p.kind = PlanOp::CONV;
    p.name = group.size() > 1 ? n.name + "+qkv" : n.name;
    p.in = x.buf;
    p.w_off = push_weights(wp, p.conv.wplane);
    p.conv.split = split_;
    auto& a = p.conv;
    a.H = a.Ho = rows;
    a.Cin = Ks;
    a.N = Np;
    a.K = Ks;
    a.Kpad = Kpad;
    p.flops_per_sample = 2.0 * rows * Ntot * K;
    p.tile_bmax = kern::choose_tile(max_batch_ * rows, Np, Ks);

    if (group.size() > 1) {
      // bias of each member's Add; outputs are column slices of one [rows][Ntot] buffer
      p.out = new_buf(static_cast<size_t>(rows) * Ntot * 2);
      for (size_t g = 0; g < group.size(); ++g) {
        done_[group[g]] = true;
        const Node& nd = m_.nodes[group[g]];
        const int ad = sole_consumer(nd.outputs[0]);
        const auto& c = m_.initializers.at(other_input(m_.nodes[ad], nd.outputs[0])).f;
        for (int j = 0; j < Ns[g]; ++j) bias[offs[g] + j] += c[j];
        done_[ad] = true;
        Val o;
        o.kind = Val::ROWS_BF16;
        o.C = Ns[g];
        o.H = rows;
        o.rank = rank;
        o.buf = p.out;
        o.ld = Ntot;
        o.col = offs[g];
        define(m_.nodes[ad].outputs[0], o);
      }
      p.bias_off = push_f32(bias);
      add_op(std::move(p));
      return;
    }

    const GemmTail t = gemm_tail(n, Np, rows, gemm, Ntot);
    for (int u : t.used) done_[u] = true;
    for (int j = 0; j < Np && !t.bias.empty(); ++j) bias[j] += t.bias[j];
    p.bias_off = push_f32(bias);
    a.relu = t.act;
    if (!t.res.empty()) p.in2 = vals_[vid_.at(t.res)].buf;
    Val o;
    o.C = Np;
    o.cl = Np != Ntot ? Ntot : 0;
    o.H = rows;
    o.rank = rank;
    if (graph_outputs_.count(t.out) && consumers(t.out).empty() && Np == Ntot) {
      p.out_f32 = kBufGraphOut;
      o.kind = Val::ROWS_F32;
      o.buf = kBufGraphOut;
    } else {
      p.out = new_buf(static_cast<size_t>(rows) * Np * 2);
      o.kind = Val::ROWS_BF16;
      o.buf = p.out;
    }
    define(t.out, o);
    add_op(std::move(p));
  }

  // ---- transformer views / ops --------------------------------------------------------------------
  bool ints_of(const std::string& nm, std::vector<int64_t>& out) const {
    auto it = vid_.find(nm);
    if (it != vid_.end() && vals_[it->second].kind == Val::SHAPE) {
      out = vals_[it->second].ints;
      return vals_[it->second].known;
    }
    auto ii = m_.initializers.find(nm);
    if (ii == m_.initializers.end()) return false;
    if (!ii->second.i.empty()) out = ii->second.i;
    else {
      out.clear();
      for (float f : ii->second.f) out.push_back(static_cast<int64_t>(f));
    }
    return true;
  }

  // Shape-computation subgraph (Shape/Gather/Concat/Unsqueeze/... on int64 shapes) and Expand.
  bool lower_shape_op(int idx) {
    const Node& n = m_.nodes[idx];
    const std::string& op = n.op_type;
    if (op == "Expand") {
      if (!is_init(n.in(0))) throw std::runtime_error("Expand " + n.name + ": only initializers can be expanded");
      const auto& t = m_.initializers.at(n.in(0));
      const int C = static_cast<int>(t.dims.empty() ? 1 : t.dims.back());
      if (static_cast<int64_t>(C) != t.numel()) throw std::runtime_error("Expand " + n.name + ": expects a [1, 1, C] token");
      Val v;
      v.kind = Val::BCAST_INIT;
      v.C = C;
      v.init_name = n.in(0);
      define(n.outputs[0], v);
      return true;
    }
    if (op == "Shape") {
      const Val x = val(n.in(0), n);
      Val s;
      s.kind = Val::SHAPE;
      if (x.kind == Val::GRAPH_IN || x.kind == Val::NHWC) s.ints = {kBatchDim, x.C, x.H, x.W};
      else if (x.kind == Val::ROWS_BF16 && x.rank == 3) s.ints = {kBatchDim, x.H * x.W, x.C};
      else if (x.kind == Val::ROWS_BF16) s.ints = {kBatchDim, x.C};
      else s.known = false;
      define(n.outputs[0], s);
      return true;
    }
    bool any_shape = false;
    for (auto& in : n.inputs) {
      auto it = vid_.find(in);
      if (it != vid_.end() && vals_[it->second].kind == Val::SHAPE) any_shape = true;
    }
    if (!any_shape || op == "Reshape") return false;
    Val s;
    s.kind = Val::SHAPE;
    std::vector<int64_t> a, b;
    if (op == "Gather" && n.get_int("axis", 0) == 0) {
      s.known = ints_of(n.in(0), a) && ints_of(n.in(1), b);
      for (int64_t i : b) {
        if (!s.known) break;
        if (i < 0) i += static_cast<int64_t>(a.size());
        if (i < 0 || i >= static_cast<int64_t>(a.size())) s.known = false;
        else s.ints.push_back(a[i]);
      }
    } else if (op == "Concat") {
      for (auto& in : n.inputs) {
        if (!ints_of(in, a)) s.known = false;
        s.ints.insert(s.ints.end(), a.begin(), a.end());
      }
    } else if (op == "Unsqueeze" || op == "Squeeze" || op == "Cast" || op == "Identity") {
      s.known = ints_of(n.in(0), s.ints);
    } else {
      s.known = false;
    }
    for (auto& o : n.outputs) define(o, s);
    return true;
  }

  // Materialise an attention context (logical [B, S, nh, hd]) as rows [B, S, nh*hd].
  int emit_attention(const Val& ctx, const std::string& name) {
    const Val& q = vals_[ctx.q];
    const Val& k = vals_[ctx.k];
    const Val& v = vals_[ctx.v];
    const int S = q.H, C = q.nh * q.hd;
    if (!kern::attention_supported(q.hd, S) || k.H != S || v.H != S)
      throw std::runtime_error("attention " + name + ": needs head dim 32, 64, 80, 96 or 128 (64 and <= 256 tokens " +
                               "without the streaming kernel)");
    PlanOp p;
    p.kind = PlanOp::ATTENTION;
    p.name = name;
    p.in = q.buf;
    p.in2 = k.buf;
    p.in3 = v.buf;
    p.col[0] = q.col;
    p.col[1] = k.col;
    p.col[2] = v.col;
    p.ld[0] = q.pitch();
    p.ld[1] = k.pitch();
    p.ld[2] = v.pitch();
    p.S = S;
    p.nh = q.nh;
    p.hd = q.hd;
    p.fscale = ctx.scale;
    p.C = C;
    p.flops_per_sample = 4.0 * S * S * q.hd * q.nh;
    p.out = new_buf(static_cast<size_t>(S) * C * 2);
    const int buf = p.out;
    add_op(std::move(p));
    return buf;
  }

  void lower_reshape(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    std::vector<int64_t> shp;
    if (!ints_of(n.in(1), shp)) throw std::runtime_error("Reshape " + n.name + ": target shape must be static");
    for (auto& d : shp)
      if (d == kBatchDim) d = 0;
    auto is_batch = [](int64_t d) { return d == 0 || d == -1; };
    // NHWC map -> [B, C, H*W]
    if (x.kind == Val::NHWC && shp.size() == 3 && is_batch(shp[0]) && shp[1] == x.C &&
        (shp[2] == -1 || shp[2] == static_cast<int64_t>(x.H) * x.W) && x.H * x.W > 1) {
      Val o = x;
      o.kind = Val::NCHW_FLAT;
      define(n.outputs[0], o);
      return;
    }
    // rows [B, S, C] -> heads [B, S, nh, hd]
    if (x.kind == Val::ROWS_BF16 && shp.size() == 4 && is_batch(shp[0]) &&
        (shp[1] == 0 || shp[1] == -1 || shp[1] == x.H * x.W)) {
      const int64_t nh = shp[2], hd = shp[3];
      if (nh > 0 && hd > 0 && nh * hd == x.C) {
        Val o = x;
        o.kind = Val::HEADS;
        o.H = x.H * x.W;
        o.W = 1;
        o.nh = static_cast<int>(nh);
        o.hd = static_cast<int>(hd);
        o.perm = {{0, 1, 2, 3}};
        define(n.outputs[0], o);
        return;
      }
    }
    // attention context [B, S, nh, hd] -> rows [B, S, nh*hd]
    if (x.kind == Val::ATTN && x.stage == 2 && x.perm == std::array<int, 4>{{0, 1, 2, 3}} && shp.size() == 3 &&
        is_batch(shp[0])) {
      const Val& q = vals_[x.q];
      Val o;
      o.kind = Val::ROWS_BF16;
      o.C = q.nh * q.hd;
      o.H = q.H;
      o.rank = 3;
      o.buf = emit_attention(x, n.name);
      define(n.outputs[0], o);
      return;
    }
    // NHWC map -> [B, C*H*W] (NCHW order): the flatten view
    if (x.kind == Val::NHWC && x.H * x.W > 1 && shp.size() == 2 && is_batch(shp[0]) &&
        (shp[1] == -1 || shp[1] == static_cast<int64_t>(x.logical()) * x.H * x.W)) {
      define(n.outputs[0], flatten_nhwc(x));
      return;
    }
    // dense rows [B, S*D] <-> [B, S, D] (same memory): rank-2 <-> rank-3 views
    if (x.kind == Val::ROWS_BF16 && !x.padded() && !x.flat_hw && x.pitch() == x.C && !x.col) {
      const int64_t total = static_cast<int64_t>(x.H) * x.W * x.C;
      if (shp.size() == 3 && is_batch(shp[0])) {
        int64_t S = shp[1], D = shp[2];
        if (S == -1 && D > 0) S = total / D;
        if (D == -1 && S > 0) D = total / S;
        if (S > 0 && D > 0 && S * D == total && D % 8 == 0) {
          Val o = x;
          o.H = static_cast<int>(S);
          o.W = 1;
          o.C = static_cast<int>(D);
          o.cl = 0;
          o.rank = 3;
          define(n.outputs[0], o);
          return;
        }
      }
      if (shp.size() == 2 && is_batch(shp[0]) && (shp[1] == -1 || shp[1] == total) && total % 8 == 0) {
        Val o = x;
        o.H = o.W = 1;
        o.C = static_cast<int>(total);
        o.cl = 0;
        o.rank = 2;
        define(n.outputs[0], o);
        return;
      }
    }
    // the graph input's rows [B, S*D] -> [B, S, D] with D % 8 != 0: the input-prep pass itself writes
    // S rows of D (stored round8(D)) per sample -- the f32 input is [B*S][D] in memory already
    if (x.kind == Val::ROWS_BF16 && x.rank == 2 && consumers(n.in(0)).size() == 1 && shp.size() == 3 &&
        is_batch(shp[0]) && !graph_outputs_.count(n.in(0))) {
      for (PlanOp& q : plan_.ops)
        if (q.kind == PlanOp::ROWS_PREP && q.out == x.buf && q.rows_per_sample == 1) {
          const int64_t F = q.C;
          int64_t S = shp[1], D = shp[2];
          if (S == -1 && D > 0) S = F / D;
          if (D == -1 && S > 0) D = F / S;
          if (S <= 0 || D <= 0 || S * D != F) break;
          q.C = static_cast<int>(D);
          q.Cp = round8(static_cast<int>(D));
          q.rows_per_sample = S;
          plan_.bufs[q.out].bytes_per_sample = static_cast<size_t>(S) * q.Cp * 2 * (split_ ? 2 : 1);
          Val o = x;
          o.H = static_cast<int>(S);
          o.W = 1;
          o.C = q.Cp;
          o.cl = q.Cp != D ? static_cast<int>(D) : 0;
          o.rank = 3;
          define(n.outputs[0], o);
          return;
        }
    }
    // one row per sample [B, C] -> [B, C, 1, 1] (gates broadcast over an image: squeeze-excitation)
    if ((x.kind == Val::ROWS_BF16 || x.kind == Val::NHWC) && x.H * x.W == 1 && shp.size() == 4 && is_batch(shp[0]) &&
        shp[1] == x.logical() && shp[2] == 1 && shp[3] == 1 && !x.flat_hw) {
      Val o = x;
      o.kind = Val::NHWC;
      o.rank = 0;
      define(n.outputs[0], o);
      return;
    }
    // rows with a single row per sample -> [B, C]
    if ((x.kind == Val::ROWS_BF16 || x.kind == Val::NHWC) && x.H * x.W == 1 && shp.size() == 2) {
      Val o = x;
      o.kind = Val::ROWS_BF16;
      o.rank = 2;
      define(n.outputs[0], o);
      return;
    }
    throw std::runtime_error("Reshape " + n.name + ": unsupported reshape for the HIP engine");
  }

  void lower_transpose(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    const auto perm = n.get_ints("perm");
    if (x.kind == Val::NCHW_FLAT && perm == std::vector<int64_t>{0, 2, 1}) {
      Val o = x;  // [B, C, HW]^T = the NHWC buffer read as rows
      o.kind = Val::ROWS_BF16;
      o.H = x.H * x.W;
      o.W = 1;
      o.rank = 3;
      define(n.outputs[0], o);
      return;
    }
    if ((x.kind == Val::HEADS || (x.kind == Val::ATTN && x.stage == 2)) && perm.size() == 4) {
      Val o = x;
      for (int i = 0; i < 4; ++i) o.perm[i] = x.perm[static_cast<int>(perm[i])];
      define(n.outputs[0], o);
      return;
    }
    throw std::runtime_error("Transpose " + n.name + ": unsupported transpose for the HIP engine");
  }

  void lower_attn_matmul(int idx) {
    const Node& n = m_.nodes[idx];
    const Val a = val(n.in(0), n);
    const Val b = val(n.in(1), n);
    const std::array<int, 4> bhsd{{0, 2, 1, 3}}, bhds{{0, 2, 3, 1}};
    if (a.kind == Val::HEADS && b.kind == Val::HEADS && a.perm == bhsd && b.perm == bhds && a.nh == b.nh &&
        a.hd == b.hd) {
      Val s;
      s.kind = Val::ATTN;
      s.stage = 0;
      s.q = vid_.at(n.in(0));
      s.k = vid_.at(n.in(1));
      define(n.outputs[0], s);
      return;
    }
    if (a.kind == Val::ATTN && a.stage == 1 && b.kind == Val::HEADS && b.perm == bhsd) {
      Val c = a;
      c.stage = 2;
      c.v = vid_.at(n.in(1));
      c.perm = bhsd;
      define(n.outputs[0], c);
      return;
    }
    // general batched MatMul of two dense rank-3 row activations: [S, K] x [K, N] per sample
    if (a.kind == Val::ROWS_BF16 && b.kind == Val::ROWS_BF16 && a.rank == 3 && b.rank == 3 && dense(a) && dense(b) &&
        a.logical() == b.H * b.W) {
      PlanOp p;
      p.kind = PlanOp::BMM;
      p.name = n.name;
      p.in = a.buf;
      p.in2 = b.buf;
      p.S = static_cast<int>(rows_of(a));
      p.gidx = a.logical();
      p.ld[0] = a.C;
      p.ld[1] = b.C;
      p.C = b.C;
      p.Cp = b.logical();
      p.rows_per_sample = rows_of(a);
      p.flops_per_sample = 2.0 * p.S * p.gidx * p.Cp;
      p.out = new_buf(static_cast<size_t>(p.S) * p.C * 2);
      Val o = a;
      o.C = b.C;
      o.cl = b.cl;
      o.buf = p.out;
      o.has_affine = false;
      define(n.outputs[0], o);
      add_op(std::move(p));
      return;
    }
    throw std::runtime_error("MatMul " + n.name + ": activation x activation MatMul outside the attention pattern and the "
                             "[S, K] x [K, N] row form");
  }

  void lower_scale(int idx) {
    const Node& n = m_.nodes[idx];
    {  // standalone erf-GELU (x / sqrt2 -> Erf -> + 1 -> * x -> * 0.5) on any activation
      std::vector<int> used;
      std::string gout;
      auto xi = vid_.find(n.in(0));
      if ((n.op_type == "Div" || n.op_type == "Mul") && xi != vid_.end() &&
          (vals_[xi->second].kind == Val::NHWC || vals_[xi->second].kind == Val::ROWS_BF16) &&
          match_gelu(n.in(0), used, gout)) {
        const Val x = vals_[xi->second];
        for (int u : used) done_[u] = true;
        return emit_unary(n, x, 2, 0.f, 0.f, gout);
      }
    }
    if (lower_binary_acts(n)) return;
    auto it = m_.initializers.find(n.in(1));
    if (n.op_type != "Sub" && vid_.count(n.in(0))) {
      const Val& x = vals_[vid_.at(n.in(0))];
      if (x.kind == Val::ATTN && x.stage == 0 && it != m_.initializers.end() && it->second.f.size() == 1) {
        Val o = x;
        o.scale = n.op_type == "Div" ? x.scale / it->second.f[0] : x.scale * it->second.f[0];
        define(n.outputs[0], o);
        return;
      }
    }
    // activation (op) per-channel / scalar constant  ->  affine
    for (int side = 0; side < 2; ++side) {
      const std::string& an = n.in(side);
      const std::string& cn = n.in(1 - side);
      if (!vid_.count(an) || !is_init(cn)) continue;
      const Val& x = vals_[vid_.at(an)];
      const auto& c = m_.initializers.at(cn).f;
      if (c.size() != 1 && static_cast<int>(c.size()) != x.logical()) continue;
      std::vector<float> sc(x.C, 1.f), sh(x.C, 0.f);
      for (int k = 0; k < x.logical(); ++k) {
        const float v = c[c.size() == 1 ? 0 : k];
        if (n.op_type == "Mul") sc[k] = v;
        else if (n.op_type == "Div" && side == 0) sc[k] = 1.f / v;
        else if (n.op_type == "Sub" && side == 0) sh[k] = -v;          // x - c
        else if (n.op_type == "Sub") { sc[k] = -1.f; sh[k] = v; }      // c - x
        else throw std::runtime_error(n.op_type + " " + n.name + ": constant / activation is not supported");
      }
      return standalone_affine(n, x, &sc, &sh, nullptr);
    }
    // Sub of two activations: a - b = (-1) * b + a
    if (n.op_type == "Sub" && vid_.count(n.in(0)) && vid_.count(n.in(1))) {
      const Val a = vals_[vid_.at(n.in(0))];
      const Val b = vals_[vid_.at(n.in(1))];
      if (a.kind == b.kind && a.C == b.C && a.H == b.H && a.W == b.W && a.pitch() == a.C && b.pitch() == b.C && !a.col && !b.col) {
        std::vector<float> sc(b.C, -1.f), sh(b.C, 0.f);
        return standalone_affine(n, b, &sc, &sh, &a);
      }
    }
    throw std::runtime_error(n.op_type + " " + n.name + ": unsupported elementwise op for the HIP engine");
  }

  void lower_softmax(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    const int64_t axis = n.get_int("axis", -1);
    if (x.kind == Val::ATTN && x.stage == 0 && (axis == -1 || axis == 3)) {
      Val o = x;
      o.stage = 1;
      define(n.outputs[0], o);
      return;
    }
    const int rank = x.rank ? x.rank : 2;
    if ((x.kind == Val::ROWS_BF16 || (x.kind == Val::NHWC && x.H * x.W == 1)) && dense(x) &&
        (axis == -1 || axis == rank - 1)) {
      PlanOp p;
      p.kind = PlanOp::SOFTMAX;
      p.name = n.name;
      p.in = x.buf;
      p.C = x.logical();  // pad columns: skipped by the reduction, written 0
      p.ld_store = x.padded() ? x.C : 0;
      p.rows_per_sample = static_cast<long long>(x.H) * x.W;
      Val o = x;
      o.kind = Val::ROWS_BF16;
      o.rank = rank;
      if (graph_outputs_.count(n.outputs[0]) && consumers(n.outputs[0]).empty()) {
        p.out_f32 = kBufGraphOut;  // probabilities straight to the f32 output
        o.kind = Val::ROWS_F32;
        o.buf = kBufGraphOut;
      } else {
        p.out = new_buf(static_cast<size_t>(p.rows_per_sample) * x.C * 2);
        o.buf = p.out;
      }
      define(n.outputs[0], o);
      add_op(std::move(p));
      return;
    }
    throw std::runtime_error("Softmax " + n.name + ": only attention scores or the last axis of rows are supported");
  }

  void lower_layernorm(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    if (x.kind != Val::ROWS_BF16 || !dense(x))
      throw std::runtime_error("LayerNormalization " + n.name + ": input must be dense rows");
    const int64_t axis = n.get_int("axis", -1);
    if (!(axis == -1 || axis == (x.rank ? x.rank : 2) - 1)) throw std::runtime_error("LayerNormalization: axis must be last");
    const int Cl = x.logical();
    std::vector<float> g = init(n.in(1), n).f, b(Cl, 0.f);
    if (n.inputs.size() > 2 && !n.in(2).empty()) b = init(n.in(2), n).f;
    if (static_cast<int>(g.size()) != Cl || static_cast<int>(b.size()) != Cl)
      throw std::runtime_error("LayerNormalization " + n.name + ": scale/bias size mismatch");
    g.resize(x.C, 0.f);  // stored pad columns: written 0 by the kernel
    b.resize(x.C, 0.f);
    PlanOp p;
    p.kind = PlanOp::LAYERNORM;
    p.name = n.name;
    p.in = x.buf;
    p.scale_off = push_f32(g);
    p.shift_off = push_f32(b);
    p.eps = n.get_float("epsilon", 1e-5f);
    p.C = x.C;
    p.Cp = Cl;
    p.rows_per_sample = static_cast<long long>(x.H) * x.W;
    p.out = new_buf(static_cast<size_t>(x.H) * x.W * x.C * 2);
    Val o = x;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  void lower_gather(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    std::vector<int64_t> ix;
    const auto it = m_.initializers.find(n.in(1));
    if (x.kind == Val::ROWS_BF16 && x.rank == 3 && n.get_int("axis", 0) == 1 && it != m_.initializers.end() &&
        it->second.dims.empty() && ints_of(n.in(1), ix) && ix.size() == 1 && x.pitch() == x.C) {
      const int S = x.H * x.W;
      int64_t i = ix[0] < 0 ? ix[0] + S : ix[0];
      if (i < 0 || i >= S) throw std::runtime_error("Gather " + n.name + ": index out of range");
      PlanOp p;
      p.kind = PlanOp::GATHER_ROWS;
      p.name = n.name;
      p.in = x.buf;
      p.S = S;
      p.gidx = static_cast<int>(i);
      p.C = x.C;
      p.out = new_buf(static_cast<size_t>(x.C) * 2);
      Val o;
      o.kind = Val::ROWS_BF16;
      o.C = x.C;
      o.rank = 2;
      o.buf = p.out;
      define(n.outputs[0], o);
      add_op(std::move(p));
      return;
    }
    throw std::runtime_error("Gather " + n.name + ": only selecting one token (axis 1, scalar index) is supported");
  }

  void lower_concat(int idx) {
    const Node& n = m_.nodes[idx];
    if (n.inputs.size() == 2 && n.get_int("axis", 0) == 1) {
      const Val a = val(n.in(0), n);
      const Val b = val(n.in(1), n);
      if (a.kind == Val::BCAST_INIT && b.kind == Val::ROWS_BF16 && b.rank == 3 && a.C == b.C && b.pitch() == b.C) {
        Val o;
        o.kind = Val::TOKCAT;
        o.C = b.C;
        o.H = b.H * b.W + 1;
        o.rank = 3;
        o.init_name = a.init_name;
        o.patches = vid_.at(n.in(1));
        define(n.outputs[0], o);
        return;
      }
    }
    return general_concat(n, n.get_int("axis", 0));
  }

  // TOKCAT (+ optional position embedding initializer) -> token assembly kernel.
  void emit_tokens(const Node& n, const Val& cat, const std::string* pos_name, const std::string& out_name) {
    const Val& pt = vals_[cat.patches];
    const int S = cat.H, C = cat.C;
    PlanOp p;
    p.kind = PlanOp::TOKENS;
    p.name = n.name;
    p.in = pt.buf;
    p.S = S - 1;
    p.C = C;
    p.scale_off = push_f32(m_.initializers.at(cat.init_name).f);
    if (pos_name) {
      const auto& pos = m_.initializers.at(*pos_name);
      if (pos.numel() != static_cast<int64_t>(S) * C)
        throw std::runtime_error("Add " + n.name + ": position embedding must be [1, S, C]");
      p.shift_off = push_f32(pos.f);
    }
    p.out = new_buf(static_cast<size_t>(S) * C * 2);
    Val o;
    o.kind = Val::ROWS_BF16;
    o.C = C;
    o.H = S;
    o.rank = 3;
    o.buf = p.out;
    define(out_name, o);
    add_op(std::move(p));
  }

  // ---- Clip / grouped conv / decomposed LayerNorm / row softmax / constant binary ops ------------
  // Clip bounds from attributes (opset < 11) or the optional min/max initializer inputs.
  bool clip_bounds(const Node& n, float& lo, float& hi) const {
    lo = -3.4e38f;
    hi = 3.4e38f;
    if (n.has("min") || n.has("max")) {
      lo = n.get_float("min", lo);
      hi = n.get_float("max", hi);
      return true;
    }
    for (int k = 1; k <= 2; ++k) {
      if (n.inputs.size() <= static_cast<size_t>(k) || n.in(k).empty()) continue;
      auto it = m_.initializers.find(n.in(k));
      if (it == m_.initializers.end() || it->second.f.size() != 1) return false;
      (k == 1 ? lo : hi) = it->second.f[0];
    }
    return true;
  }

  // Activation consumer of `cur` (Relu / Clip): folds it into the producing op.
  int take_act(std::string& cur, float& lo, float& hi) {
    const int c = sole_consumer(cur);
    if (c < 0) return 0;
    const Node& a = m_.nodes[c];
    int act = 0;
    if (a.op_type == "Relu") act = 1;
    else if (a.op_type == "Clip" && clip_bounds(a, lo, hi)) act = 3;
    if (!act) return 0;
    done_[c] = true;
    cur = a.outputs[0];
    return act;
  }

  // Grouped / depthwise Conv (group > 1): direct NHWC kernel, BN folded, ReLU/Clip epilogue.
  void lower_gconv(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    if (x.kind != Val::NHWC) throw std::runtime_error("Conv " + n.name + ": grouped conv input must be an image tensor");
    const auto& wt = init(n.in(1), n);
    const int G = static_cast<int>(n.get_int("group", 1));
    const int Cout = static_cast<int>(wt.dims[0]), cpg = static_cast<int>(wt.dims[1]);
    const int KH = static_cast<int>(wt.dims[2]), KW = static_cast<int>(wt.dims[3]);
    if (cpg * G != x.C || Cout % G || Cout % 8 || x.C % 8)
      throw std::runtime_error("Conv " + n.name + ": grouped conv needs Cin = group * Cin/group and channels % 8 == 0");
    auto st = n.get_ints("strides", {1, 1});
    auto dl = n.get_ints("dilations", {1, 1});
    auto pads = conv_pads(n);
    if (st[0] != st[1] || dl[0] != dl[1]) throw std::runtime_error("Conv " + n.name + ": anisotropic stride/dilation");
    const std::string ap = n.get_string("auto_pad", "NOTSET");
    if (ap == "SAME_UPPER" || ap == "SAME_LOWER") {
      for (int d = 0; d < 2; ++d) {
        const int in = d ? x.W : x.H, k = d ? KW : KH;
        const int out = (in + static_cast<int>(st[0]) - 1) / static_cast<int>(st[0]);
        const int total = std::max(0, (out - 1) * static_cast<int>(st[0]) + (k - 1) * static_cast<int>(dl[0]) + 1 - in);
        const int lo = ap == "SAME_UPPER" ? total / 2 : total - total / 2;
        pads[d] = lo;
        pads[d + 2] = total - lo;
      }
    } else if (ap == "VALID") {
      pads = {0, 0, 0, 0};
    }
    const int s = static_cast<int>(st[0]), d = static_cast<int>(dl[0]);
    const int Ho = (x.H + static_cast<int>(pads[0] + pads[2]) - d * (KH - 1) - 1) / s + 1;
    const int Wo = (x.W + static_cast<int>(pads[1] + pads[3]) - d * (KW - 1) - 1) / s + 1;
    std::vector<float> scale(Cout, 1.f), shift(Cout, 0.f);
    if (!n.in(2).empty()) shift = init(n.in(2), n).f;
    std::string cur = n.outputs[0];
    int c1 = sole_consumer(cur);
    if (c1 >= 0 && m_.nodes[c1].op_type == "BatchNormalization") {
      std::vector<float> sc, sh;
      bn_affine(m_.nodes[c1], sc, sh);
      for (int c = 0; c < Cout; ++c) {
        scale[c] = sc[c];
        shift[c] = shift[c] * sc[c] + sh[c];
      }
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    }
    PlanOp p;
    p.kind = PlanOp::GCONV;
    p.name = n.name;
    p.in = x.buf;
    p.act = take_act(cur, p.clip_lo, p.clip_hi);
    // fp32 weights [Cout][KH][KW][cpg] with the BN scale folded
    std::vector<float> w(static_cast<size_t>(Cout) * KH * KW * cpg);
    for (int co = 0; co < Cout; ++co)
      for (int ci = 0; ci < cpg; ++ci)
        for (int ky = 0; ky < KH; ++ky)
          for (int kx = 0; kx < KW; ++kx)
            w[((static_cast<size_t>(co) * KH + ky) * KW + kx) * cpg + ci] =
                wt.f[((static_cast<size_t>(co) * cpg + ci) * KH + ky) * KW + kx] * scale[co];
    p.w_off = push_f32(w);
    p.bias_off = push_f32(shift);
    p.groups = G;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.Ho = Ho;
    p.Wo = Wo;
    p.Cp = Cout;
    p.kh = KH;
    p.kw = KW;
    p.sh = s;
    p.sw = d;  // dilation
    p.ph = static_cast<int>(pads[0]);
    p.pw = static_cast<int>(pads[1]);
    p.flops_per_sample = 2.0 * Ho * Wo * Cout * KH * KW * cpg;
    p.out = new_buf(static_cast<size_t>(Ho) * Wo * Cout * 2);
    Val o;
    o.kind = Val::NHWC;
    o.C = Cout;
    o.H = Ho;
    o.W = Wo;
    o.buf = p.out;
    define(cur, o);
    add_op(std::move(p));
  }

  void lower_clip(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    float lo, hi;
    if (!clip_bounds(n, lo, hi)) throw std::runtime_error("Clip " + n.name + ": bounds must be constants");
    standalone_affine(n, x, nullptr, nullptr, nullptr, 3, lo, hi);
  }

  static int64_t last_axis_of(const Node& n, const onnx::Model& m, bool& ok) {
    std::vector<int64_t> ax = n.get_ints("axes");
    if (ax.empty() && n.inputs.size() > 1 && !n.in(1).empty()) {
      auto it = m.initializers.find(n.in(1));
      if (it != m.initializers.end()) ax = it->second.i;
    }
    ok = ax.size() == 1 && n.get_int("keepdims", 1) == 1;
    return ok ? ax[0] : 0;
  }

  // torch's LayerNorm export below opset 17: ReduceMean -> Sub -> Pow(2) -> ReduceMean -> Add(eps)
  // -> Sqrt -> Div [-> Mul(gamma)] [-> Add(beta)]  ==> one LAYERNORM op.
  // ReduceMean / ReduceSum / ReduceMax over the spatial axes of an image or the token axis of
  // rows: the GAP kernel in mode 0 / 1 / 2.  False when the reduction is some other one.
  bool lower_spatial_reduce(int idx, int mode) {
    const Node& n = m_.nodes[idx];
    const Val x = materialize_in(n.in(0), n);
    std::vector<int64_t> ax = n.get_ints("axes");
    if (ax.empty() && n.inputs.size() > 1 && !n.in(1).empty()) ints_of(n.in(1), ax);
    std::sort(ax.begin(), ax.end());
    const bool keep = n.get_int("keepdims", 1) != 0;
    const bool spatial = x.kind == Val::NHWC && (ax == std::vector<int64_t>{2, 3} || ax == std::vector<int64_t>{-2, -1});
    const bool tokens = x.kind == Val::ROWS_BF16 && x.rank == 3 && (ax == std::vector<int64_t>{1} || ax == std::vector<int64_t>{-2});
    if (!(spatial || tokens) || !dense(x)) return false;
    PlanOp p;
    p.kind = PlanOp::GAP;
    p.gidx = mode;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.out = new_buf(static_cast<size_t>(x.C) * 2);
    Val o;
    o.kind = spatial && keep ? Val::NHWC : Val::ROWS_BF16;
    o.C = x.C;
    o.cl = x.cl;
    o.rank = tokens && keep ? 3 : 2;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
    return true;
  }

  void lower_reduce_mean(int idx) {
    const Node& n = m_.nodes[idx];
    if (lower_spatial_reduce(idx, 0)) return;
    const Val x = val(n.in(0), n);
    auto fail = [&](const std::string& why) {
      throw std::runtime_error("ReduceMean " + n.name + ": only the decomposed LayerNormalization pattern is supported (" +
                               why + ")");
    };
    bool ok;
    const int64_t axis = last_axis_of(n, m_, ok);
    const int rank = x.rank ? x.rank : 2;
    if (!ok || !(axis == -1 || axis == rank - 1)) fail("reduction over the last axis with keepdims");
    if (x.kind != Val::ROWS_BF16 || x.pitch() != x.C || x.col) fail("input must be dense rows");
    const std::string& xn = n.in(0);
    const std::string& mu = n.outputs[0];
    int sub = -1;
    for (int c : consumers(mu))
      if (m_.nodes[c].op_type == "Sub" && m_.nodes[c].in(0) == xn && m_.nodes[c].in(1) == mu) sub = c;
    if (sub < 0) fail("no x - mean");
    const std::string& d = m_.nodes[sub].outputs[0];
    int sq = -1, div = -1;
    for (int c : consumers(d)) {
      const Node& q = m_.nodes[c];
      if ((q.op_type == "Pow" && q.in(0) == d && scalar_is(q.in(1), 2.f)) || (q.op_type == "Mul" && q.in(0) == d && q.in(1) == d))
        sq = c;
      else if (q.op_type == "Div" && q.in(0) == d)
        div = c;
    }
    if (sq < 0 || div < 0) fail("no variance / normalisation");
    const int rm2 = sole_consumer(m_.nodes[sq].outputs[0]);
    if (rm2 < 0 || m_.nodes[rm2].op_type != "ReduceMean") fail("no variance mean");
    const int add = sole_consumer(m_.nodes[rm2].outputs[0]);
    if (add < 0 || m_.nodes[add].op_type != "Add") fail("no variance + eps");
    const std::string eps_name = other_input(m_.nodes[add], m_.nodes[rm2].outputs[0]);
    auto ei = m_.initializers.find(eps_name);
    if (ei == m_.initializers.end() || ei->second.f.size() != 1) fail("eps must be a scalar constant");
    const int sq_rt = sole_consumer(m_.nodes[add].outputs[0]);
    if (sq_rt < 0 || m_.nodes[sq_rt].op_type != "Sqrt" || m_.nodes[div].in(1) != m_.nodes[sq_rt].outputs[0])
      fail("no sqrt feeding the division");
    std::vector<float> g(x.C, 1.f), b(x.C, 0.f);
    std::string cur = m_.nodes[div].outputs[0];
    std::vector<int> used = {sub, sq, rm2, add, sq_rt, div};
    int c = sole_consumer(cur);
    if (c >= 0 && m_.nodes[c].op_type == "Mul" && is_init(other_input(m_.nodes[c], cur)) &&
        static_cast<int>(m_.initializers.at(other_input(m_.nodes[c], cur)).f.size()) == x.C) {
      g = m_.initializers.at(other_input(m_.nodes[c], cur)).f;
      used.push_back(c);
      cur = m_.nodes[c].outputs[0];
      c = sole_consumer(cur);
    }
    if (c >= 0 && m_.nodes[c].op_type == "Add" && is_init(other_input(m_.nodes[c], cur)) &&
        static_cast<int>(m_.initializers.at(other_input(m_.nodes[c], cur)).f.size()) == x.C) {
      b = m_.initializers.at(other_input(m_.nodes[c], cur)).f;
      used.push_back(c);
      cur = m_.nodes[c].outputs[0];
    }
    if (x.padded()) fail("C % 8 == 0 (stored pad columns)");
    for (int u : used) done_[u] = true;
    PlanOp p;
    p.kind = PlanOp::LAYERNORM;
    p.name = n.name + "+decomposed_layernorm";
    p.in = x.buf;
    p.scale_off = push_f32(g);
    p.shift_off = push_f32(b);
    p.eps = ei->second.f[0];
    p.C = x.C;
    p.rows_per_sample = static_cast<long long>(x.H) * x.W;
    p.out = new_buf(static_cast<size_t>(x.H) * x.W * x.C * 2);
    Val o = x;
    o.buf = p.out;
    define(cur, o);
    add_op(std::move(p));
  }

  // Explicit pads of a conv plus those of a zero Pad folded into it (lower_pad).
  std::vector<int64_t> conv_pads(const Node& n) const {
    auto pads = n.get_ints("pads", {0, 0, 0, 0});
    if (pads.size() != 4) throw std::runtime_error("Conv " + n.name + ": expected 4 pads");
    auto it = folded_pad_.find(n.in(0));
    if (it != folded_pad_.end())
      for (int k = 0; k < 4; ++k) pads[k] += it->second[k];
    return pads;
  }

  // Pad (constant mode, value 0, spatial axes of an NHWC image only, /root/reference has no Pad
  // kernel -- ONNX Runtime's CPU EP runs it there).  A Pad whose only reader is a Conv with explicit
  // pads folds into that conv (the conv kernels read out-of-range pixels as zero); otherwise one
  // NHWC pad pass writes the padded image.
  // ZeroInsert (domain "die", from rewrite_conv_transpose): the same pass with strides: zeros between
  // the input's pixels and `pads` = [top, left, bottom, right] around them.
  void lower_pad(int idx) {
    const Node& n = m_.nodes[idx];
    int sy = 1, sx = 1;
    std::array<int64_t, 4> tlbr{};
    if (n.op_type == "ZeroInsert") {
      const auto st = n.get_ints("strides", {1, 1}), pd = n.get_ints("pads", {0, 0, 0, 0});
      sy = static_cast<int>(st.at(0));
      sx = static_cast<int>(st.at(1));
      for (int k = 0; k < 4; ++k) tlbr[k] = pd.at(k);
      const Val x = materialize_in(n.in(0), n);
      if (x.kind != Val::NHWC || !dense(x)) throw std::runtime_error("ConvTranspose " + n.name + ": input must be an image");
      return emit_pad(n, x, tlbr, sy, sx);
    }
    if (n.get_string("mode", "constant") != "constant") throw std::runtime_error("Pad " + n.name + ": only constant mode");
    std::vector<int64_t> pads = n.get_ints("pads");
    float value = n.get_float("value", 0.f);
    if (pads.empty() && n.inputs.size() >= 2) ints_of(n.in(1), pads);
    if (n.inputs.size() >= 3 && !n.in(2).empty()) {
      const auto& cv = init(n.in(2), n);
      value = cv.f.empty() ? (cv.i.empty() ? 0.f : static_cast<float>(cv.i[0])) : cv.f[0];
    }
    if (n.inputs.size() >= 4 && !n.in(3).empty()) throw std::runtime_error("Pad " + n.name + ": the axes input is not supported");
    if (value != 0.f) throw std::runtime_error("Pad " + n.name + ": only zero padding");
    const Val x = materialize_in(n.in(0), n);
    if (x.kind != Val::NHWC || pads.size() != 8 || pads[0] || pads[1] || pads[4] || pads[5])
      throw std::runtime_error("Pad " + n.name + ": only the spatial axes of an [N, C, H, W] image");
    for (auto v : pads)
      if (v < 0) throw std::runtime_error("Pad " + n.name + ": negative pads (cropping) are not supported");
    tlbr = {{pads[2], pads[3], pads[6], pads[7]}};
    emit_pad(n, x, tlbr, 1, 1);
  }

  void emit_pad(const Node& n, const Val& x, const std::array<int64_t, 4>& tlbr, int sy, int sx) {
    const int c = sole_consumer(n.outputs[0]);
    if (sy == 1 && sx == 1 && c >= 0 && m_.nodes[c].op_type == "Conv" && m_.nodes[c].in(0) == n.outputs[0] &&
        m_.nodes[c].get_string("auto_pad", "NOTSET") == "NOTSET") {
      folded_pad_[n.outputs[0]] = tlbr;
      define(n.outputs[0], x);
      return;
    }
    PlanOp p;
    p.kind = PlanOp::PAD;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.ph = static_cast<int>(tlbr[0]);
    p.pw = static_cast<int>(tlbr[1]);
    p.sh = sy;
    p.sw = sx;
    p.Ho = (x.H - 1) * sy + 1 + static_cast<int>(tlbr[0] + tlbr[2]);
    p.Wo = (x.W - 1) * sx + 1 + static_cast<int>(tlbr[1] + tlbr[3]);
    p.out = new_buf(static_cast<size_t>(p.Ho) * p.Wo * x.C * 2);
    Val o = x;
    o.H = p.Ho;
    o.W = p.Wo;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  bool scalar_init(const std::string& name, float& v) const {
    auto it = m_.initializers.find(name);
    if (it == m_.initializers.end() || it->second.numel() != 1) return false;
    v = it->second.f.empty() ? static_cast<float>(it->second.i.at(0)) : it->second.f[0];
    return true;
  }

  // Comparisons (bool results are stored as 1 / 0 activations): two activations -> a binary op,
  // an activation and a scalar constant -> a unary code (the constant on the left mirrors the test).
  void lower_compare(int idx) {
    const Node& n = m_.nodes[idx];
    static const std::map<std::string, int> codes = {
        {"Greater", 18}, {"Less", 19}, {"Equal", 20}, {"GreaterOrEqual", 21}, {"LessOrEqual", 22}};
    float c = 0.f;
    if (scalar_init(n.in(1), c)) return emit_unary(n, materialize_in(n.in(0), n), codes.at(n.op_type), c, 0.f, n.outputs[0]);
    if (scalar_init(n.in(0), c)) {
      int code = codes.at(n.op_type);
      code = code == 18 ? 19 : code == 19 ? 18 : code == 21 ? 22 : code == 22 ? 21 : code;
      return emit_unary(n, materialize_in(n.in(1), n), code, c, 0.f, n.outputs[0]);
    }
    if (lower_binary_acts(n)) return;
    throw std::runtime_error(n.op_type + " " + n.name + ": only two activations of one shape or one and a scalar");
  }

  // Where(cond, a, b): cond an activation; a / b activations of cond's shape or scalar constants.
  void lower_where(int idx) {
    const Node& n = m_.nodes[idx];
    const Val c = materialize_in(n.in(0), n);
    if (!dense(c)) throw std::runtime_error("Where " + n.name + ": the condition must be a dense activation");
    PlanOp p;
    p.kind = PlanOp::WHERE;
    p.name = n.name;
    p.in = c.buf;
    float* sv[2] = {&p.clip_lo, &p.clip_hi};
    int* bufs[2] = {&p.in2, &p.in3};
    const Val* like = &c;
    Val vb[2];
    for (int k = 0; k < 2; ++k) {
      if (scalar_init(n.in(1 + k), *sv[k])) continue;
      vb[k] = materialize_in(n.in(1 + k), n);
      if (!dense(vb[k]) || vb[k].kind != c.kind || vb[k].H != c.H || vb[k].W != c.W || vb[k].C != c.C ||
          vb[k].logical() != c.logical())
        throw std::runtime_error("Where " + n.name + ": the branches must be scalars or activations of the condition's shape");
      *bufs[k] = vb[k].buf;
      like = &vb[k];
    }
    p.C = c.C;
    p.Cp = c.logical();
    p.rows_per_sample = rows_of(c);
    p.out = new_buf(static_cast<size_t>(rows_of(c)) * c.C * 2);
    Val o = *like;
    o.buf = p.out;
    o.has_affine = false;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  // Cast of an activation: to a float type -> the same values; to bool -> v != 0.  Integer targets
  // would need rounding the stored representation cannot express exactly: rejected.
  void lower_cast(int idx) {
    const Node& n = m_.nodes[idx];
    const int to = static_cast<int>(n.get_int("to", onnx::FLOAT));
    if (to == onnx::BOOL) return emit_unary(n, materialize_in(n.in(0), n), 24, 0.f, 0.f, n.outputs[0]);
    if (!onnx::is_float_type(to)) throw std::runtime_error("Cast " + n.name + ": only casts to float types or bool");
    define(n.outputs[0], val(n.in(0), n));
  }

  // Resize (opset 10+: scales / sizes inputs) and Upsample (scales attribute or input) of an
  // image: nearest or linear over H, W.
  void lower_resize(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = materialize_in(n.in(0), n);
    if (x.kind != Val::NHWC || !dense(x)) throw std::runtime_error(n.op_type + " " + n.name + ": only images");
    const std::string mode = n.get_string("mode", "nearest");
    if (mode != "nearest" && mode != "linear" && mode != "bilinear")
      throw std::runtime_error(n.op_type + " " + n.name + ": mode " + mode + " is not supported (nearest, linear)");
    if (n.get_int("antialias", 0) != 0) throw std::runtime_error(n.op_type + " " + n.name + ": antialias is not supported");
    if (n.has("axes")) throw std::runtime_error(n.op_type + " " + n.name + ": the axes attribute is not supported");
    std::vector<float> scales = n.get_floats("scales");
    std::vector<int64_t> sizes;
    const bool upsample = n.op_type == "Upsample";
    auto floats_of = [&](const std::string& nm) {
      auto it = m_.initializers.find(nm);
      if (it == m_.initializers.end()) throw std::runtime_error(n.op_type + " " + n.name + ": scales must be a constant");
      return it->second.f;
    };
    if (scales.empty()) {
      if (upsample && n.inputs.size() >= 2) scales = floats_of(n.in(1));
      if (!upsample && n.inputs.size() == 2 && !n.in(1).empty()) scales = floats_of(n.in(1));  // opset 10
      if (!upsample && n.inputs.size() >= 3 && !n.in(2).empty() && !floats_of(n.in(2)).empty()) scales = floats_of(n.in(2));
      if (!upsample && scales.empty() && n.inputs.size() >= 4 && !n.in(3).empty() && !ints_of(n.in(3), sizes))
        throw std::runtime_error(n.op_type + " " + n.name + ": sizes must be known at load time");
    }
    float sh, sw;
    int Ho, Wo;
    if (!sizes.empty()) {
      if (sizes.size() != 4 || (sizes[1] != x.logical() && sizes[1] != kBatchDim))
        throw std::runtime_error(n.op_type + " " + n.name + ": sizes must be [N, C, H, W] with C unchanged");
      Ho = static_cast<int>(sizes[2]);
      Wo = static_cast<int>(sizes[3]);
      sh = static_cast<float>(Ho) / x.H;
      sw = static_cast<float>(Wo) / x.W;
    } else {
      if (scales.size() != 4 || scales[0] != 1.f || scales[1] != 1.f)
        throw std::runtime_error(n.op_type + " " + n.name + ": scales must be [1, 1, sh, sw]");
      sh = scales[2];
      sw = scales[3];
      Ho = static_cast<int>(std::floor(x.H * static_cast<double>(sh)));
      Wo = static_cast<int>(std::floor(x.W * static_cast<double>(sw)));
    }
    if (Ho < 1 || Wo < 1 || !(sh > 0.f) || !(sw > 0.f)) throw std::runtime_error(n.op_type + " " + n.name + ": empty output");
    static const std::map<std::string, int> coords = {{"half_pixel", 0}, {"asymmetric", 1}, {"align_corners", 2},
                                                      {"pytorch_half_pixel", 3}, {"tf_half_pixel_for_nn", 4}};
    static const std::map<std::string, int> nearests = {
        {"round_prefer_floor", 0}, {"round_prefer_ceil", 1}, {"floor", 2}, {"ceil", 3}};
    // Upsample and opset-10 Resize: asymmetric coordinates, floor rounding for nearest
    const bool legacy = upsample || m_.opset() < 11;
    const std::string cm = legacy ? "asymmetric" : n.get_string("coordinate_transformation_mode", "half_pixel");
    const std::string nm = legacy ? "floor" : n.get_string("nearest_mode", "round_prefer_floor");
    if (!coords.count(cm) || !nearests.count(nm))
      throw std::runtime_error(n.op_type + " " + n.name + ": coordinate mode " + cm + " / nearest mode " + nm + " is not supported");
    PlanOp p;
    p.kind = PlanOp::RESIZE;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.Ho = Ho;
    p.Wo = Wo;
    p.clip_lo = sh;
    p.clip_hi = sw;
    p.gidx = coords.at(cm);
    p.act = mode == "nearest" ? 0 : 1;
    p.is_max = nearests.at(nm);
    p.out = new_buf(static_cast<size_t>(Ho) * Wo * x.C * 2);
    Val o = x;
    o.H = Ho;
    o.W = Wo;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  // Channel range [s0, e0) of a dense image / rows value -> a column copy (s0 % 8 == 0).
  void emit_channel_slice(const Node& n, const Val& x, int64_t s0, int64_t e0, const std::string& out) {
    const int len = static_cast<int>(e0 - s0), Cs = round8(len);
    PlanOp p;
    p.kind = PlanOp::COPY_COLS;
    p.name = n.name;
    p.in = x.buf;
    p.col[0] = static_cast<int>(s0);
    p.ld[0] = x.C;
    p.col[1] = 0;
    p.ld[1] = Cs;
    p.C = std::min(Cs, x.C - static_cast<int>(s0));
    p.rows_per_sample = rows_of(x);
    p.out = new_buf(static_cast<size_t>(rows_of(x)) * Cs * 2);
    Val o = x;
    o.C = Cs;
    o.cl = Cs != len ? len : 0;
    o.buf = p.out;
    define(out, o);
    add_op(std::move(p));
  }

  // Split along the channel axis (sizes from the attribute, the input, or equal parts): one column
  // copy per output; every boundary but the end must be a multiple of 8.
  void lower_split(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = materialize_in(n.in(0), n);
    const int64_t axis = n.get_int("axis", 0);
    if (!dense(x) || !is_channel_axis(x, axis))
      throw std::runtime_error("Split " + n.name + ": only along the channel axis of an image or rows");
    std::vector<int64_t> sizes = n.get_ints("split");
    if (sizes.empty() && n.inputs.size() >= 2 && !n.in(1).empty()) ints_of(n.in(1), sizes);
    const int64_t Cl = x.logical(), parts = static_cast<int64_t>(n.outputs.size());
    if (sizes.empty()) {
      const int64_t each = (Cl + parts - 1) / parts;  // equal parts (opset 18: the last may be smaller)
      for (int64_t k = 0, s = 0; k < parts; ++k, s += each) sizes.push_back(std::min(each, Cl - s));
    }
    if (static_cast<int64_t>(sizes.size()) != parts) throw std::runtime_error("Split " + n.name + ": sizes/outputs mismatch");
    int64_t s0 = 0;
    for (int64_t k = 0; k < parts; ++k) {
      if (s0 % 8 || sizes[k] <= 0 || s0 + sizes[k] > Cl)
        throw std::runtime_error("Split " + n.name + ": parts must start at multiples of 8 channels");
      if (!n.outputs[k].empty()) emit_channel_slice(n, x, s0, s0 + sizes[k], n.outputs[k]);
      s0 += sizes[k];
    }
    if (s0 != Cl) throw std::runtime_error("Split " + n.name + ": sizes do not cover the axis");
  }

  // Slice of one token along axis 1 of [B, S, C] rows (e.g. the cls token) -> row gather; a channel
  // range -> a column copy.
  void lower_slice(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = val(n.in(0), n);
    std::vector<int64_t> starts = n.get_ints("starts"), ends = n.get_ints("ends"), axes = n.get_ints("axes"), steps;
    if (starts.empty() && n.inputs.size() >= 3) {  // opset >= 10: inputs
      ints_of(n.in(1), starts);
      ints_of(n.in(2), ends);
      if (n.inputs.size() > 3 && !n.in(3).empty()) ints_of(n.in(3), axes);
      if (n.inputs.size() > 4 && !n.in(4).empty()) ints_of(n.in(4), steps);
    }
    if (axes.empty())
      for (size_t i = 0; i < starts.size(); ++i) axes.push_back(static_cast<int64_t>(i));
    const int S = x.H * x.W;
    if (x.kind == Val::ROWS_BF16 && x.rank == 3 && x.pitch() == x.C && starts.size() == 1 && ends.size() == 1 &&
        axes.size() == 1 && axes[0] == 1 && (steps.empty() || steps[0] == 1)) {
      int64_t s0 = starts[0] < 0 ? starts[0] + S : starts[0];
      int64_t e0 = ends[0] < 0 ? ends[0] + S : std::min<int64_t>(ends[0], S);
      if (s0 >= 0 && e0 == s0 + 1) {
        PlanOp p;
        p.kind = PlanOp::GATHER_ROWS;
        p.name = n.name;
        p.in = x.buf;
        p.S = S;
        p.gidx = static_cast<int>(s0);
        p.C = x.C;
        p.out = new_buf(static_cast<size_t>(x.C) * 2);
        Val o;
        o.kind = Val::ROWS_BF16;
        o.C = x.C;
        o.H = 1;
        o.rank = 3;
        o.buf = p.out;
        define(n.outputs[0], o);
        add_op(std::move(p));
        return;
      }
    }
    // channel-axis slice [start, end) with start % 8 == 0: a column copy
    if (dense(x) && starts.size() == 1 && ends.size() == 1 && axes.size() == 1 && is_channel_axis(x, axes[0]) &&
        (steps.empty() || steps[0] == 1)) {
      const int64_t Cl = x.logical();
      int64_t s0 = starts[0] < 0 ? starts[0] + Cl : std::min<int64_t>(starts[0], Cl);
      int64_t e0 = ends[0] < 0 ? ends[0] + Cl : std::min<int64_t>(ends[0], Cl);
      if (s0 >= 0 && e0 > s0 && s0 % 8 == 0 && (e0 % 8 == 0 || e0 == Cl)) {
        emit_channel_slice(n, x, s0, e0, n.outputs[0]);
        return;
      }
    }
    throw std::runtime_error("Slice " + n.name + ": supported: one token along axis 1 of [B, S, C] rows, or a channel "
                             "range starting at a multiple of 8");
  }

  void lower_bn(int idx) {
    const Node& n = m_.nodes[idx];
    Val& x = val(n.in(0), n);
    std::vector<float> sc, sh;
    bn_affine(n, sc, sh);
    if (x.kind == Val::GRAPH_IN) {  // fold into input prep
      Val v = x;
      if (v.has_affine) {
        for (size_t c = 0; c < sc.size(); ++c) {
          v.ash[c] = v.ash[c] * sc[c] + sh[c];
          v.asc[c] *= sc[c];
        }
      } else {
        v.has_affine = true;
        v.asc = sc;
        v.ash = sh;
      }
      define(n.outputs[0], v);
      return;
    }
    sc.resize(x.C, 1.f);
    sh.resize(x.C, 0.f);
    standalone_affine(n, x, &sc, &sh, nullptr);
  }

  void lower_relu(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = materialize_in(n.in(0), n);
    standalone_affine(n, x, nullptr, nullptr, nullptr);
  }

  void lower_add(int idx) {
    const Node& n = m_.nodes[idx];
    // [cls, patches] + position embedding -> token assembly
    for (int side = 0; side < 2; ++side) {
      auto it = vid_.find(n.in(side));
      if (it != vid_.end() && vals_[it->second].kind == Val::TOKCAT && is_init(n.in(1 - side))) {
        const Val cat = vals_[it->second];
        return emit_tokens(n, cat, &n.in(1 - side), n.outputs[0]);
      }
    }
    for (int side = 0; side < 2; ++side) {  // activation + per-channel / scalar constant
      if (!vid_.count(n.in(side)) || !is_init(n.in(1 - side))) continue;
      const Val& x = vals_[vid_.at(n.in(side))];
      const auto& c = m_.initializers.at(n.in(1 - side)).f;
      if (c.size() != 1 && static_cast<int>(c.size()) != x.logical()) continue;
      std::vector<float> sc(x.C, 1.f), sh(x.C, 0.f);
      for (int k = 0; k < x.logical(); ++k) sh[k] = c[c.size() == 1 ? 0 : k];
      return standalone_affine(n, x, &sc, &sh, nullptr);
    }
    for (int side = 0; side < 2; ++side)
      if (vid_.count(n.in(side)) && vals_[vid_.at(n.in(side))].kind == Val::GRAPH_IN) materialize_in(n.in(side), n);
    if (lower_binary_acts(n)) return;
    const Val a = val(n.in(0), n);
    const Val b = val(n.in(1), n);
    if (a.pitch() != a.C || b.pitch() != b.C || a.col || b.col)
      throw std::runtime_error("Add " + n.name + ": strided operands are not supported");
    if (a.kind != b.kind || a.C != b.C || a.H != b.H || a.W != b.W)
      throw std::runtime_error("Add " + n.name + ": broadcasting adds are not supported by the HIP engine");
    standalone_affine(n, a, nullptr, nullptr, &b);
  }

  // ---- general path: any-activation unary, broadcast binary, concat / slice -----------------------
  static bool dense(const Val& v) { return (v.kind == Val::NHWC || v.kind == Val::ROWS_BF16) && v.pitch() == v.C && !v.col && !v.flat_hw; }
  static long long rows_of(const Val& v) { return static_cast<long long>(v.H) * v.W; }

  void lower_unary(int idx) {
    const Node& n = m_.nodes[idx];
    const Val x = materialize_in(n.in(0), n);
    const std::string& op = n.op_type;
    if (op == "Gelu" && n.get_string("approximate", "none") != "none")
      throw std::runtime_error("Gelu " + n.name + ": only the exact (erf) form is supported");
    static const std::map<std::string, int> codes = {
        {"Gelu", 2}, {"Sigmoid", 4}, {"Tanh", 5}, {"LeakyRelu", 6}, {"Exp", 7}, {"Abs", 8}, {"Sqrt", 9}, {"Neg", 10},
        {"Reciprocal", 11}, {"Log", 12}, {"Erf", 13}, {"Pow", 14}, {"HardSigmoid", 15}, {"HardSwish", 16}, {"Softplus", 17}};
    const int act = codes.at(op);
    float a = 0.f, b = 0.f;
    if (op == "LeakyRelu") a = n.get_float("alpha", 0.01f);
    if (op == "HardSigmoid") {
      a = n.get_float("alpha", 0.2f);
      b = n.get_float("beta", 0.5f);
    }
    if (op == "Pow") {  // activation ^ scalar constant
      auto it = m_.initializers.find(n.in(1));
      if (it == m_.initializers.end() || it->second.f.size() != 1)
        throw std::runtime_error("Pow " + n.name + ": the exponent must be a scalar constant");
      a = it->second.f[0];
    }
    emit_unary(n, x, act, a, b, n.outputs[0]);
  }

  void emit_unary(const Node& n, const Val& x, int act, float a, float b, const std::string& out_name) {
    if (!dense(x)) throw std::runtime_error(n.op_type + " " + n.name + ": input must be a dense image or rows tensor");
    PlanOp p;
    p.kind = PlanOp::UNARY;
    p.name = n.name;
    p.in = x.buf;
    p.act = act;
    p.clip_lo = a;
    p.clip_hi = b;
    p.C = x.C;
    p.Cp = x.logical();  // pad columns are written 0 (exp(0) = 1, 1/0 = inf must not reach a GEMM)
    p.rows_per_sample = rows_of(x);
    p.out = new_buf(static_cast<size_t>(rows_of(x)) * x.C * 2);
    Val o = x;
    o.buf = p.out;
    o.has_affine = false;
    define(out_name, o);
    add_op(std::move(p));
  }

  // Add / Sub / Mul / Div of two activations: same shape, or the second one broadcast per sample
  // ([B, C, 1, 1] or [B, C] gates over an image's pixels / a sequence's rows: squeeze-excitation,
  // GLU-style gating).  Returns false when the operands do not fit (the caller tries other forms).
  bool lower_binary_acts(const Node& n) {
    if (n.inputs.size() != 2 || !vid_.count(n.in(0)) || !vid_.count(n.in(1))) return false;
    const std::string& t = n.op_type;
    static const std::map<std::string, int> ops = {
        {"Add", 0}, {"Sub", 1}, {"Mul", 2}, {"Div", 3}, {"Max", 4}, {"Min", 5}, {"Or", 4}, {"And", 5},
        {"Greater", 6}, {"Less", 7}, {"Equal", 8}, {"GreaterOrEqual", 9}, {"LessOrEqual", 10}};
    auto oi = ops.find(t);
    if (oi == ops.end()) return false;
    int op = oi->second;
    for (int side = 0; side < 2; ++side)
      if (vals_[vid_.at(n.in(side))].kind == Val::GRAPH_IN) materialize_in(n.in(side), n);
    Val a = vals_[vid_.at(n.in(0))], b = vals_[vid_.at(n.in(1))];
    if (!dense(a) || !dense(b) || a.C != b.C || a.logical() != b.logical()) return false;
    int ymode;
    if (a.kind == b.kind && a.H == b.H && a.W == b.W) {
      if (op == 0) return false;  // plain same-shape Add: the affine kernel's residual path
      ymode = 0;
    } else if (rows_of(b) == 1 && rows_of(a) > 1) {
      ymode = 1;
    } else if (rows_of(a) == 1 && rows_of(b) > 1 && op != 1 && op != 3) {
      std::swap(a, b);  // broadcast operand second: commutative ops, comparisons mirrored
      if (op >= 6) op = op == 6 ? 7 : op == 7 ? 6 : op == 9 ? 10 : op == 10 ? 9 : op;
      ymode = 1;
    } else {
      return false;
    }
    std::string cur = n.outputs[0];
    float lo = 0.f, hi = 0.f;
    PlanOp p;
    p.kind = PlanOp::BINARY;
    p.name = n.name;
    p.in = a.buf;
    p.in2 = b.buf;
    p.gidx = op;
    p.S = ymode;
    p.act = take_act(cur, lo, hi);
    p.clip_lo = lo;
    p.clip_hi = hi;
    p.C = a.C;
    p.Cp = a.logical();  // pad columns are written 0 (Div of two zero pads would be NaN)
    p.rows_per_sample = rows_of(a);
    p.out = new_buf(static_cast<size_t>(rows_of(a)) * a.C * 2);
    Val o = a;
    o.buf = p.out;
    o.has_affine = false;
    define(cur, o);
    add_op(std::move(p));
    return true;
  }

  // The channel axis of a value (NHWC: NCHW axis 1; rows: the last axis) for Concat / Slice.
  static bool is_channel_axis(const Val& v, int64_t axis) {
    if (v.kind == Val::NHWC) return axis == 1 || axis == -3;
    const int r = v.rank ? v.rank : 2;
    return v.kind == Val::ROWS_BF16 && (axis == -1 || axis == r - 1);
  }

  void general_concat(const Node& n, int64_t axis) {
    std::vector<Val> xs;
    for (auto& in : n.inputs) xs.push_back(val(in, n));
    int Cs = 0, Cl = 0;
    for (size_t i = 0; i < xs.size(); ++i) {
      const Val& v = xs[i];
      if (!dense(v) || !is_channel_axis(v, axis) || v.kind != xs[0].kind || v.H != xs[0].H || v.W != xs[0].W)
        throw std::runtime_error("Concat " + n.name + ": inputs must be dense tensors of one shape, joined on the channel axis");
      if (i + 1 < xs.size() && v.padded())
        throw std::runtime_error("Concat " + n.name + ": only the last input may have a channel count that is not a multiple of 8");
      Cs += i + 1 < xs.size() ? v.logical() : v.C;
      Cl += v.logical();
    }
    const int out = new_buf(static_cast<size_t>(rows_of(xs[0])) * Cs * 2);
    int col = 0;
    for (size_t i = 0; i < xs.size(); ++i) {
      PlanOp p;
      p.kind = PlanOp::COPY_COLS;
      p.name = n.name + "#" + std::to_string(i);
      p.in = xs[i].buf;
      p.out = out;
      p.col[0] = 0;
      p.ld[0] = xs[i].C;
      p.col[1] = col;
      p.ld[1] = Cs;
      p.C = xs[i].C;
      p.rows_per_sample = rows_of(xs[0]);
      add_op(std::move(p));
      col += xs[i].logical();
    }
    Val o = xs[0];
    o.C = Cs;
    o.cl = Cl != Cs ? Cl : 0;
    o.buf = out;
    define(n.outputs[0], o);
  }

  void standalone_affine(const Node& n, const Val& x, const std::vector<float>* sc, const std::vector<float>* sh,
                         const Val* z, int own_act = 0, float own_lo = 0.f, float own_hi = 0.f) {
    if (x.kind != Val::NHWC && x.kind != Val::ROWS_BF16)
      throw std::runtime_error(n.op_type + " " + n.name + ": unsupported input layout");
    if (x.C % 8) throw std::runtime_error(n.op_type + " " + n.name + ": channels must be a multiple of 8");
    if (x.pitch() != x.C || x.col) throw std::runtime_error(n.op_type + " " + n.name + ": strided operand");
    std::string cur = n.outputs[0];
    int act = n.op_type == "Relu" ? 1 : own_act;
    float lo = own_lo, hi = own_hi;
    if (!act) act = take_act(cur, lo, hi);
    PlanOp p;
    p.clip_lo = lo;
    p.clip_hi = hi;
    p.kind = PlanOp::AFFINE;
    p.name = n.name;
    p.in = x.buf;
    p.in2 = z ? z->buf : -1;
    if (sc) {
      p.scale_off = push_f32(*sc);
      p.shift_off = push_f32(*sh);
    }
    p.act = act;
    p.C = x.C;
    p.rows_per_sample = static_cast<long long>(x.H) * x.W;
    p.out = new_buf(static_cast<size_t>(x.H) * x.W * x.C * 2);
    Val o = x;
    o.buf = p.out;
    o.has_affine = false;
    define(cur, o);
    add_op(std::move(p));
  }

  void lower_pool(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = materialize_in(n.in(0), n);
    if (x.kind != Val::NHWC) throw std::runtime_error(n.op_type + " " + n.name + ": input must be an image tensor");
    auto k = n.get_ints("kernel_shape");
    auto st = n.get_ints("strides", {1, 1});
    auto pads = n.get_ints("pads", {0, 0, 0, 0});
    const bool cip_avg = n.op_type == "AveragePool" && n.get_int("count_include_pad", 0);
    if ((pads[0] != pads[2] || pads[1] != pads[3]) && cip_avg)
      throw std::runtime_error(n.op_type + " " + n.name + ": count_include_pad with asymmetric pads is not supported");
    const bool ceil_mode = n.get_int("ceil_mode", 0) != 0;
    auto od = [&](int in, int d) {
      double v = static_cast<double>(in + pads[d] + pads[d + 2] - k[d]) / st[d];
      return static_cast<int>(ceil_mode ? std::ceil(v) : std::floor(v)) + 1;
    };
    PlanOp p;
    p.kind = PlanOp::POOL;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.Ho = od(x.H, 0);
    p.Wo = od(x.W, 1);
    p.kh = static_cast<int>(k[0]);
    p.kw = static_cast<int>(k[1]);
    p.sh = static_cast<int>(st[0]);
    p.sw = static_cast<int>(st[1]);
    p.ph = static_cast<int>(pads[0]);
    p.pw = static_cast<int>(pads[1]);
    p.is_max = n.op_type == "MaxPool";
    p.cip = static_cast<int>(n.get_int("count_include_pad", 0));
    p.out = new_buf(static_cast<size_t>(p.Ho) * p.Wo * x.C * 2);
    Val o = x;
    o.H = p.Ho;
    o.W = p.Wo;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  // GlobalAveragePool (mode 0) / GlobalMaxPool (mode 2)
  void lower_gap(int idx, int mode = 0) {
    const Node& n = m_.nodes[idx];
    Val x = materialize_in(n.in(0), n);
    if (x.kind != Val::NHWC) throw std::runtime_error(n.op_type + ": input must be an image tensor");
    PlanOp p;
    p.kind = PlanOp::GAP;
    p.gidx = mode;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.out = new_buf(static_cast<size_t>(x.C) * 2);
    Val o;
    o.kind = Val::NHWC;  // [C,1,1]
    o.C = x.C;
    o.cl = x.cl;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  void lower_flatten(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = val(n.in(0), n);
    if (n.op_type == "Flatten" && n.get_int("axis", 1) != 1) throw std::runtime_error("Flatten: axis must be 1");
    if (x.kind == Val::NHWC && x.H * x.W > 1 && n.op_type == "Flatten") {
      define(n.outputs[0], flatten_nhwc(x));
      return;
    }
    if (!((x.kind == Val::ROWS_BF16 || x.kind == Val::NHWC) && x.H == 1 && x.W == 1))
      throw std::runtime_error(n.op_type + " " + n.name + ": only flattening of 1x1 feature maps is supported");
    Val o = x;
    o.kind = Val::ROWS_BF16;
    o.rank = 2;
    define(n.outputs[0], o);
  }

  // [B, C, H, W] -> [B, C*H*W] over an NHWC buffer: a lazy view in (h, w, c) order that only a
  // Gemm/MatMul with an initializer can consume (it permutes its weight rows to match).
  Val flatten_nhwc(const Val& x) const {
    Val o;
    o.kind = Val::ROWS_BF16;
    o.rank = 2;
    o.C = x.H * x.W * x.C;
    o.buf = x.buf;
    o.flat_hw = x.H * x.W;
    o.flat_c = x.logical();
    return o;
  }

  void finalize_output() {
    const std::string& name = m_.outputs[0].name;
    auto it = vid_.find(name);
    if (it == vid_.end()) throw std::runtime_error("graph output " + name + " is not produced");
    Val v = vals_[it->second];
    if (v.kind == Val::TOKCAT) {  // never materialised by a consumer
      emit_tokens(m_.nodes[0], v, nullptr, name + "#tokens");
      v = vals_[vid_.at(name + "#tokens")];
    }
    if (v.kind == Val::ROWS_F32 && v.buf == kBufGraphOut) {
      plan_.output_shape = {1, v.logical()};
      if (v.rank == 3) plan_.output_shape = {1, v.H, v.logical()};
    } else if (v.kind == Val::ROWS_BF16 || (v.kind == Val::NHWC && v.H == 1 && v.W == 1 &&
                                           m_.outputs[0].dims.size() == 2)) {
      PlanOp p;
      p.kind = PlanOp::BF16_TO_F32;
      p.name = "output_cast";
      if (v.pitch() != v.C || v.col || v.flat_hw) throw std::runtime_error("graph output is a strided view");
      p.in = v.buf;
      // padded rows: [rows][logical] f32 from rows of pitch C
      p.C = v.padded() ? v.logical() : v.C * v.H * v.W;
      p.ld_store = v.padded() ? v.C : 0;
      p.rows_per_sample = v.padded() ? static_cast<long long>(v.H) * v.W : 1;
      p.out_f32 = kBufGraphOut;
      add_op(std::move(p));
      plan_.output_shape = {1, v.logical()};
      if (v.kind == Val::ROWS_BF16 && v.rank == 3) plan_.output_shape = {1, v.H * v.W, v.logical()};
    } else if (v.kind == Val::NHWC) {
      PlanOp p;
      p.kind = PlanOp::TO_NCHW_F32;
      p.name = "output_nchw";
      p.in = v.buf;
      p.C = v.logical();
      p.ld_store = v.padded() ? v.C : 0;
      p.H = v.H;
      p.W = v.W;
      p.out_f32 = kBufGraphOut;
      add_op(std::move(p));
      plan_.output_shape = {1, v.logical(), v.H, v.W};
    } else {
      throw std::runtime_error("unsupported graph output layout");
    }
    plan_.output_numel = 1;
    for (auto dim : plan_.output_shape) plan_.output_numel *= static_cast<size_t>(dim);
  }

  // Pool -> BN(+ReLU) where the pooled value has no other reader (ResNet-v2: the stem's max pool
  // feeds only stage 1's pre-activation BN, the first unit having a projection shortcut): the pool
  // kernel applies the per-channel affine and activation before its single store.
  void fuse_pool_affine() {
    std::vector<int> readers(plan_.bufs.size(), 0);
    for (const PlanOp& p : plan_.ops)
      for (int b : {p.in, p.in2, p.in3})
        if (b >= 0) readers[b]++;
    std::vector<PlanOp> out;
    out.reserve(plan_.ops.size());
    for (size_t i = 0; i < plan_.ops.size(); ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind == PlanOp::AFFINE && p.in2 < 0 && p.in >= 0 && readers[p.in] == 1 && !out.empty() &&
          out.back().kind == PlanOp::POOL && out.back().out == p.in && out.back().scale_off == SIZE_MAX &&
          out.back().act == 0 && p.rows_per_sample == static_cast<long long>(out.back().Ho) * out.back().Wo) {
        PlanOp& pool = out.back();
        pool.scale_off = p.scale_off;
        pool.shift_off = p.shift_off;
        pool.act = p.act;
        pool.out = p.out;
        pool.name += "+" + p.name;
        continue;
      }
      out.push_back(std::move(p));
    }
    plan_.ops = std::move(out);
  }

  // Stem -> 3x3/2 max pool (pad 1) [-> the pooled value's BN/ReLU, fuse_pool_affine] where the stem
  // map has no other reader: one STEM op with is_max = 1 (kernels/stem.hip stem_pool_nchw_kernel);
  // the stem map is never stored.  Ho/Wo become the pooled size, s2_off/b2_off/act the pool's affine.
  void fuse_stem_pool() {
    std::vector<int> readers(plan_.bufs.size(), 0);
    for (const PlanOp& p : plan_.ops)
      for (int b : {p.in, p.in2, p.in3})
        if (b >= 0) readers[b]++;
    std::vector<PlanOp> out;
    out.reserve(plan_.ops.size());
    for (size_t i = 0; i < plan_.ops.size(); ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind == PlanOp::POOL && p.is_max && p.kh == 3 && p.kw == 3 && p.sh == 2 && p.sw == 2 && p.ph == 1 &&
          p.pw == 1 && p.act <= 1 && p.C == 64 && p.in >= 0 && readers[p.in] == 1 && !out.empty()) {
        PlanOp& s = out.back();
        const auto& c = s.conv;
        if (s.kind == PlanOp::STEM && s.in == kBufGraphIn && !s.is_max && s.out == p.in && c.Ho == p.H && c.Wo == p.W &&
            kern::stem_pool_supported(c.H, c.W, c.Ho, c.Wo, p.Ho, p.Wo, split_)) {
          permute_weight_rows(s.w_off, 64, 224, c.wplane);
          s.is_max = 1;
          s.Ho = p.Ho;
          s.Wo = p.Wo;
          s.s2_off = p.scale_off;
          s.b2_off = p.shift_off;
          s.act = p.act;
          s.out = p.out;
          s.name += "+" + p.name;
          continue;
        }
      }
      out.push_back(std::move(p));
    }
    plan_.ops = std::move(out);
  }

  // Global pool -> the FC head (Gemm / 1x1 conv over the pooled [C] vector) that is its ONLY reader,
  // with an fp32 output (a buffer or the graph output, directly or through a BF16_TO_F32 op) and no
  // residual / second output: one GAP_FC op at the pool's position
  // (kernels/misc.hip gap_fc_kernel); the pooled vector is never stored.
  void fuse_gap_fc() {
    std::vector<int> readers(plan_.bufs.size(), 0), reader_op(plan_.bufs.size(), -1);
    const int nops = static_cast<int>(plan_.ops.size());
    for (int i = 0; i < nops; ++i)
      for (int b : {plan_.ops[i].in, plan_.ops[i].in2, plan_.ops[i].in3})
        if (b >= 0) {
          readers[b]++;
          reader_op[b] = i;
        }
    std::vector<bool> drop(nops, false);
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind != PlanOp::GAP || p.out < 0 || p.out2 >= 0 || p.out_f32 != -1 || p.join >= 0 || p.in < 0 ||
          readers[p.out] != 1)
        continue;
      const int j = reader_op[p.out];
      if (j <= i || drop[j]) continue;
      const PlanOp& q = plan_.ops[j];
      const kern::ConvArgs& c = q.conv;
      if (q.kind != PlanOp::CONV || q.in != p.out || q.in2 >= 0 || q.in3 >= 0 || q.out2 >= 0 || q.join >= 0 ||
          c.relu > 1 || q.in_scale_off != SIZE_MAX || c.KH != 1 || c.KW != 1 || c.H != 1 || c.W != 1 ||
          c.Cin != p.C || c.K != p.C)
        continue;
      // the f32 logits come from the conv itself, or (N % 8 != 0) from the BF16_TO_F32 op that is
      // the only reader of its bf16 output -- the fused op writes them directly, in fp32
      int conv_out = -1, nout = c.N, k = -1;
      if (q.out_f32 != -1 && q.out < 0) {
        conv_out = q.out_f32;
      } else if (q.out_f32 == -1 && q.out >= 0 && readers[q.out] == 1) {
        k = reader_op[q.out];
        const PlanOp& r = plan_.ops[k];
        if (k <= j || drop[k] || r.kind != PlanOp::BF16_TO_F32 || r.in != q.out || r.out_f32 == -1 || r.join >= 0 ||
            (r.ld_store > 0 && r.rows_per_sample != 1) || r.C > c.N)
          continue;
        conv_out = r.out_f32;
        nout = r.C;
      } else {
        continue;
      }
      if (!kern::gap_fc_slice(p.C, max_batch_, nout, kern::kSplitKWorkspaceBytes)) continue;
      p.kind = PlanOp::GAP_FC;
      p.name += "+" + q.name;
      p.conv = c;
      p.Cp = nout;  // logits per sample (= the f32 row pitch)
      p.w_off = q.w_off;
      p.bias_off = q.bias_off;
      p.act = c.relu;
      p.out = -1;  // the pooled buffer is dropped (no op references it any more)
      p.out_f32 = conv_out;
      p.flops_per_sample += q.flops_per_sample;
      drop[j] = true;
      if (k >= 0) drop[k] = true;
    }
    std::vector<PlanOp> out;
    out.reserve(plan_.ops.size());
    for (int i = 0; i < nops; ++i)
      if (!drop[i]) out.push_back(std::move(plan_.ops[i]));
    plan_.ops = std::move(out);
  }

  // LayerNorm -> GEMMs (ViT / BERT pre-norm blocks: the norm feeds the QKV or the first MLP GEMM
  // only).  LN(x) W + b = rstd (x (gamma W) - mean colsum(gamma W)) + (beta W + b) per row, so the
  // GEMMs read x itself with gamma folded into their weights, beta into their bias, and apply the
  // per-row (mean, rstd) in the epilogue (ConvArgs::row_stats); the LayerNorm only computes the
  // statistics -- the normalised rows are never written or read.  Exact in real arithmetic; in
  // fp32 the error grows with |mean| / std of a row (ViT residual rows: mean ~ 0).
  double weight_at(size_t w_off, long long plane, int kpad, int n, int k) const {
    const uint16_t* w = reinterpret_cast<const uint16_t*>(plan_.params.data() + w_off);
    const size_t i = static_cast<size_t>(n) * kpad + k;
    double v = from_bf16(w[i]);
    if (plane > 0) v += from_bf16(w[i + plane]);
    return v;
  }
  void set_weight(size_t w_off, long long plane, int kpad, int n, int k, float v) {
    uint16_t* w = reinterpret_cast<uint16_t*>(plan_.params.data() + w_off);
    const size_t i = static_cast<size_t>(n) * kpad + k;
    const uint16_t hi = to_bf16(v);
    w[i] = hi;
    if (plane > 0) w[i + plane] = to_bf16(v - static_cast<float>(from_bf16(hi)));
  }
  void fold_layernorm() {
    const int nops = static_cast<int>(plan_.ops.size());
    std::vector<std::vector<int>> readers(plan_.bufs.size());
    for (int i = 0; i < nops; ++i)
      for (int b : {plan_.ops[i].in, plan_.ops[i].in2, plan_.ops[i].in3})
        if (b >= 0) readers[b].push_back(i);
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind != PlanOp::LAYERNORM || p.stats_only || p.out < 0 || p.in < 0 || p.C != p.Cp || p.join >= 0 ||
          readers[p.out].empty())
        continue;
      bool ok = true;
      for (int j : readers[p.out]) {
        const PlanOp& q = plan_.ops[j];
        const kern::ConvArgs& c = q.conv;
        ok = ok && j > i && q.kind == PlanOp::CONV && q.in == p.out && q.in2 != p.out && q.in3 < 0 && q.join < 0 &&
             q.in_scale_off == SIZE_MAX && c.KH == 1 && c.KW == 1 && c.stride == 1 && c.pad_h == 0 && c.pad_w == 0 &&
             c.K == p.C && c.Cin == p.C && c.Kpad == c.K && c.Ho * c.Wo == p.rows_per_sample;
      }
      if (!ok) continue;
      const float* gamma = reinterpret_cast<const float*>(plan_.params.data() + p.scale_off);
      const float* beta = reinterpret_cast<const float*>(plan_.params.data() + p.shift_off);
      const std::vector<float> g(gamma, gamma + p.C), be(beta, beta + p.C);
      const int stats = new_buf(static_cast<size_t>(p.rows_per_sample) * 2 * 4);
      for (int j : readers[p.out]) {
        PlanOp& q = plan_.ops[j];
        const kern::ConvArgs& c = q.conv;
        const int Npad = static_cast<int>(round_up(c.N, 128));
        std::vector<float> bias(Npad, 0.f), colsum(round_up(c.N, 8), 0.f);
        if (q.bias_off != SIZE_MAX) {
          const float* b0 = reinterpret_cast<const float*>(plan_.params.data() + q.bias_off);
          std::copy(b0, b0 + c.N, bias.begin());
        }
        for (int n = 0; n < c.N; ++n) {
          double bsum = bias[n], csum = 0.0;
          for (int k = 0; k < c.K; ++k) {
            const double w = weight_at(q.w_off, c.wplane, c.Kpad, n, k);
            bsum += static_cast<double>(be[k]) * w;
            set_weight(q.w_off, c.wplane, c.Kpad, n, k, static_cast<float>(w * g[k]));
            csum += weight_at(q.w_off, c.wplane, c.Kpad, n, k);  // what the GEMM multiplies by
          }
          bias[n] = static_cast<float>(bsum);
          colsum[n] = static_cast<float>(csum);
        }
        bias.resize(round_up(c.N, 8));
        q.bias_off = push_f32(bias);
        q.colsum_off = push_f32(colsum);
        q.conv.bias = nullptr;
        q.in = p.in;
        q.in3 = stats;
        q.name = p.name + "+" + q.name;
      }
      p.stats_only = 1;
      p.out = stats;
    }
  }

  // Statistics-only LayerNorm whose input is the stored output of a rows GEMM (ViT pre-norm
  // blocks: the attention-out and MLP2 GEMMs, residual add in their epilogue) -> deleted.  That GEMM
  // also writes per-(row, 64-column group) (mean, M2) partials from the values it holds in registers
  // (ConvArgs::stats_out), and every block of a folded reader merges its rows' groups in a fixed
  // order while its first operand tiles load (ConvArgs::row_parts): no launch, no re-read of the rows.
  // The block-0 LayerNorm's input comes from the token assembly, which emits the same partials.
  void stats_from_producer() {
    const int nops = static_cast<int>(plan_.ops.size());
    std::vector<std::vector<int>> readers(plan_.bufs.size());
    for (int i = 0; i < nops; ++i)
      for (int b : {plan_.ops[i].in, plan_.ops[i].in2, plan_.ops[i].in3})
        if (b >= 0) readers[b].push_back(i);
    std::vector<int> writer(plan_.bufs.size(), -1);  // latest op writing each buffer
    std::vector<bool> drop(nops, false);
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      const int w = p.kind == PlanOp::LAYERNORM && p.stats_only && p.in >= 0 ? writer[p.in] : -1;
      if (w >= 0 && p.C == p.Cp && p.C % 64 == 0 && p.C <= 2048 && p.join < 0) {
        PlanOp& q = plan_.ops[w];
        const kern::ConvArgs& c = q.conv;
        // rows GEMM (attention-out / MLP2), or the token assembly (block 0)
        const bool gemm = q.kind == PlanOp::CONV && c.N == p.C && c.Ho * c.Wo == p.rows_per_sample && q.out2 < 0;
        const bool tokens = q.kind == PlanOp::TOKENS && q.C == p.C && q.S + 1 == p.rows_per_sample;
        bool ok = (gemm || tokens) && q.out == p.in && q.out_stats < 0 && q.join < 0;
        for (int j : readers[p.out]) {
          const PlanOp& r = plan_.ops[j];
          ok = ok && j > i && r.kind == PlanOp::CONV && r.in3 == p.out && r.colsum_off != SIZE_MAX &&
               r.conv.N % 8 == 0 && r.conv.K == p.C && r.join < 0;
        }
        if (ok && !readers[p.out].empty()) {
          const int st = new_buf(static_cast<size_t>(p.rows_per_sample) * (p.C / 64) * 2 * 4);
          q.out_stats = st;
          q.name += "+stats";
          for (int j : readers[p.out]) {
            PlanOp& r = plan_.ops[j];
            r.in3 = st;
            r.in3_parts = 1;
            r.eps = p.eps;
          }
          drop[i] = true;
        }
      }
      for (int b : {p.out, p.out2, p.out3, p.out_f32})
        if (b >= 0) writer[b] = i;
    }
    std::vector<PlanOp> out;
    out.reserve(plan_.ops.size());
    for (int i = 0; i < nops; ++i)
      if (!drop[i]) out.push_back(std::move(plan_.ops[i]));
    plan_.ops = std::move(out);
  }

  // Back-to-back 1x1 pair (ResNet-v2 bottleneck boundary).  A dual-store expand conv P writes the
  // raw sum x (next residual) and a = act(bn(x)); when a's ONLY reader is a plain 1x1/s1 reduce conv
  // Q, both become one CONV_PAIR op at P's position (Q has no other input, so computing it early is
  // safe) and `a` is never stored: kernels/conv_pair.hip consumes it from LDS.  Rows of both weight
  // matrices are permuted in place (kern::pair_permute_row) -- P and Q exist only inside the pair.
  void permute_weight_rows(size_t off, int rows, int kpad, long long plane) {
    const int planes = plane > 0 ? 2 : 1;
    std::vector<uint16_t> tmp(static_cast<size_t>(rows) * kpad);
    for (int pl = 0; pl < planes; ++pl) {
      uint16_t* w = reinterpret_cast<uint16_t*>(plan_.params.data() + off) + static_cast<size_t>(pl) * plane;
      std::memcpy(tmp.data(), w, tmp.size() * 2);
      for (int n = 0; n < rows; ++n)
        std::memcpy(w + static_cast<size_t>(kern::pair_permute_row(n)) * kpad, tmp.data() + static_cast<size_t>(n) * kpad,
                    static_cast<size_t>(kpad) * 2);
    }
  }
  static bool plain_1x1(const kern::ConvArgs& c) {
    return c.KH == 1 && c.KW == 1 && c.stride == 1 && c.pad_h == 0 && c.pad_w == 0 && c.dil == 1 && c.H == c.Ho &&
           c.W == c.Wo && c.K == c.Cin && c.Kpad == c.K;
  }
  // With other readers of `a` (a stage boundary: the next stage's projection shortcut reads it
  // too) the pair also stores a (PlanOp::out3) and those readers keep reading it.
  // Reduce widths up to 128: the kernel takes 256 (stage 2 -> 3) but at one block per CU it is
  // faster than the two convs only at small batches (B=20: 43.3 vs 51.1 us; B=32: 76.4 vs 69.1).
  static constexpr int kMaxPairN2 = 128;
  void fuse_conv_pairs() {
    const int nops = static_cast<int>(plan_.ops.size());
    std::vector<std::vector<int>> readers(plan_.bufs.size());
    for (int i = 0; i < nops; ++i)
      for (int b : {plan_.ops[i].in, plan_.ops[i].in2, plan_.ops[i].in3})
        if (b >= 0) readers[b].push_back(i);
    std::vector<bool> drop(nops, false);
    auto reduce_ok = [&](const PlanOp& p, const PlanOp& q) {
      return q.kind == PlanOp::CONV && q.in == p.out2 && q.in2 < 0 && q.in3 < 0 && q.out >= 0 && q.out2 < 0 &&
             q.out_f32 < 0 && q.conv.relu <= 1 && q.in_scale_off == SIZE_MAX && plain_1x1(q.conv) &&
             q.conv.Cin == p.conv.N && q.conv.H == p.conv.Ho && q.conv.W == p.conv.Wo && q.join < 0 &&
             q.conv.N <= kMaxPairN2 && kern::conv_pair_supported(p.conv.K, p.conv.N, q.conv.N);
    };
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind != PlanOp::CONV || p.in2 < 0 || p.out2 < 0 || p.s2_off == SIZE_MAX || p.out_f32 >= 0 ||
          p.conv.relu != 0 || p.in_scale_off != SIZE_MAX || !plain_1x1(p.conv) || p.join >= 0)
        continue;
      const std::vector<int>& rd = readers[p.out2];
      int j = -1;
      for (int r : rd)
        if (r > i && !drop[r] && reduce_ok(p, plan_.ops[r])) {
          j = r;
          break;
        }
      if (j < 0) continue;
      bool others_ok = true;  // every other reader runs after the pair (at P's position) and reads a as an input
      for (int r : rd)
        if (r != j && (r <= i || plan_.ops[r].join >= 0)) others_ok = false;
      if (!others_ok) continue;
      const PlanOp& q = plan_.ops[j];
      permute_weight_rows(p.w_off, static_cast<int>(round_up(p.conv.N, 128)), p.conv.Kpad, p.conv.wplane);
      permute_weight_rows(q.w_off, static_cast<int>(round_up(q.conv.N, 128)), q.conv.Kpad, q.conv.wplane);
      p.kind = PlanOp::CONV_PAIR;
      p.name += "+" + q.name;
      p.w2_off = q.w_off;
      p.bias2_off = q.bias_off;
      p.w2plane = q.conv.wplane;
      p.n2 = q.conv.N;
      p.pair_relu = q.conv.relu;
      p.out3 = rd.size() > 1 ? p.out2 : -1;  // a stored for its other readers, else dropped
      p.out2 = q.out;
      p.flops_per_sample += q.flops_per_sample;
      drop[j] = true;
    }
    std::vector<PlanOp> out;
    out.reserve(plan_.ops.size());
    for (int i = 0; i < nops; ++i)
      if (!drop[i]) out.push_back(std::move(plan_.ops[i]));
    plan_.ops = std::move(out);
  }

  // Pre-activation on load (opt-in, EngineOptions::bn_on_load).  A dual-store conv writes x (the raw sum: next residual) AND
  // a = act(bn(x)) (the next unit's input).  When every reader of `a` is a 1x1 conv the LDS-DMA
  // loop can run (K = Cin <= 2048, Cin % 64 == 0), those convs read x and apply bn+act to their
  // operand fragments instead, and the producer stores x only: one activation-sized write and
  // read fewer per unit (ResNet-v2 expand convs are store-bound).
  void preact_on_load() {
    const int nops = static_cast<int>(plan_.ops.size());
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      if (p.kind != PlanOp::CONV || p.out < 0 || p.out2 < 0 || p.s2_off == SIZE_MAX) continue;
      std::vector<int> readers;
      bool ok = true;
      for (int k = 0; k < nops && ok; ++k) {
        if (k == i) continue;
        const PlanOp& q = plan_.ops[k];
        if (q.in2 == p.out2 || q.in3 == p.out2 || q.out == p.out2 || q.out2 == p.out2) ok = false;
        if (q.in != p.out2) continue;
        const kern::ConvArgs& c = q.conv;
        ok = q.kind == PlanOp::CONV && c.KH == 1 && c.KW == 1 && c.pad_h == 0 && c.pad_w == 0 && c.K == c.Cin &&
             c.Cin % 64 == 0 && c.K <= 2048 && q.in_scale_off == SIZE_MAX;
        readers.push_back(k);
      }
      if (!ok || readers.empty()) continue;
      for (int k : readers) {
        PlanOp& q = plan_.ops[k];
        q.in = p.out;
        q.in_scale_off = p.s2_off;
        q.in_shift_off = p.b2_off;
        q.in_relu = p.conv.relu2;
      }
      p.out2 = -1;
      p.s2_off = p.b2_off = SIZE_MAX;
      p.conv.relu2 = 0;
    }
  }

  // Branch concurrency: a conv whose output is first consumed two or more ops later (ResNet's
  // projection shortcut: consumed as the residual of the unit's expand conv, after the reduce and
  // 3x3 convs) is independent of the ops in between.  At serving batch sizes every one of those
  // convs is latency-bound and leaves CUs idle, so the engine runs the branch on a second stream
  // and joins it at its consumer.  One branch open at a time.
  void mark_side_branches() {
    const int nops = static_cast<int>(plan_.ops.size());
    int open_until = -1;
    for (int i = 0; i < nops; ++i) {
      PlanOp& p = plan_.ops[i];
      if (i <= open_until || p.kind != PlanOp::CONV || p.out < 0 || p.out_f32 >= 0 || p.out_stats >= 0) continue;
      int j = -1;
      for (int k = i + 1; k < nops && j < 0; ++k) {
        const PlanOp& q = plan_.ops[k];
        for (int b : {q.in, q.in2, q.in3})
          if (b >= 0 && (b == p.out || b == p.out2)) j = k;
      }
      if (j < i + 2) continue;
      p.join = j;
      open_until = j;
    }
  }

  void assign_arena() {
    const int nops = static_cast<int>(plan_.ops.size());
    for (int i = 0; i < nops; ++i) {
      const PlanOp& p = plan_.ops[i];
      for (int b : {p.out, p.out2, p.out3, p.out_stats})
        if (b >= 0 && plan_.bufs[b].first_use < 0) plan_.bufs[b].first_use = i;
      for (int b : {p.in, p.in2, p.in3, p.out, p.out2, p.out3, p.out_stats})
        if (b >= 0) plan_.bufs[b].last_use = std::max(plan_.bufs[b].last_use, i);
      // a side branch may still be reading its inputs until its join
      if (p.join >= 0)
        for (int b : {p.in, p.in2, p.in3})
          if (b >= 0) plan_.bufs[b].last_use = std::max(plan_.bufs[b].last_use, p.join);
    }
    // Offsets: greedy by size (largest first, each at the lowest offset that does not overlap an
    // already placed buffer whose lifetime intersects its own) -- for ResNet50 this packs the
    // arena ~1.5x tighter than first-fit in program order, which keeps activations + weights inside
    // the 256 MiB Infinity Cache.
    std::vector<int> order;
    for (size_t i = 0; i < plan_.bufs.size(); ++i)
      if (plan_.bufs[i].first_use >= 0 || plan_.bufs[i].last_use >= 0) order.push_back(static_cast<int>(i));
    auto bytes_of = [&](int bi) { return round_up(plan_.bufs[bi].bytes_per_sample * max_batch_, 256); };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return bytes_of(a) > bytes_of(b); });
    struct Placed {
      size_t off, size;
      int first, last;
    };
    std::vector<Placed> placed;
    size_t top = 0;
    for (int bi : order) {
      PlanBuf& b = plan_.bufs[bi];
      const size_t size = bytes_of(bi);
      const int first = b.first_use < 0 ? 0 : b.first_use;
      const int last = std::max(b.last_use, first);
      std::vector<std::pair<size_t, size_t>> busy;  // ranges of lifetime-overlapping buffers
      for (const Placed& q : placed)
        if (q.first <= last && first <= q.last) busy.emplace_back(q.off, q.off + q.size);
      std::sort(busy.begin(), busy.end());
      size_t cand = 0;
      for (const auto& r : busy) {
        if (r.first >= cand + size) break;
        cand = std::max(cand, r.second);
      }
      b.offset = cand;
      placed.push_back(Placed{cand, size, first, last});
      top = std::max(top, cand + size);
    }
    plan_.arena_bytes = top;
    double fl = 0;
    for (auto& p : plan_.ops) fl += p.flops_per_sample;
    plan_.flops_per_sample = fl;
  }

  const onnx::Model& m_;
  int max_batch_;
  bool side_branches_ = false;
  bool split_ = false;  // fp32 mode: split (hi, lo) activations and weights
  bool bn_on_load_ = false;  // EngineOptions::bn_on_load (bf16 plans only)
  bool fuse_pairs_ = true;   // EngineOptions::fuse_pairs
  bool fuse_stem_pool_ = true;  // EngineOptions::fuse_stem_pool
  bool fuse_gap_fc_ = false;    // EngineOptions::fuse_gap_fc
  bool fold_layernorm_ = true;  // EngineOptions::fold_layernorm
  bool ln_stats_epilogue_ = true;  // EngineOptions::ln_stats_epilogue
  Plan plan_;
  std::vector<Val> vals_;
  std::unordered_map<std::string, int> vid_;
  std::unordered_map<std::string, std::vector<int>> consumers_;
  std::unordered_set<std::string> graph_outputs_;
  std::unordered_map<std::string, int> prepped_;
  std::unordered_map<std::string, std::array<int64_t, 4>> folded_pad_;  // Pad output -> (t, l, b, r) for its conv
  std::vector<bool> done_;
};

}  // namespace

std::string Plan::summary() const {
  std::ostringstream os;
  size_t convs = 0;
  for (auto& o : ops) convs += o.kind == PlanOp::CONV || o.kind == PlanOp::STEM || o.kind == PlanOp::CONV_PAIR;
  os << ops.size() << " device ops (" << convs << " MFMA conv/gemm), arena " << arena_bytes / (1 << 20) << " MiB, params "
     << params.size() / (1 << 20) << " MiB, " << flops_per_sample / 1e9 << " GFLOP/sample";
  return os.str();
}

namespace {

onnx::Attribute ints_attr(const std::string& name, std::vector<int64_t> v) {
  onnx::Attribute a;
  a.name = name;
  a.type = onnx::Attribute::INTS;
  a.ints = std::move(v);
  return a;
}

bool has_conv_transpose(const onnx::Model& m) {
  for (const auto& n : m.nodes)
    if (n.op_type == "ConvTranspose" && n.domain.empty()) return true;
  return false;
}

// ConvTranspose (2-D, group 1, dilation 1, explicit pads, weights an initializer) -> ZeroInsert +
// Conv: the input with stride - 1 zeros between its pixels and k - 1 - p zero borders (+ the output
// padding at the end), convolved at stride 1 with the transposed, flipped kernel -- the MFMA conv
// path instead of a scatter kernel.  Other ConvTranspose forms are left for the planner to report.
onnx::Model rewrite_conv_transpose(const onnx::Model& src) {
  onnx::Model m = src;
  std::vector<onnx::Node> out;
  for (const auto& n : src.nodes) {
    auto wi = m.initializers.find(n.in(1));
    bool ok = n.op_type == "ConvTranspose" && n.domain.empty() && wi != m.initializers.end() && wi->second.dims.size() == 4 &&
              n.get_int("group", 1) == 1 && !n.has("output_shape") && n.get_string("auto_pad", "NOTSET") == "NOTSET";
    const auto dl = n.get_ints("dilations", {1, 1}), st = n.get_ints("strides", {1, 1});
    const auto pd = n.get_ints("pads", {0, 0, 0, 0}), op = n.get_ints("output_padding", {0, 0});
    ok = ok && dl.size() == 2 && dl[0] == 1 && dl[1] == 1 && st.size() == 2 && pd.size() == 4 && op.size() == 2;
    if (!ok) {
      out.push_back(n);
      continue;
    }
    const auto& w = wi->second;
    const int64_t Cin = w.dims[0], Cout = w.dims[1], kh = w.dims[2], kw = w.dims[3];
    const std::vector<int64_t> zp = {kh - 1 - pd[0], kw - 1 - pd[1], kh - 1 - pd[2] + op[0], kw - 1 - pd[3] + op[1]};
    if (*std::min_element(zp.begin(), zp.end()) < 0) {  // cropping transposed convs: not rewritten
      out.push_back(n);
      continue;
    }
    onnx::Node zi;
    zi.name = n.name + "/zero_insert";
    zi.op_type = "ZeroInsert";
    zi.domain = "die";
    zi.inputs = {n.in(0)};
    zi.outputs = {n.outputs.at(0) + "/zero_insert"};
    zi.attrs["strides"] = ints_attr("strides", st);
    zi.attrs["pads"] = ints_attr("pads", zp);
    onnx::Tensor cw;
    cw.name = n.in(1) + "/as_conv";
    cw.dims = {Cout, Cin, kh, kw};
    cw.f.resize(static_cast<size_t>(Cout * Cin * kh * kw));
    for (int64_t ci = 0; ci < Cin; ++ci)
      for (int64_t co = 0; co < Cout; ++co)
        for (int64_t y = 0; y < kh; ++y)
          for (int64_t x = 0; x < kw; ++x)
            cw.f[((co * Cin + ci) * kh + y) * kw + x] = w.f[((ci * Cout + co) * kh + (kh - 1 - y)) * kw + (kw - 1 - x)];
    m.initializers[cw.name] = cw;
    onnx::Node cv;
    cv.name = n.name;
    cv.op_type = "Conv";
    cv.inputs = {zi.outputs[0], cw.name};
    if (!n.in(2).empty()) cv.inputs.push_back(n.in(2));
    cv.outputs = n.outputs;
    cv.attrs["kernel_shape"] = ints_attr("kernel_shape", {kh, kw});
    cv.attrs["strides"] = ints_attr("strides", {1, 1});
    cv.attrs["pads"] = ints_attr("pads", {0, 0, 0, 0});
    cv.attrs["dilations"] = ints_attr("dilations", {1, 1});
    out.push_back(std::move(zi));
    out.push_back(std::move(cv));
  }
  m.nodes = std::move(out);
  return m;
}

}  // namespace

Plan build_plan(const onnx::Model& m, int max_batch, bool side_branches, bool split, bool bn_on_load, bool fuse_pairs,
                bool fuse_stem_pool, bool fuse_gap_fc, bool fold_layernorm, bool ln_stats_epilogue) {
  if (has_conv_transpose(m)) {
    const onnx::Model r = rewrite_conv_transpose(m);
    return Planner(r, max_batch, side_branches, split, bn_on_load, fuse_pairs, fuse_stem_pool, fuse_gap_fc,
                   fold_layernorm, ln_stats_epilogue).run();
  }
  return Planner(m, max_batch, side_branches, split, bn_on_load, fuse_pairs, fuse_stem_pool, fuse_gap_fc,
                 fold_layernorm, ln_stats_epilogue).run();
}

std::string PlanReport::text() const {
  std::ostringstream os;
  for (const Item& it : unsupported) os << "  " << it.op << " '" << it.node << "': " << it.error << "\n";
  if (blocked) os << "  (" << blocked << " further node(s) depend on these)\n";
  return os.str();
}

PlanReport plan_report(const onnx::Model& m, int max_batch, bool split) {
  const bool rw = has_conv_transpose(m);
  const onnx::Model r = rw ? rewrite_conv_transpose(m) : onnx::Model();
  Planner p(rw ? r : m, max_batch, false, split, false);
  try {
    p.run();
  } catch (const std::exception& e) {
    if (p.report_.supported) {  // failed outside the per-node walk (input, output layout)
      p.report_.supported = false;
      p.report_.unsupported.push_back(PlanReport::Item{"(graph)", "", e.what()});
    }
  }
  std::unordered_set<std::string> ct;
  for (const auto& n : m.nodes)
    if (n.op_type == "ConvTranspose") ct.insert(n.name);
  for (auto& it : p.report_.unsupported) {  // report rewritten nodes under the model's own names
    if (ct.count(it.node)) it.op = "ConvTranspose";
    const std::string suf = "/zero_insert";
    if (it.node.size() > suf.size() && it.node.compare(it.node.size() - suf.size(), suf.size(), suf) == 0) {
      it.node.resize(it.node.size() - suf.size());
      it.op = "ConvTranspose";
    }
  }
  return p.report_;
}

}  // namespace die
