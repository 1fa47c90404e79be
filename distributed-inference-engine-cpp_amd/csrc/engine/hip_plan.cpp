#include "hip_plan.h"

#include <algorithm>
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

struct Val {
  enum Kind { GRAPH_IN, NHWC, ROWS_BF16, ROWS_F32 } kind = NHWC;
  int C = 0, H = 1, W = 1;
  int buf = -1;
  bool has_affine = false;
  std::vector<float> asc, ash;
};

class Planner {
 public:
  Planner(const onnx::Model& m, int max_batch) : m_(m), max_batch_(max_batch) {}

  Plan run() {
    if (m_.inputs.empty() || m_.outputs.empty()) throw std::runtime_error("model needs an input and an output");
    for (size_t i = 0; i < m_.nodes.size(); ++i)
      for (auto& in : m_.nodes[i].inputs) consumers_[in].push_back(static_cast<int>(i));
    for (auto& o : m_.outputs) graph_outputs_.insert(o.name);
    // graph input
    const auto& vi = m_.inputs[0];
    if (vi.dims.size() != 4) throw std::runtime_error("HIP engine expects a 4-D NCHW image input, got rank " + std::to_string(vi.dims.size()));
    Val in;
    in.kind = Val::GRAPH_IN;
    in.C = static_cast<int>(vi.dims[1]);
    in.H = static_cast<int>(vi.dims[2]);
    in.W = static_cast<int>(vi.dims[3]);
    in.buf = kBufGraphIn;
    if (in.C <= 0 || in.H <= 0 || in.W <= 0) throw std::runtime_error("input dims must be static except the batch");
    define(vi.name, in);
    plan_.input_shape = {1, in.C, in.H, in.W};
    plan_.input_numel = static_cast<size_t>(in.C) * in.H * in.W;

    done_.assign(m_.nodes.size(), false);
    for (size_t i = 0; i < m_.nodes.size(); ++i) {
      if (done_[i]) continue;
      done_[i] = true;
      lower(static_cast<int>(i));
    }
    finalize_output();
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
  int new_buf(size_t bytes_per_sample) {
    PlanBuf b;
    b.bytes_per_sample = bytes_per_sample;
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
  void add_op(PlanOp op) { plan_.ops.push_back(std::move(op)); }

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
    if (op == "Conv") return lower_conv(idx);
    if (op == "Gemm" || (op == "MatMul" && is_init(n.in(1)))) return lower_gemm(idx);
    if (op == "BatchNormalization") return lower_bn(idx);
    if (op == "Relu") return lower_relu(idx);
    if (op == "Add") return lower_add(idx);
    if (op == "MaxPool" || op == "AveragePool") return lower_pool(idx);
    if (op == "GlobalAveragePool") return lower_gap(idx);
    if (op == "Flatten" || op == "Reshape" || op == "Squeeze") return lower_flatten(idx);
    if (op == "Identity" || op == "Dropout") {
      define(n.outputs[0], val(n.in(0), n));
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
    if (x.C > 8) throw std::runtime_error("HIP engine: input with more than 8 channels is not supported");
    p.Cp = x.C <= 4 ? 4 : 8;
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
    auto pads = n.get_ints("pads", {0, 0, 0, 0});
    if (st[0] != st[1] || dl[0] != dl[1]) throw std::runtime_error("Conv " + n.name + ": anisotropic stride/dilation");
    const std::string ap = n.get_string("auto_pad", "NOTSET");
    int in_buf;
    int Cstore;
    if (x.kind == Val::GRAPH_IN) {
      in_buf = ensure_nhwc_input(x, n.in(0));
      Cstore = x.C <= 4 ? 4 : 8;
    } else if (x.kind == Val::NHWC) {
      in_buf = x.buf;
      Cstore = x.C;
    } else {
      throw std::runtime_error("Conv " + n.name + ": input must be an image tensor");
    }
    if (Cin != x.C) throw std::runtime_error("Conv " + n.name + ": channel mismatch");
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
    if (pads[0] != pads[2] || pads[1] != pads[3])
      throw std::runtime_error("Conv " + n.name + ": asymmetric padding is not supported");
    const int s = static_cast<int>(st[0]), d = static_cast<int>(dl[0]);
    const int Ho = (x.H + 2 * static_cast<int>(pads[0]) - d * (KH - 1) - 1) / s + 1;
    const int Wo = (x.W + 2 * static_cast<int>(pads[1]) - d * (KW - 1) - 1) / s + 1;
    if (Cout % 8) throw std::runtime_error("Conv " + n.name + ": output channels must be a multiple of 8");

    // --- fusion lookahead ---
    std::vector<float> scale(Cout, 1.f), shift(Cout, 0.f);
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
    std::string res_name;
    c1 = sole_consumer(cur);
    if (c1 >= 0 && m_.nodes[c1].op_type == "Relu") {
      relu = 1;
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    } else if (c1 >= 0 && m_.nodes[c1].op_type == "Add") {
      const Node& add = m_.nodes[c1];
      const std::string other = add.in(0) == cur ? add.in(1) : add.in(0);
      auto it = vid_.find(other);
      if (it != vid_.end() && vals_[it->second].kind == Val::NHWC && vals_[it->second].C == Cout &&
          vals_[it->second].H == Ho && vals_[it->second].W == Wo && add.in(0) != add.in(1)) {
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
    const int Npad = static_cast<int>(round_up(Cout, 128));
    std::vector<uint16_t> wp(static_cast<size_t>(Npad) * Kpad, 0);
    for (int co = 0; co < Cout; ++co)
      for (int ci = 0; ci < Cin; ++ci)
        for (int ky = 0; ky < KH; ++ky)
          for (int kx = 0; kx < KW; ++kx) {
            const float w = wt.f[((static_cast<size_t>(co) * Cin + ci) * KH + ky) * KW + kx] * scale[co];
            wp[static_cast<size_t>(co) * Kpad + (ky * KW + kx) * Cstore + ci] = to_bf16(w);
          }

    PlanOp p;
    p.kind = PlanOp::CONV;
    p.name = n.name;
    p.in = in_buf;
    p.in2 = res_buf;
    p.w_off = push_bf16(wp);
    p.bias_off = push_f32(shift);
    auto& a = p.conv;
    a.H = x.H;
    a.W = x.W;
    a.Cin = Cstore;
    a.Ho = Ho;
    a.Wo = Wo;
    a.N = Cout;
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
    p.flops_per_sample = 2.0 * Ho * Wo * Cout * (KH * KW * Cin);
    p.tile_bmax = kern::choose_tile(max_batch_ * Ho * Wo, Cout, K);
    const size_t out_bytes = static_cast<size_t>(Ho) * Wo * Cout * 2;
    Val o;
    o.kind = Val::NHWC;
    o.C = Cout;
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

  void lower_gemm(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = val(n.in(0), n);
    if (!(x.kind == Val::ROWS_BF16 || (x.kind == Val::NHWC && x.H == 1 && x.W == 1)))
      throw std::runtime_error(n.op_type + " " + n.name + ": input must be a [batch, features] matrix");
    const auto& wt = init(n.in(1), n);
    if (wt.dims.size() != 2) throw std::runtime_error(n.op_type + " " + n.name + ": weight must be 2-D");
    const bool gemm = n.op_type == "Gemm";
    if (gemm && n.get_int("transA", 0)) throw std::runtime_error("Gemm " + n.name + ": transA is not supported");
    const bool tb = gemm && n.get_int("transB", 0);
    const float alpha = gemm ? n.get_float("alpha", 1.f) : 1.f;
    const float beta = gemm ? n.get_float("beta", 1.f) : 1.f;
    const int K = static_cast<int>(tb ? wt.dims[1] : wt.dims[0]);
    const int N = static_cast<int>(tb ? wt.dims[0] : wt.dims[1]);
    if (K != x.C) throw std::runtime_error(n.op_type + " " + n.name + ": inner dimension mismatch");
    if (K % 8) throw std::runtime_error(n.op_type + " " + n.name + ": K % 8 must be 0");
    std::vector<float> bias(N, 0.f);
    if (gemm && !n.in(2).empty()) {
      const auto& c = init(n.in(2), n).f;
      for (int j = 0; j < N; ++j) bias[j] = beta * c[c.size() == 1 ? 0 : j % c.size()];
    }
    std::string cur = n.outputs[0];
    int relu = 0;
    int c1 = sole_consumer(cur);
    if (!gemm && c1 >= 0 && m_.nodes[c1].op_type == "Add" && is_init(m_.nodes[c1].in(0) == cur ? m_.nodes[c1].in(1) : m_.nodes[c1].in(0))) {
      const Node& add = m_.nodes[c1];
      const auto& c = init(add.in(0) == cur ? add.in(1) : add.in(0), add).f;
      if (c.size() == static_cast<size_t>(N) || c.size() == 1) {
        for (int j = 0; j < N; ++j) bias[j] += c[c.size() == 1 ? 0 : j];
        done_[c1] = true;
        cur = add.outputs[0];
        c1 = sole_consumer(cur);
      }
    }
    if (c1 >= 0 && m_.nodes[c1].op_type == "Relu") {
      relu = 1;
      done_[c1] = true;
      cur = m_.nodes[c1].outputs[0];
    }
    const int Kpad = static_cast<int>(round_up(K, 64));
    const int Npad = static_cast<int>(round_up(N, 128));
    std::vector<uint16_t> wp(static_cast<size_t>(Npad) * Kpad, 0);
    for (int j = 0; j < N; ++j)
      for (int k = 0; k < K; ++k) {
        const float w = tb ? wt.f[static_cast<size_t>(j) * K + k] : wt.f[static_cast<size_t>(k) * N + j];
        wp[static_cast<size_t>(j) * Kpad + k] = to_bf16(alpha * w);
      }
    PlanOp p;
    p.kind = PlanOp::CONV;
    p.name = n.name;
    p.in = x.buf;
    p.w_off = push_bf16(wp);
    p.bias_off = push_f32(bias);
    auto& a = p.conv;
    a.Cin = K;
    a.N = N;
    a.K = K;
    a.Kpad = Kpad;
    a.relu = relu;
    p.flops_per_sample = 2.0 * N * K;
    p.tile_bmax = kern::choose_tile(max_batch_, N, K);
    Val o;
    o.C = N;
    if (graph_outputs_.count(cur) && consumers(cur).empty()) {
      p.out_f32 = kBufGraphOut;
      o.kind = Val::ROWS_F32;
      o.buf = kBufGraphOut;
    } else {
      p.out = new_buf(static_cast<size_t>(N) * 2);
      o.kind = Val::ROWS_BF16;
      o.buf = p.out;
    }
    define(cur, o);
    add_op(std::move(p));
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
    standalone_affine(n, x, &sc, &sh, nullptr);
  }

  void lower_relu(int idx) {
    const Node& n = m_.nodes[idx];
    Val& x = val(n.in(0), n);
    standalone_affine(n, x, nullptr, nullptr, nullptr);
  }

  void lower_add(int idx) {
    const Node& n = m_.nodes[idx];
    Val& a = val(n.in(0), n);
    Val& b = val(n.in(1), n);
    if (a.kind != b.kind || a.C != b.C || a.H != b.H || a.W != b.W)
      throw std::runtime_error("Add " + n.name + ": broadcasting adds are not supported by the HIP engine");
    standalone_affine(n, a, nullptr, nullptr, &b);
  }

  void standalone_affine(const Node& n, const Val& x, const std::vector<float>* sc, const std::vector<float>* sh,
                         const Val* z) {
    if (x.kind != Val::NHWC && x.kind != Val::ROWS_BF16)
      throw std::runtime_error(n.op_type + " " + n.name + ": unsupported input layout");
    if (x.C % 8) throw std::runtime_error(n.op_type + " " + n.name + ": channels must be a multiple of 8");
    std::string cur = n.outputs[0];
    int act = n.op_type == "Relu" ? 1 : 0;
    if (!act) {
      const int c1 = sole_consumer(cur);
      if (c1 >= 0 && m_.nodes[c1].op_type == "Relu") {
        act = 1;
        done_[c1] = true;
        cur = m_.nodes[c1].outputs[0];
      }
    }
    PlanOp p;
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
    Val x = val(n.in(0), n);
    if (x.kind != Val::NHWC) throw std::runtime_error(n.op_type + " " + n.name + ": input must be an image tensor");
    auto k = n.get_ints("kernel_shape");
    auto st = n.get_ints("strides", {1, 1});
    auto pads = n.get_ints("pads", {0, 0, 0, 0});
    if (pads[0] != pads[2] || pads[1] != pads[3]) throw std::runtime_error(n.op_type + ": asymmetric pads");
    const bool ceil_mode = n.get_int("ceil_mode", 0) != 0;
    auto od = [&](int in, int d) {
      double v = static_cast<double>(in + 2 * pads[d] - k[d]) / st[d];
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

  void lower_gap(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = val(n.in(0), n);
    if (x.kind != Val::NHWC) throw std::runtime_error("GlobalAveragePool: input must be an image tensor");
    PlanOp p;
    p.kind = PlanOp::GAP;
    p.name = n.name;
    p.in = x.buf;
    p.C = x.C;
    p.H = x.H;
    p.W = x.W;
    p.out = new_buf(static_cast<size_t>(x.C) * 2);
    Val o;
    o.kind = Val::NHWC;  // [C,1,1]
    o.C = x.C;
    o.buf = p.out;
    define(n.outputs[0], o);
    add_op(std::move(p));
  }

  void lower_flatten(int idx) {
    const Node& n = m_.nodes[idx];
    Val x = val(n.in(0), n);
    if (n.op_type == "Flatten" && n.get_int("axis", 1) != 1) throw std::runtime_error("Flatten: axis must be 1");
    if (!(x.kind == Val::ROWS_BF16 || (x.kind == Val::NHWC && x.H == 1 && x.W == 1)))
      throw std::runtime_error(n.op_type + " " + n.name + ": only flattening of 1x1 feature maps is supported");
    Val o = x;
    o.kind = Val::ROWS_BF16;
    o.H = o.W = 1;
    define(n.outputs[0], o);
  }

  void finalize_output() {
    const std::string& name = m_.outputs[0].name;
    auto it = vid_.find(name);
    if (it == vid_.end()) throw std::runtime_error("graph output " + name + " is not produced");
    Val v = vals_[it->second];
    if (v.kind == Val::ROWS_F32 && v.buf == kBufGraphOut) {
      plan_.output_shape = {1, v.C};
    } else if (v.kind == Val::ROWS_BF16 || (v.kind == Val::NHWC && v.H == 1 && v.W == 1 &&
                                           m_.outputs[0].dims.size() == 2)) {
      PlanOp p;
      p.kind = PlanOp::BF16_TO_F32;
      p.name = "output_cast";
      p.in = v.buf;
      p.C = v.C;
      p.out_f32 = kBufGraphOut;
      add_op(std::move(p));
      plan_.output_shape = {1, v.C};
    } else if (v.kind == Val::NHWC) {
      PlanOp p;
      p.kind = PlanOp::TO_NCHW_F32;
      p.name = "output_nchw";
      p.in = v.buf;
      p.C = v.C;
      p.H = v.H;
      p.W = v.W;
      p.out_f32 = kBufGraphOut;
      add_op(std::move(p));
      plan_.output_shape = {1, v.C, v.H, v.W};
    } else {
      throw std::runtime_error("unsupported graph output layout");
    }
    plan_.output_numel = 1;
    for (auto dim : plan_.output_shape) plan_.output_numel *= static_cast<size_t>(dim);
  }

  void assign_arena() {
    const int nops = static_cast<int>(plan_.ops.size());
    for (int i = 0; i < nops; ++i) {
      const PlanOp& p = plan_.ops[i];
      for (int b : {p.out, p.out2})
        if (b >= 0 && plan_.bufs[b].first_use < 0) plan_.bufs[b].first_use = i;
      for (int b : {p.in, p.in2, p.out, p.out2})
        if (b >= 0) plan_.bufs[b].last_use = std::max(plan_.bufs[b].last_use, i);
    }
    struct Block {
      size_t off, size;
      int last;
    };
    std::vector<Block> live;
    size_t top = 0;
    std::vector<int> order(plan_.bufs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<int>(i);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return plan_.bufs[a].first_use < plan_.bufs[b].first_use; });
    for (int bi : order) {
      PlanBuf& b = plan_.bufs[bi];
      const size_t size = round_up(b.bytes_per_sample * max_batch_, 256);
      live.erase(std::remove_if(live.begin(), live.end(), [&](const Block& k) { return k.last < b.first_use; }),
                 live.end());
      std::sort(live.begin(), live.end(), [](const Block& a, const Block& c) { return a.off < c.off; });
      size_t cand = 0;
      bool placed = false;
      for (const Block& k : live) {
        if (k.off >= cand + size) {
          placed = true;
          break;
        }
        cand = std::max(cand, k.off + k.size);
      }
      (void)placed;
      b.offset = cand;
      live.push_back(Block{cand, size, b.last_use});
      top = std::max(top, cand + size);
    }
    plan_.arena_bytes = top;
    double fl = 0;
    for (auto& p : plan_.ops) fl += p.flops_per_sample;
    plan_.flops_per_sample = fl;
  }

  const onnx::Model& m_;
  int max_batch_;
  Plan plan_;
  std::vector<Val> vals_;
  std::unordered_map<std::string, int> vid_;
  std::unordered_map<std::string, std::vector<int>> consumers_;
  std::unordered_set<std::string> graph_outputs_;
  std::unordered_map<std::string, int> prepped_;
  std::vector<bool> done_;
};

}  // namespace

std::string Plan::summary() const {
  std::ostringstream os;
  size_t convs = 0;
  for (auto& o : ops) convs += o.kind == PlanOp::CONV;
  os << ops.size() << " device ops (" << convs << " MFMA conv/gemm), arena " << arena_bytes / (1 << 20) << " MiB, params "
     << params.size() / (1 << 20) << " MiB, " << flops_per_sample / 1e9 << " GFLOP/sample";
  return os.str();
}

Plan build_plan(const onnx::Model& m, int max_batch) { return Planner(m, max_batch).run(); }

}  // namespace die
