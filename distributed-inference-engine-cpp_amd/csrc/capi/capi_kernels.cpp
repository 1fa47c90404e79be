// C ABI for launching individual HIP kernels on caller-provided device pointers (numerics tests
// compare them with torch on the GPU box).  Pointers/streams travel as uint64 (torch data_ptr()
// and torch.cuda.current_stream().cuda_stream).
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../core/json.h"
#include "../engine/engine.h"
#include "../engine/hip_plan.h"
#include "../kernels/kernels.h"
#include "../onnx/onnx_model.h"

using namespace die;

namespace {
template <typename T>
T* P(uint64_t v) {
  return reinterpret_cast<T*>(static_cast<uintptr_t>(v));
}
hipStream_t S(uint64_t v) { return reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(v)); }
int geti(const Json& j, const char* k, int d) {
  auto* v = j.find(k);
  return v ? static_cast<int>(v->as_int()) : d;
}
char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.data(), s.size() + 1);
  return p;
}
}  // namespace

extern "C" {

// geometry JSON: B,H,W,Cin,Ho,Wo,N,KH,KW,stride,pad_h,pad_w,dil,K,Kpad,relu,relu2
int die_kern_conv(const char* geom, uint64_t x, uint64_t w, uint64_t bias, uint64_t res, uint64_t out,
                  uint64_t out_f32, uint64_t scale2, uint64_t shift2, uint64_t out2, int tile, uint64_t stream) {
  try {
    Json j = Json::parse(geom);
    kern::ConvArgs a;
    a.B = geti(j, "B", 1);
    a.H = geti(j, "H", 1);
    a.W = geti(j, "W", 1);
    a.Cin = geti(j, "Cin", 1);
    a.Ho = geti(j, "Ho", 1);
    a.Wo = geti(j, "Wo", 1);
    a.N = geti(j, "N", 1);
    a.KH = geti(j, "KH", 1);
    a.KW = geti(j, "KW", 1);
    a.stride = geti(j, "stride", 1);
    a.pad_h = geti(j, "pad_h", 0);
    a.pad_w = geti(j, "pad_w", 0);
    a.dil = geti(j, "dil", 1);
    a.K = geti(j, "K", a.KH * a.KW * a.Cin);
    a.Kpad = geti(j, "Kpad", (a.K + 63) / 64 * 64);
    a.M = a.B * a.Ho * a.Wo;
    a.relu = geti(j, "relu", 0);
    a.relu2 = geti(j, "relu2", 0);
    a.x = P<const uint16_t>(x);
    a.w = P<const uint16_t>(w);
    a.bias = P<const float>(bias);
    a.res = P<const uint16_t>(res);
    a.out = P<uint16_t>(out);
    a.out_f32 = P<float>(out_f32);
    a.scale2 = P<const float>(scale2);
    a.shift2 = P<const float>(shift2);
    a.out2 = P<uint16_t>(out2);
    a.splits = geti(j, "splits", 1);
    a.order = geti(j, "order", 0);
    a.probe = geti(j, "probe", 0);
    a.tail = geti(j, "tail", 0);
    a.sk = geti(j, "sk", 0);
    if (auto* v = j.find("live")) a.live = P<const long long>(static_cast<uint64_t>(v->as_int()));  // live batch (int64 on the device)
    if (auto* v = j.find("ws")) a.ws = P<float>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("zeros")) a.zeros = P<const uint16_t>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("counters")) a.counters = P<int>(static_cast<uint64_t>(v->as_int()));
    a.counters_n = geti(j, "counters_n", 0);
    a.split = geti(j, "split", 0);
    if (auto* v = j.find("wplane")) a.wplane = v->as_int();
    // LayerNorm folding / statistics (ConvArgs::row_stats, col_sum, row_parts, stats_out, ln_eps)
    if (auto* v = j.find("row_stats")) a.row_stats = P<const float>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("col_sum")) a.col_sum = P<const float>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("row_parts")) a.row_parts = P<const float>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("stats_out")) a.stats_out = P<float>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("ln_eps")) a.ln_eps = static_cast<float>(v->as_double());
    if (tile < 0) tile = kern::choose_tile(a.M, a.N, a.K);
    return static_cast<int>(kern::conv_igemm(a, tile, S(stream)));
  } catch (...) {
    return -1;
  }
}

// geometry JSON: M, K1, N1, N2, relu, relu2, split, wplane1, wplane2, zeros
int die_kern_conv_pair(const char* geom, uint64_t x, uint64_t w1, uint64_t bias1, uint64_t res, uint64_t xout,
                       uint64_t scale2, uint64_t shift2, uint64_t w2, uint64_t bias2, uint64_t out, uint64_t stream) {
  try {
    Json j = Json::parse(geom);
    kern::PairArgs a;
    a.M = geti(j, "M", 0);
    a.K1 = geti(j, "K1", 64);
    a.N1 = geti(j, "N1", 256);
    a.N2 = geti(j, "N2", 64);
    a.relu = geti(j, "relu", 1);
    a.relu2 = geti(j, "relu2", 1);
    a.split = geti(j, "split", 0);
    a.shared_w = geti(j, "shared_w", -1);
    if (auto* v = j.find("wplane1")) a.wplane1 = v->as_int();
    if (auto* v = j.find("wplane2")) a.wplane2 = v->as_int();
    if (auto* v = j.find("zeros")) a.zeros = P<const uint16_t>(static_cast<uint64_t>(v->as_int()));
    if (auto* v = j.find("aout")) a.aout = P<uint16_t>(static_cast<uint64_t>(v->as_int()));
    a.x = P<const uint16_t>(x);
    a.w1 = P<const uint16_t>(w1);
    a.bias1 = P<const float>(bias1);
    a.res = P<const uint16_t>(res);
    a.xout = P<uint16_t>(xout);
    a.scale2 = P<const float>(scale2);
    a.shift2 = P<const float>(shift2);
    a.w2 = P<const uint16_t>(w2);
    a.bias2 = P<const float>(bias2);
    a.out = P<uint16_t>(out);
    return static_cast<int>(kern::conv_pair(a, S(stream)));
  } catch (...) {
    return -1;
  }
}

int die_pair_permute_row(int n) { return kern::pair_permute_row(n); }

int die_kern_input_prep(uint64_t x, uint64_t scale, uint64_t shift, uint64_t out, int B, int C, int H, int W, int Cp,
                        uint64_t stream, int split) {
  return static_cast<int>(kern::input_prep(P<const float>(x), P<const float>(scale), P<const float>(shift),
                                           P<uint16_t>(out), B, C, H, W, Cp, S(stream), split));
}

int die_kern_pool2d(uint64_t x, uint64_t y, int B, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                    int ph, int pw, int is_max, int cip, uint64_t stream, int split) {
  return static_cast<int>(kern::pool2d(P<const uint16_t>(x), P<uint16_t>(y), B, H, W, C, Ho, Wo, kh, kw, sh, sw, ph,
                                       pw, is_max, cip, S(stream), nullptr, nullptr, nullptr, 0, split));
}

int die_kern_gap(uint64_t x, uint64_t out, uint64_t out_f32, uint64_t scale, uint64_t shift, int relu, int B, int HW,
                 int C, uint64_t stream, int split) {
  return static_cast<int>(kern::global_avgpool(P<const uint16_t>(x), P<uint16_t>(out), P<float>(out_f32),
                                               P<const float>(scale), P<const float>(shift), relu, B, HW, C, S(stream),
                                               nullptr, split));
}

int die_kern_affine(uint64_t x, uint64_t z, uint64_t scale, uint64_t shift, int act, uint64_t y, long long M, int C,
                    uint64_t stream, int split) {
  return static_cast<int>(kern::affine_act(P<const uint16_t>(x), P<const uint16_t>(z), P<const float>(scale),
                                           P<const float>(shift), act, P<uint16_t>(y), M, C, S(stream), nullptr, 0,
                                           split));
}

int die_kern_nhwc_to_nchw(uint64_t x, uint64_t y, int B, int H, int W, int C, uint64_t stream, int split) {
  return static_cast<int>(kern::nhwc_to_nchw_f32(P<const uint16_t>(x), P<float>(y), B, H, W, C, S(stream), split));
}

int die_kern_layernorm(uint64_t x, uint64_t y, uint64_t gamma, uint64_t beta, float eps, long long rows, int C,
                       uint64_t stream, int split, int variant) {
  return static_cast<int>(kern::layernorm_rows(P<const uint16_t>(x), P<uint16_t>(y), P<const float>(gamma),
                                               P<const float>(beta), eps, rows, C, S(stream), split, 0, variant));
}

int die_kern_tokens(uint64_t patches, uint64_t cls, uint64_t pos, uint64_t out, int B, int S0, int C, uint64_t stream,
                    int split) {
  return static_cast<int>(kern::tokens_assemble(P<const uint16_t>(patches), P<const float>(cls), P<const float>(pos),
                                                P<uint16_t>(out), B, S0, C, S(stream), split));
}

int die_kern_gather_rows(uint64_t x, uint64_t y, int B, int Sq, int idx, int C, uint64_t stream, int split) {
  return static_cast<int>(kern::gather_rows(P<const uint16_t>(x), P<uint16_t>(y), B, Sq, idx, C, S(stream), split));
}

void die_kern_set_gap_fc_stop(int v) { kern::set_gap_fc_stop(v); }

int die_kern_gap_fc(uint64_t x, int B, int HW, int C, int mode, uint64_t w, long long wplane, int Kpad, uint64_t bias,
                    int N, int act, uint64_t out, uint64_t ws, long long ws_bytes, uint64_t counters, int counters_n,
                    uint64_t stream, int split) {
  return static_cast<int>(kern::gap_fc(P<const uint16_t>(x), B, HW, C, mode, P<const uint16_t>(w), wplane, Kpad,
                                       P<const float>(bias), N, act, P<float>(out), P<float>(ws),
                                       static_cast<size_t>(ws_bytes), P<int>(counters), counters_n, S(stream), nullptr,
                                       split));
}

void die_kern_set_attention_variant(int v) { kern::set_attention_variant(v); }
void die_kern_set_decode_variant(int v) { kern::set_decode_variant(v); }
void die_kern_set_layernorm_xcd(int v) { kern::set_layernorm_xcd(v); }
void die_kern_set_pair_shared_w(int v) { kern::set_pair_shared_w(v); }

int die_kern_attention(uint64_t q, uint64_t k, uint64_t v, uint64_t out, int B, int Sq, int H, int D, int ldq, int ldk,
                       int ldv, int ldo, float scale, uint64_t stream, int split) {
  return static_cast<int>(kern::attention(P<const uint16_t>(q), P<const uint16_t>(k), P<const uint16_t>(v),
                                          P<uint16_t>(out), B, Sq, H, D, ldq, ldk, ldv, ldo, scale, S(stream), split));
}

// geometry JSON: B,H,W,Cin,Ho,Wo,Cout,groups,KH,KW,stride,pad_h,pad_w,dil,act,clip_lo,clip_hi,split
int die_kern_gconv(const char* geom, uint64_t x, uint64_t w, uint64_t bias, uint64_t out, uint64_t stream) {
  try {
    Json j = Json::parse(geom);
    kern::GConvArgs a;
    a.B = geti(j, "B", 1);
    a.H = geti(j, "H", 1);
    a.W = geti(j, "W", 1);
    a.Cin = geti(j, "Cin", 8);
    a.Ho = geti(j, "Ho", 1);
    a.Wo = geti(j, "Wo", 1);
    a.Cout = geti(j, "Cout", 8);
    a.groups = geti(j, "groups", 1);
    a.KH = geti(j, "KH", 1);
    a.KW = geti(j, "KW", 1);
    a.stride = geti(j, "stride", 1);
    a.pad_h = geti(j, "pad_h", 0);
    a.pad_w = geti(j, "pad_w", 0);
    a.dil = geti(j, "dil", 1);
    a.act = geti(j, "act", 0);
    if (auto* v = j.find("clip_lo")) a.clip_lo = static_cast<float>(v->as_double());
    if (auto* v = j.find("clip_hi")) a.clip_hi = static_cast<float>(v->as_double());
    a.split = geti(j, "split", 0);
    a.x = P<const uint16_t>(x);
    a.w = P<const float>(w);
    a.bias = P<const float>(bias);
    a.out = P<uint16_t>(out);
    return static_cast<int>(kern::grouped_conv(a, S(stream)));
  } catch (...) {
    return -1;
  }
}

int die_kern_softmax(uint64_t x, uint64_t y, uint64_t yf, long long rows, int C, uint64_t stream, int split) {
  return static_cast<int>(kern::softmax_rows(P<const uint16_t>(x), P<uint16_t>(y), P<float>(yf), rows, C, S(stream), split));
}

long long die_decode_scratch_bytes(int max_batch, long long text_cap) {
  return static_cast<long long>(kern::decode_scratch_bytes(max_batch, static_cast<size_t>(text_cap)));
}

int die_kern_decode(uint64_t text, uint64_t offs, long long text_cap, uint64_t lens, int B, uint64_t out,
                    long long numel, uint64_t status, uint64_t ntok, uint64_t scratch, uint64_t stream) {
  return static_cast<int>(kern::decode_json_numbers(P<const unsigned char>(text), P<const long long>(offs),
                                                    static_cast<size_t>(text_cap), P<const long long>(lens), B,
                                                    P<float>(out), numel, P<int>(status), P<int>(ntok), P<void>(scratch),
                                                    S(stream)));
}

// packed: 4-bit packed samples at packed + poffs[b] (poffs[b] < 0: raw text at text + offs[b])
int die_kern_decode_packed(uint64_t text, uint64_t offs, uint64_t packed, uint64_t poffs, long long text_cap,
                           uint64_t lens, int B, uint64_t out, long long numel, uint64_t status, uint64_t ntok,
                           uint64_t scratch, uint64_t stream) {
  return static_cast<int>(kern::decode_json_numbers(P<const unsigned char>(text), P<const long long>(offs),
                                                    static_cast<size_t>(text_cap), P<const long long>(lens), B,
                                                    P<float>(out), numel, P<int>(status), P<int>(ntok), P<void>(scratch),
                                                    S(stream), P<const unsigned char>(packed), P<const long long>(poffs)));
}

int die_kern_stem(uint64_t x, uint64_t w, uint64_t bias, uint64_t out, int B, int H, int W, int Ho, int Wo, int relu,
                  uint64_t stream, int split) {
  return static_cast<int>(kern::conv_stem7x7(P<const uint16_t>(x), P<const uint16_t>(w), P<const float>(bias),
                                             P<uint16_t>(out), B, H, W, Ho, Wo, relu, S(stream), nullptr, split));
}

int die_kern_stem_nchw(uint64_t x, int C, uint64_t scale, uint64_t shift, uint64_t w, uint64_t bias, uint64_t out, int B,
                       int H, int W, int Ho, int Wo, int relu, uint64_t stream, int split, int max_blocks) {
  return static_cast<int>(kern::conv_stem7x7_nchw(P<const float>(x), C, P<const float>(scale), P<const float>(shift),
                                                  P<const uint16_t>(w), P<const float>(bias), P<uint16_t>(out), B, H, W,
                                                  Ho, Wo, relu, S(stream), nullptr, split, max_blocks));
}

// Load-time support report: every node the HIP planner cannot lower, with the reason.
char* die_plan_report(const char* model_path, int split, char** err) {
  try {
    const PlanReport r = plan_report(onnx::load_onnx(model_path), 8, split != 0);
    Json j = Json::object();
    j["supported"] = r.supported;
    Json items = Json::array();
    for (const auto& it : r.unsupported) {
      Json e = Json::object();
      e["node"] = it.node;
      e["op"] = it.op;
      e["error"] = it.error;
      items.push_back(e);
    }
    j["unsupported"] = items;
    j["blocked"] = r.blocked;
    j["text"] = r.text();
    return dup(j.dump());
  } catch (const std::exception& e) {
    if (err) *err = dup(e.what());
    return nullptr;
  }
}

// Plan summary of a model (op list with fused epilogues), for tests and docs.
// Hybrid HIP + CPU partition of a model (engine/hybrid_engine.cpp), computed on the host.
char* die_hybrid_partition(const char* model_path, int max_batch, int split, char** err) {
  try {
    const onnx::Model m = onnx::load_onnx(model_path);
    Json out = Json::array();
    for (const HybridSegment& s : hybrid_partition(m, max_batch, split != 0)) {
      Json e = Json::object();
      e["device"] = s.hip ? "hip" : "cpu";
      e["first"] = s.first;
      e["last"] = s.last;
      e["input"] = s.input;
      e["output"] = s.output;
      e["gemm_nodes"] = s.convs;
      Json ops = Json::array();
      for (int k = s.first; k <= s.last; ++k) ops.push_back(m.nodes[static_cast<size_t>(k)].op_type);
      e["ops"] = ops;
      out.push_back(e);
    }
    return dup(out.dump());
  } catch (const std::exception& ex) {
    if (err) *err = dup(ex.what());
    return nullptr;
  }
}

// fuse: bit 0 conv pairs, bit 1 stem + pool, bit 2 global pool + FC head, bit 3 LayerNorm folding,
// bit 4 LayerNorm statistics from the producing GEMM's epilogue
char* die_plan_summary(const char* model_path, int max_batch, int side_branches, int split, int fuse, char** err) {
  try {
    Plan p = build_plan(onnx::load_onnx(model_path), max_batch, side_branches != 0, split != 0, false, (fuse & 1) != 0,
                        (fuse & 2) != 0, (fuse & 4) != 0, (fuse & 8) != 0, (fuse & 16) != 0);
    Json j = Json::object();
    j["summary"] = p.summary();
    j["arena_bytes"] = static_cast<long long>(p.arena_bytes);
    j["param_bytes"] = static_cast<long long>(p.params.size());
    j["gflop_per_sample"] = p.flops_per_sample / 1e9;
    j["precision"] = p.split ? "fp32" : "bf16";
    Json ops = Json::array();
    for (auto& o : p.ops) {
      Json e = Json::object();
      static const char* kinds[] = {"input_prep", "conv", "pool", "gap", "affine", "to_nchw_f32", "bf16_to_f32",
                                    "layernorm", "tokens", "gather_rows", "attention", "stem", "gconv", "softmax",
                                    "rows_prep", "copy_cols", "binary", "unary", "conv_pair", "pad", "where", "resize", "bmm", "gap_fc"};
      static_assert(sizeof(kinds) / sizeof(kinds[0]) == PlanOp::GAP_FC + 1, "one name per PlanOp kind");
      e["kind"] = kinds[o.kind];
      e["name"] = o.name;
      e["gflop"] = o.flops_per_sample / 1e9;
      e["join"] = o.join;
      // arena ranges [offset, offset + bytes) at max_batch of the op's buffers, by role
      Json bufs = Json::object();
      const char* roles[] = {"in", "in2", "in3", "out", "out2", "out3", "out_stats"};
      const int ids[] = {o.in, o.in2, o.in3, o.out, o.out2, o.out3, o.out_stats};
      for (int r = 0; r < 7; ++r)
        if (ids[r] >= 0) {
          Json range = Json::array();
          range.push_back(static_cast<long long>(p.bufs[ids[r]].offset));
          range.push_back(static_cast<long long>(p.bufs[ids[r]].offset + p.bufs[ids[r]].bytes_per_sample * max_batch));
          bufs[roles[r]] = range;
        }
      e["bufs"] = bufs;
      if (o.kind == PlanOp::CONV) {
        e["N"] = o.conv.N;
        e["K"] = o.conv.K;
        e["KH"] = o.conv.KH;
        e["stride"] = o.conv.stride;
        e["relu"] = o.conv.relu;
        e["residual"] = o.in2 >= 0;
        e["dual_store"] = o.out2 >= 0;
        e["preact_on_load"] = o.in_scale_off != SIZE_MAX;
        e["store_main"] = o.out >= 0 || o.out_f32 != -1;
        e["relu2"] = o.conv.relu2;
        e["act"] = o.conv.relu;
        e["rows"] = o.conv.Ho * o.conv.Wo;
        e["layernorm_folded"] = o.colsum_off != SIZE_MAX;
        e["stats_from_producer"] = o.in3_parts != 0;  // reads (merges) LayerNorm statistics partials
      }
      if (o.kind == PlanOp::LAYERNORM) e["stats_only"] = o.stats_only != 0;
      if (o.kind == PlanOp::CONV || o.kind == PlanOp::TOKENS) e["stats_out"] = o.out_stats >= 0;  // writes the partials
      if (o.kind == PlanOp::STEM) {
        e["pool_fused"] = o.is_max != 0;
        e["rows"] = o.is_max ? o.Ho * o.Wo : o.conv.Ho * o.conv.Wo;
      }
      if (o.kind == PlanOp::CONV_PAIR) {
        e["K1"] = o.conv.K;
        e["N1"] = o.conv.N;
        e["N2"] = o.n2;
        e["residual"] = o.in2 >= 0;
        e["store_main"] = o.out >= 0;
        e["store_preact"] = o.out3 >= 0;
        e["relu"] = o.pair_relu;
        e["rows"] = o.conv.Ho * o.conv.Wo;
      }
      ops.push_back(e);
    }
    j["ops"] = ops;
    Json in = Json::array(), out = Json::array();
    for (auto d : p.input_shape) in.push_back(static_cast<long long>(d));
    for (auto d : p.output_shape) out.push_back(static_cast<long long>(d));
    j["input_shape"] = in;
    j["output_shape"] = out;
    return dup(j.dump());
  } catch (const std::exception& e) {
    if (err) *err = dup(e.what());
    return nullptr;
  }
}

}  // extern "C"
