#include "cpu_exec.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <stdexcept>

namespace die {

using onnx::Node;

namespace {

[[noreturn]] void fail(const Node& n, const std::string& msg) {
  throw std::runtime_error("cpu executor: " + n.op_type + " (" + n.name + "): " + msg);
}

CpuValuePtr make_f(std::vector<int64_t> shape) {
  auto v = std::make_shared<CpuValue>();
  v->shape = std::move(shape);
  v->f.assign(static_cast<size_t>(v->numel()), 0.f);
  return v;
}
CpuValuePtr make_i(std::vector<int64_t> shape) {
  auto v = std::make_shared<CpuValue>();
  v->shape = std::move(shape);
  v->is_int = true;
  v->i.assign(static_cast<size_t>(v->numel()), 0);
  return v;
}

std::vector<int64_t> as_ints(const CpuValue& v) {
  if (v.is_int) return v.i;
  std::vector<int64_t> r(v.f.size());
  for (size_t k = 0; k < r.size(); ++k) r[k] = static_cast<int64_t>(v.f[k]);
  return r;
}

std::vector<int64_t> strides_of(const std::vector<int64_t>& s) {
  std::vector<int64_t> st(s.size(), 1);
  for (int k = static_cast<int>(s.size()) - 2; k >= 0; --k) st[k] = st[k + 1] * s[k + 1];
  return st;
}

int64_t norm_axis(int64_t a, size_t rank) { return a < 0 ? a + static_cast<int64_t>(rank) : a; }

}  // namespace

// ------------------------------------------------------------------------------------------------
// GEMM: C[M,N] (+)= A[M,K] * B[K,N], row-major.  Parallel over row blocks, K/N blocked so the B
// panel stays in L2 and the inner axpy vectorises.
// ------------------------------------------------------------------------------------------------
void cpu_gemm(int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
              bool accumulate) {
  constexpr int KB = 256, NB = 512;
#pragma omp parallel for schedule(dynamic, 1) if (static_cast<long>(M) * N * K > 1 << 16)
  for (int i0 = 0; i0 < M; i0 += 4) {
    const int i1 = std::min(M, i0 + 4);
    if (!accumulate)
      for (int i = i0; i < i1; ++i) std::memset(C + static_cast<size_t>(i) * ldc, 0, sizeof(float) * N);
    for (int n0 = 0; n0 < N; n0 += NB) {
      const int nn = std::min(NB, N - n0);
      for (int k0 = 0; k0 < K; k0 += KB) {
        const int k1 = std::min(K, k0 + KB);
        for (int i = i0; i < i1; ++i) {
          float* __restrict c = C + static_cast<size_t>(i) * ldc + n0;
          const float* a = A + static_cast<size_t>(i) * lda;
          int k = k0;
          for (; k + 4 <= k1; k += 4) {
            const float a0 = a[k], a1 = a[k + 1], a2 = a[k + 2], a3 = a[k + 3];
            const float* b0 = B + static_cast<size_t>(k) * ldb + n0;
            const float* b1 = b0 + ldb;
            const float* b2 = b1 + ldb;
            const float* b3 = b2 + ldb;
#pragma omp simd
            for (int j = 0; j < nn; ++j) c[j] += a0 * b0[j] + a1 * b1[j] + a2 * b2[j] + a3 * b3[j];
          }
          for (; k < k1; ++k) {
            const float av = a[k];
            const float* b = B + static_cast<size_t>(k) * ldb + n0;
#pragma omp simd
            for (int j = 0; j < nn; ++j) c[j] += av * b[j];
          }
        }
      }
    }
  }
}

namespace {

// ---- Conv -----------------------------------------------------------------------------------------
CpuValuePtr op_conv(const Node& n, const CpuValue& x, const CpuValue& w, const CpuValue* b) {
  if (x.shape.size() != 4 || w.shape.size() != 4) fail(n, "only 2-D convolution is supported");
  const int64_t N = x.shape[0], C = x.shape[1], H = x.shape[2], W = x.shape[3];
  const int64_t M = w.shape[0], kh = w.shape[2], kw = w.shape[3];
  const int64_t G = n.get_int("group", 1);
  if (w.shape[1] * G != C) fail(n, "channel mismatch");
  auto st = n.get_ints("strides", {1, 1});
  auto dl = n.get_ints("dilations", {1, 1});
  auto pads = n.get_ints("pads", {0, 0, 0, 0});
  std::string ap = n.get_string("auto_pad", "NOTSET");
  if (ap == "SAME_UPPER" || ap == "SAME_LOWER") {
    for (int d = 0; d < 2; ++d) {
      int64_t in = d ? W : H, k = (d ? kw : kh), s = st[d], dil = dl[d];
      int64_t out = (in + s - 1) / s;
      int64_t total = std::max<int64_t>(0, (out - 1) * s + (k - 1) * dil + 1 - in);
      int64_t lo = ap == "SAME_UPPER" ? total / 2 : total - total / 2;
      pads[d] = lo;
      pads[d + 2] = total - lo;
    }
  } else if (ap == "VALID") {
    pads = {0, 0, 0, 0};
  }
  const int64_t Ho = (H + pads[0] + pads[2] - (dl[0] * (kh - 1) + 1)) / st[0] + 1;
  const int64_t Wo = (W + pads[1] + pads[3] - (dl[1] * (kw - 1) + 1)) / st[1] + 1;
  auto y = make_f({N, M, Ho, Wo});
  const int64_t Cg = C / G, Mg = M / G, Kdim = Cg * kh * kw, P = Ho * Wo;
  const bool direct = kh == 1 && kw == 1 && st[0] == 1 && st[1] == 1 && pads[0] == 0 && pads[1] == 0 &&
                      pads[2] == 0 && pads[3] == 0;
  std::vector<float> col;
  if (!direct) col.resize(static_cast<size_t>(Kdim * P));
  for (int64_t b0 = 0; b0 < N; ++b0) {
    for (int64_t g = 0; g < G; ++g) {
      const float* xin = x.f.data() + (b0 * C + g * Cg) * H * W;
      const float* B;
      if (direct) {
        B = xin;
      } else {
#pragma omp parallel for collapse(2) if (Kdim * P > 1 << 14)
        for (int64_t c = 0; c < Cg; ++c)
          for (int64_t ky = 0; ky < kh; ++ky)
            for (int64_t kx = 0; kx < kw; ++kx) {
              float* dst = col.data() + ((c * kh + ky) * kw + kx) * P;
              for (int64_t oy = 0; oy < Ho; ++oy) {
                const int64_t iy = oy * st[0] - pads[0] + ky * dl[0];
                for (int64_t ox = 0; ox < Wo; ++ox) {
                  const int64_t ix = ox * st[1] - pads[1] + kx * dl[1];
                  dst[oy * Wo + ox] =
                      (iy >= 0 && iy < H && ix >= 0 && ix < W) ? xin[(c * H + iy) * W + ix] : 0.f;
                }
              }
            }
        B = col.data();
      }
      float* out = y->f.data() + (b0 * M + g * Mg) * P;
      cpu_gemm(static_cast<int>(Mg), static_cast<int>(P), static_cast<int>(Kdim), w.f.data() + g * Mg * Kdim,
               static_cast<int>(Kdim), B, static_cast<int>(P), out, static_cast<int>(P), false);
      if (b)
        for (int64_t m = 0; m < Mg; ++m) {
          const float bv = b->f[g * Mg + m];
          for (int64_t p = 0; p < P; ++p) out[m * P + p] += bv;
        }
    }
  }
  return y;
}

// ---- pooling ---------------------------------------------------------------------------------------
CpuValuePtr op_pool(const Node& n, const CpuValue& x, bool is_max) {
  const int64_t N = x.shape[0], C = x.shape[1], H = x.shape[2], W = x.shape[3];
  auto k = n.get_ints("kernel_shape");
  auto st = n.get_ints("strides", {1, 1});
  auto pads = n.get_ints("pads", {0, 0, 0, 0});
  const bool ceil_mode = n.get_int("ceil_mode", 0) != 0;
  const bool count_pad = n.get_int("count_include_pad", 0) != 0;
  if (n.get_string("auto_pad", "NOTSET") != "NOTSET" && n.get_string("auto_pad", "NOTSET") != "VALID")
    fail(n, "auto_pad SAME is not supported for pooling");
  auto outdim = [&](int64_t in, int d) {
    double v = static_cast<double>(in + pads[d] + pads[d + 2] - k[d]) / st[d];
    return static_cast<int64_t>(ceil_mode ? std::ceil(v) : std::floor(v)) + 1;
  };
  const int64_t Ho = outdim(H, 0), Wo = outdim(W, 1);
  auto y = make_f({N, C, Ho, Wo});
#pragma omp parallel for collapse(2)
  for (int64_t b = 0; b < N; ++b)
    for (int64_t c = 0; c < C; ++c) {
      const float* in = x.f.data() + (b * C + c) * H * W;
      float* out = y->f.data() + (b * C + c) * Ho * Wo;
      for (int64_t oy = 0; oy < Ho; ++oy)
        for (int64_t ox = 0; ox < Wo; ++ox) {
          float acc = is_max ? -std::numeric_limits<float>::infinity() : 0.f;
          int cnt = 0;
          for (int64_t ky = 0; ky < k[0]; ++ky)
            for (int64_t kx = 0; kx < k[1]; ++kx) {
              const int64_t iy = oy * st[0] - pads[0] + ky, ix = ox * st[1] - pads[1] + kx;
              if (iy < 0 || iy >= H || ix < 0 || ix >= W) {
                if (count_pad && iy < H + pads[2] && ix < W + pads[3]) ++cnt;
                continue;
              }
              const float v = in[iy * W + ix];
              if (is_max) acc = std::max(acc, v);
              else acc += v;
              ++cnt;
            }
          out[oy * Wo + ox] = is_max ? acc : (cnt ? acc / cnt : 0.f);
        }
    }
  return y;
}

CpuValuePtr op_global_pool(const CpuValue& x, bool is_max) {
  const int64_t N = x.shape[0], C = x.shape[1];
  int64_t S = 1;
  for (size_t d = 2; d < x.shape.size(); ++d) S *= x.shape[d];
  std::vector<int64_t> os = {N, C};
  for (size_t d = 2; d < x.shape.size(); ++d) os.push_back(1);
  auto y = make_f(os);
#pragma omp parallel for
  for (int64_t i = 0; i < N * C; ++i) {
    const float* in = x.f.data() + i * S;
    double acc = is_max ? -std::numeric_limits<double>::infinity() : 0.0;
    for (int64_t s = 0; s < S; ++s) acc = is_max ? std::max<double>(acc, in[s]) : acc + in[s];
    y->f[i] = static_cast<float>(is_max ? acc : acc / S);
  }
  return y;
}

// ---- broadcasting binary ops ---------------------------------------------------------------------
std::vector<int64_t> broadcast_shape(const Node& n, const std::vector<int64_t>& a, const std::vector<int64_t>& b) {
  const size_t r = std::max(a.size(), b.size());
  std::vector<int64_t> o(r);
  for (size_t k = 0; k < r; ++k) {
    const int64_t da = k < r - a.size() ? 1 : a[k - (r - a.size())];
    const int64_t db = k < r - b.size() ? 1 : b[k - (r - b.size())];
    if (da != db && da != 1 && db != 1) fail(n, "shapes are not broadcastable");
    o[k] = da == 1 ? db : da;
  }
  return o;
}

// Strides of `s` broadcast to rank/shape `o` (0 on broadcast dims).
std::vector<int64_t> bstrides(const std::vector<int64_t>& s, const std::vector<int64_t>& o) {
  std::vector<int64_t> st(o.size(), 0);
  auto cs = strides_of(s);
  const size_t off = o.size() - s.size();
  for (size_t k = 0; k < s.size(); ++k) st[k + off] = s[k] == 1 ? 0 : cs[k];
  return st;
}

template <typename T, typename F>
void broadcast_apply(const std::vector<int64_t>& os, const T* a, const std::vector<int64_t>& as, const T* b,
                     const std::vector<int64_t>& bs, T* out, F f) {
  int64_t total = 1;
  for (auto d : os) total *= d;
  if (as == os && bs == os) {
#pragma omp parallel for if (total > 1 << 16)
    for (int64_t k = 0; k < total; ++k) out[k] = f(a[k], b[k]);
    return;
  }
  auto sa = bstrides(as, os), sb = bstrides(bs, os);
  const int r = static_cast<int>(os.size());
  const int64_t inner = r ? os[r - 1] : 1;
  const int64_t ia = r ? sa[r - 1] : 0, ib = r ? sb[r - 1] : 0;
  const int64_t rows = inner ? total / inner : 0;
#pragma omp parallel for if (total > 1 << 16)
  for (int64_t row = 0; row < rows; ++row) {
    int64_t oa = 0, ob = 0, rem = row;
    for (int k = r - 2; k >= 0; --k) {
      const int64_t idx = rem % os[k];
      rem /= os[k];
      oa += idx * sa[k];
      ob += idx * sb[k];
    }
    T* o = out + row * inner;
    for (int64_t j = 0; j < inner; ++j) o[j] = f(a[oa + j * ia], b[ob + j * ib]);
  }
}

CpuValuePtr op_binary(const Node& n, const CpuValue& a, const CpuValue& b) {
  const std::string& op = n.op_type;
  auto os = broadcast_shape(n, a.shape, b.shape);
  if (a.is_int && b.is_int) {
    auto y = make_i(os);
    auto fi = [&](int64_t x, int64_t z) -> int64_t {
      if (op == "Add") return x + z;
      if (op == "Sub") return x - z;
      if (op == "Mul") return x * z;
      if (op == "Div") return z ? x / z : 0;
      if (op == "Max") return std::max(x, z);
      if (op == "Min") return std::min(x, z);
      if (op == "Equal") return x == z;
      return static_cast<int64_t>(std::pow(x, z));
    };
    broadcast_apply<int64_t>(os, a.i.data(), a.shape, b.i.data(), b.shape, y->i.data(), fi);
    return y;
  }
  CpuValue af, bf;
  const CpuValue* pa = &a;
  const CpuValue* pb = &b;
  if (a.is_int) {
    af.shape = a.shape;
    af.f.assign(a.i.begin(), a.i.end());
    pa = &af;
  }
  if (b.is_int) {
    bf.shape = b.shape;
    bf.f.assign(b.i.begin(), b.i.end());
    pb = &bf;
  }
  auto y = make_f(os);
  const float* x = pa->f.data();
  const float* z = pb->f.data();
  if (op == "Add") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return p + q; });
  else if (op == "Sub") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return p - q; });
  else if (op == "Mul") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return p * q; });
  else if (op == "Div") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return p / q; });
  else if (op == "Pow") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return std::pow(p, q); });
  else if (op == "Max") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return std::max(p, q); });
  else if (op == "Min") broadcast_apply<float>(os, x, pa->shape, z, pb->shape, y->f.data(), [](float p, float q) { return std::min(p, q); });
  else fail(n, "unsupported binary op");
  return y;
}

CpuValuePtr op_unary(const Node& n, const CpuValue& x) {
  auto y = make_f(x.shape);
  const std::string& op = n.op_type;
  const float* a = x.f.data();
  float* o = y->f.data();
  const int64_t N = x.numel();
  std::function<float(float)> f;
  if (op == "Relu") f = [](float v) { return v > 0.f ? v : 0.f; };
  else if (op == "Sigmoid") f = [](float v) { return 1.f / (1.f + std::exp(-v)); };
  else if (op == "Tanh") f = [](float v) { return std::tanh(v); };
  else if (op == "Erf") f = [](float v) { return std::erf(v); };
  else if (op == "Sqrt") f = [](float v) { return std::sqrt(v); };
  else if (op == "Exp") f = [](float v) { return std::exp(v); };
  else if (op == "Log") f = [](float v) { return std::log(v); };
  else if (op == "Neg") f = [](float v) { return -v; };
  else if (op == "Abs") f = [](float v) { return std::fabs(v); };
  else if (op == "Reciprocal") f = [](float v) { return 1.f / v; };
  else if (op == "Sin") f = [](float v) { return std::sin(v); };
  else if (op == "Cos") f = [](float v) { return std::cos(v); };
  else if (op == "Floor") f = [](float v) { return std::floor(v); };
  else if (op == "Ceil") f = [](float v) { return std::ceil(v); };
  else if (op == "Round") f = [](float v) { return std::nearbyint(v); };  // half to even
  else if (op == "Sign") f = [](float v) { return static_cast<float>((v > 0.f) - (v < 0.f)); };
  else if (op == "HardSwish") f = [](float v) { return v * std::min(std::max(v / 6.f + 0.5f, 0.f), 1.f); };
  else if (op == "Softplus") f = [](float v) { return v > 20.f ? v : std::log1p(std::exp(v)); };
  else if (op == "HardSigmoid") {
    const float al = n.get_float("alpha", 0.2f), be = n.get_float("beta", 0.5f);
    f = [al, be](float v) { return std::min(std::max(al * v + be, 0.f), 1.f); };
  }
  else if (op == "LeakyRelu") {
    const float al = n.get_float("alpha", 0.01f);
    f = [al](float v) { return v >= 0.f ? v : al * v; };
  } else if (op == "Gelu") {
    if (n.get_string("approximate", "none") == "tanh")
      f = [](float v) { return 0.5f * v * (1.f + std::tanh(0.7978845608f * (v + 0.044715f * v * v * v))); };
    else
      f = [](float v) { return 0.5f * v * (1.f + std::erf(v * 0.70710678118f)); };
  } else {
    fail(n, "unsupported unary op");
  }
#pragma omp parallel for if (N > 1 << 16)
  for (int64_t k = 0; k < N; ++k) o[k] = f(a[k]);
  return y;
}

// ---- matmul -------------------------------------------------------------------------------------
CpuValuePtr op_matmul(const Node& n, const CpuValue& a, const CpuValue& b) {
  std::vector<int64_t> as = a.shape, bs = b.shape;
  const bool a1 = as.size() == 1, b1 = bs.size() == 1;
  if (a1) as.insert(as.begin(), 1);
  if (b1) bs.push_back(1);
  const int64_t M = as[as.size() - 2], K = as.back(), K2 = bs[bs.size() - 2], N = bs.back();
  if (K != K2) fail(n, "inner dimensions differ");
  std::vector<int64_t> ba(as.begin(), as.end() - 2), bb(bs.begin(), bs.end() - 2);
  auto bo = broadcast_shape(n, ba, bb);
  std::vector<int64_t> os = bo;
  if (!a1) os.push_back(M);
  if (!b1) os.push_back(N);
  auto y = make_f(os);
  int64_t batches = 1;
  for (auto d : bo) batches *= d;
  auto sa = bstrides(ba, bo), sb = bstrides(bb, bo);
  for (int64_t bi = 0; bi < batches; ++bi) {
    int64_t oa = 0, ob = 0, rem = bi;
    for (int k = static_cast<int>(bo.size()) - 1; k >= 0; --k) {
      const int64_t idx = rem % bo[k];
      rem /= bo[k];
      oa += idx * sa[k];
      ob += idx * sb[k];
    }
    cpu_gemm(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), a.f.data() + oa * M * K,
             static_cast<int>(K), b.f.data() + ob * K * N, static_cast<int>(N), y->f.data() + bi * M * N,
             static_cast<int>(N), false);
  }
  return y;
}

CpuValuePtr op_gemm(const Node& n, const CpuValue& a, const CpuValue& b, const CpuValue* c) {
  const bool ta = n.get_int("transA", 0) != 0, tb = n.get_int("transB", 0) != 0;
  const float alpha = n.get_float("alpha", 1.f), beta = n.get_float("beta", 1.f);
  const int64_t M = ta ? a.shape[1] : a.shape[0], K = ta ? a.shape[0] : a.shape[1];
  const int64_t N = tb ? b.shape[0] : b.shape[1];
  std::vector<float> at, bt;
  const float* A = a.f.data();
  const float* B = b.f.data();
  if (ta) {
    at.resize(M * K);
    for (int64_t i = 0; i < M; ++i)
      for (int64_t k = 0; k < K; ++k) at[i * K + k] = a.f[k * M + i];
    A = at.data();
  }
  if (tb) {
    bt.resize(K * N);
    for (int64_t k = 0; k < K; ++k)
      for (int64_t j = 0; j < N; ++j) bt[k * N + j] = b.f[j * K + k];
    B = bt.data();
  }
  auto y = make_f({M, N});
  cpu_gemm(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), A, static_cast<int>(K), B,
           static_cast<int>(N), y->f.data(), static_cast<int>(N), false);
  for (auto& v : y->f) v *= alpha;
  if (c && beta != 0.f) {
    auto sc = bstrides(c->shape, {M, N});
    for (int64_t i = 0; i < M; ++i)
      for (int64_t j = 0; j < N; ++j) y->f[i * N + j] += beta * c->f[i * sc[0] + j * sc[1]];
  }
  return y;
}

// ---- shape / data movement -----------------------------------------------------------------------
CpuValuePtr reshaped(const CpuValue& x, std::vector<int64_t> shape) {
  auto y = std::make_shared<CpuValue>(x);
  y->shape = std::move(shape);
  return y;
}

CpuValuePtr op_transpose(const Node& n, const CpuValue& x) {
  const size_t r = x.shape.size();
  std::vector<int64_t> perm = n.get_ints("perm");
  if (perm.empty()) {
    perm.resize(r);
    for (size_t k = 0; k < r; ++k) perm[k] = static_cast<int64_t>(r - 1 - k);
  }
  std::vector<int64_t> os(r);
  for (size_t k = 0; k < r; ++k) os[k] = x.shape[perm[k]];
  auto y = x.is_int ? make_i(os) : make_f(os);
  auto is = strides_of(x.shape);
  std::vector<int64_t> ps(r);
  for (size_t k = 0; k < r; ++k) ps[k] = is[perm[k]];
  const int64_t total = y->numel();
#pragma omp parallel for if (total > 1 << 16)
  for (int64_t o = 0; o < total; ++o) {
    int64_t rem = o, src = 0;
    for (int k = static_cast<int>(r) - 1; k >= 0; --k) {
      src += (rem % os[k]) * ps[k];
      rem /= os[k];
    }
    if (x.is_int) y->i[o] = x.i[src];
    else y->f[o] = x.f[src];
  }
  return y;
}

CpuValuePtr op_concat(const Node& n, const std::vector<const CpuValue*>& xs) {
  const int64_t axis = norm_axis(n.get_int("axis", 0), xs[0]->shape.size());
  std::vector<int64_t> os = xs[0]->shape;
  os[axis] = 0;
  bool is_int = true;
  for (auto* x : xs) {
    os[axis] += x->shape[axis];
    is_int = is_int && x->is_int;
  }
  auto y = is_int ? make_i(os) : make_f(os);
  int64_t outer = 1, inner = 1;
  for (int64_t k = 0; k < axis; ++k) outer *= os[k];
  for (size_t k = axis + 1; k < os.size(); ++k) inner *= os[k];
  int64_t off = 0;
  for (auto* x : xs) {
    const int64_t len = x->shape[axis] * inner;
    for (int64_t o = 0; o < outer; ++o)
      for (int64_t j = 0; j < len; ++j) {
        const int64_t di = o * os[axis] * inner + off + j, si = o * len + j;
        if (is_int) y->i[di] = x->i[si];
        else y->f[di] = x->is_int ? static_cast<float>(x->i[si]) : x->f[si];
      }
    off += len;
  }
  return y;
}

CpuValuePtr op_gather(const Node& n, const CpuValue& x, const CpuValue& idx) {
  const int64_t axis = norm_axis(n.get_int("axis", 0), x.shape.size());
  std::vector<int64_t> ind = as_ints(idx);
  std::vector<int64_t> os;
  for (int64_t k = 0; k < axis; ++k) os.push_back(x.shape[k]);
  for (auto d : idx.shape) os.push_back(d);
  for (size_t k = axis + 1; k < x.shape.size(); ++k) os.push_back(x.shape[k]);
  auto y = x.is_int ? make_i(os) : make_f(os);
  int64_t outer = 1, inner = 1;
  for (int64_t k = 0; k < axis; ++k) outer *= x.shape[k];
  for (size_t k = axis + 1; k < x.shape.size(); ++k) inner *= x.shape[k];
  const int64_t D = x.shape[axis];
  const int64_t nI = static_cast<int64_t>(ind.size());
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t t = 0; t < nI; ++t) {
      int64_t s = ind[t] < 0 ? ind[t] + D : ind[t];
      if (s < 0 || s >= D) fail(n, "index out of range");
      for (int64_t j = 0; j < inner; ++j) {
        const int64_t di = (o * nI + t) * inner + j, si = (o * D + s) * inner + j;
        if (x.is_int) y->i[di] = x.i[si];
        else y->f[di] = x.f[si];
      }
    }
  return y;
}

CpuValuePtr op_slice(const Node& n, const std::vector<const CpuValue*>& in, int64_t opset) {
  const CpuValue& x = *in[0];
  const size_t r = x.shape.size();
  std::vector<int64_t> starts, ends, axes, steps;
  if (opset < 10) {
    starts = n.get_ints("starts");
    ends = n.get_ints("ends");
    axes = n.get_ints("axes");
  } else {
    starts = as_ints(*in[1]);
    ends = as_ints(*in[2]);
    if (in.size() > 3 && in[3]) axes = as_ints(*in[3]);
    if (in.size() > 4 && in[4]) steps = as_ints(*in[4]);
  }
  if (axes.empty())
    for (size_t k = 0; k < starts.size(); ++k) axes.push_back(static_cast<int64_t>(k));
  if (steps.empty()) steps.assign(starts.size(), 1);
  std::vector<int64_t> b(r, 0), st(r, 1), os = x.shape;
  for (size_t k = 0; k < axes.size(); ++k) {
    const int64_t ax = norm_axis(axes[k], r), D = x.shape[ax], sp = steps[k];
    int64_t s = starts[k], e = ends[k];
    if (s < 0) s += D;
    if (e < 0) e += D;
    if (sp > 0) {
      s = std::clamp<int64_t>(s, 0, D);
      e = std::clamp<int64_t>(e, 0, D);
      os[ax] = std::max<int64_t>(0, (e - s + sp - 1) / sp);
    } else {
      s = std::clamp<int64_t>(s, 0, D - 1);
      e = std::clamp<int64_t>(e, -1, D - 1);
      os[ax] = std::max<int64_t>(0, (s - e - sp - 1) / (-sp));
    }
    b[ax] = s;
    st[ax] = sp;
  }
  auto y = x.is_int ? make_i(os) : make_f(os);
  auto is = strides_of(x.shape);
  const int64_t total = y->numel();
  for (int64_t o = 0; o < total; ++o) {
    int64_t rem = o, src = 0;
    for (int k = static_cast<int>(r) - 1; k >= 0; --k) {
      const int64_t idx = rem % os[k];
      rem /= os[k];
      src += (b[k] + idx * st[k]) * is[k];
    }
    if (x.is_int) y->i[o] = x.i[src];
    else y->f[o] = x.f[src];
  }
  return y;
}

CpuValuePtr op_softmax(const Node& n, const CpuValue& x, int64_t opset) {
  const size_t r = x.shape.size();
  const int64_t axis = norm_axis(n.get_int("axis", opset >= 13 ? -1 : 1), r);
  auto y = make_f(x.shape);
  int64_t outer = 1, D = 1, inner = 1;
  if (opset >= 13) {
    for (int64_t k = 0; k < axis; ++k) outer *= x.shape[k];
    D = x.shape[axis];
    for (size_t k = axis + 1; k < r; ++k) inner *= x.shape[k];
  } else {  // coerce to 2-D at axis
    for (int64_t k = 0; k < axis; ++k) outer *= x.shape[k];
    for (size_t k = axis; k < r; ++k) D *= x.shape[k];
  }
#pragma omp parallel for collapse(2) if (outer * inner > 64)
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t j = 0; j < inner; ++j) {
      const float* in = x.f.data() + o * D * inner + j;
      float* out = y->f.data() + o * D * inner + j;
      float m = -std::numeric_limits<float>::infinity();
      for (int64_t d = 0; d < D; ++d) m = std::max(m, in[d * inner]);
      double s = 0;
      for (int64_t d = 0; d < D; ++d) {
        const float e = std::exp(in[d * inner] - m);
        out[d * inner] = e;
        s += e;
      }
      const float inv = static_cast<float>(1.0 / s);
      for (int64_t d = 0; d < D; ++d) out[d * inner] *= inv;
    }
  return y;
}

CpuValuePtr op_layernorm(const Node& n, const CpuValue& x, const CpuValue* scale, const CpuValue* bias) {
  const size_t r = x.shape.size();
  const int64_t axis = norm_axis(n.get_int("axis", -1), r);
  const float eps = n.get_float("epsilon", 1e-5f);
  int64_t outer = 1, D = 1;
  for (int64_t k = 0; k < axis; ++k) outer *= x.shape[k];
  for (size_t k = axis; k < r; ++k) D *= x.shape[k];
  auto y = make_f(x.shape);
#pragma omp parallel for if (outer > 16)
  for (int64_t o = 0; o < outer; ++o) {
    const float* in = x.f.data() + o * D;
    float* out = y->f.data() + o * D;
    double mean = 0, var = 0;
    for (int64_t d = 0; d < D; ++d) mean += in[d];
    mean /= D;
    for (int64_t d = 0; d < D; ++d) var += (in[d] - mean) * (in[d] - mean);
    var /= D;
    const float inv = static_cast<float>(1.0 / std::sqrt(var + eps));
    for (int64_t d = 0; d < D; ++d) {
      float v = static_cast<float>(in[d] - mean) * inv;
      if (scale) v *= scale->f[d % scale->f.size()];
      if (bias) v += bias->f[d % bias->f.size()];
      out[d] = v;
    }
  }
  return y;
}

CpuValuePtr op_reduce(const Node& n, const std::vector<const CpuValue*>& in, int64_t opset) {
  const CpuValue& x = *in[0];
  const size_t r = x.shape.size();
  std::vector<int64_t> axes = n.get_ints("axes");
  if (axes.empty() && in.size() > 1 && in[1]) axes = as_ints(*in[1]);
  (void)opset;
  const bool keep = n.get_int("keepdims", 1) != 0;
  std::vector<bool> red(r, axes.empty());
  for (auto a : axes) red[norm_axis(a, r)] = true;
  std::vector<int64_t> os, ks;
  for (size_t k = 0; k < r; ++k) {
    if (red[k]) {
      if (keep) os.push_back(1);
      ks.push_back(1);
    } else {
      os.push_back(x.shape[k]);
      ks.push_back(x.shape[k]);
    }
  }
  auto y = make_f(os);
  const bool is_max = n.op_type == "ReduceMax";
  std::vector<double> acc(static_cast<size_t>(y->numel()), is_max ? -std::numeric_limits<double>::infinity() : 0.0);
  auto xs = strides_of(x.shape), kst = strides_of(ks);
  const int64_t total = x.numel();
  int64_t cnt = 1;
  for (size_t k = 0; k < r; ++k)
    if (red[k]) cnt *= x.shape[k];
  for (int64_t e = 0; e < total; ++e) {
    int64_t rem = e, o = 0;
    for (size_t k = 0; k < r; ++k) {
      const int64_t idx = rem / xs[k];
      rem %= xs[k];
      if (!red[k]) o += idx * kst[k];
    }
    if (is_max) acc[o] = std::max(acc[o], static_cast<double>(x.f[e]));
    else acc[o] += x.f[e];
  }
  const bool mean = n.op_type == "ReduceMean";
  for (size_t k = 0; k < acc.size(); ++k) y->f[k] = static_cast<float>(mean ? acc[k] / cnt : acc[k]);
  return y;
}

}  // namespace

// Pad: constant (value from the attribute or input 2), reflect or edge, any rank; negative pads crop.
CpuValuePtr op_pad(const Node& n, const std::vector<const CpuValue*>& in) {
  const CpuValue& x = *in[0];
  const size_t r = x.shape.size();
  std::vector<int64_t> pads = n.get_ints("pads");
  if (pads.empty() && in.size() > 1 && in[1]) pads = as_ints(*in[1]);
  float value = n.get_float("value", 0.f);
  if (in.size() > 2 && in[2]) value = in[2]->is_int ? static_cast<float>(in[2]->i.at(0)) : in[2]->f.at(0);
  std::vector<int64_t> full(2 * r, 0);
  if (in.size() > 3 && in[3]) {  // opset 18 axes
    auto axes = as_ints(*in[3]);
    if (pads.size() != 2 * axes.size()) fail(n, "pads/axes mismatch");
    for (size_t k = 0; k < axes.size(); ++k) {
      const int64_t a = norm_axis(axes[k], r);
      full[a] = pads[k];
      full[a + r] = pads[k + axes.size()];
    }
  } else {
    if (pads.size() != 2 * r) fail(n, "expected 2 * rank pads");
    full = pads;
  }
  const std::string mode = n.get_string("mode", "constant");
  std::vector<int64_t> os(r);
  for (size_t k = 0; k < r; ++k) os[k] = x.shape[k] + full[k] + full[k + r];
  auto y = make_f(os);
  auto xs = strides_of(x.shape), ys = strides_of(os);
  const int64_t total = y->numel();
#pragma omp parallel for if (total > 1 << 16)
  for (int64_t e = 0; e < total; ++e) {
    int64_t rem = e, src = 0;
    bool inside = true;
    for (size_t k = 0; k < r; ++k) {
      int64_t i = rem / ys[k] - full[k];
      rem %= ys[k];
      const int64_t D = x.shape[k];
      if (i < 0 || i >= D) {
        if (mode == "edge") i = i < 0 ? 0 : D - 1;
        else if (mode == "reflect") {
          const int64_t p = 2 * (D - 1);
          i = p ? ((i % p) + p) % p : 0;
          if (i >= D) i = p - i;
        } else inside = false;
      }
      src += i * xs[k];
    }
    y->f[e] = inside ? x.f[src] : value;
  }
  return y;
}

// ConvTranspose (2-D, any group / stride / dilation / pads / output_padding / output_shape), as the
// scatter form of its definition: every input pixel adds its kernel-weighted copy into the output.
CpuValuePtr op_conv_transpose(const Node& n, const CpuValue& x, const CpuValue& w, const CpuValue* b) {
  if (x.shape.size() != 4 || w.shape.size() != 4) fail(n, "only 2-D transposed convolution is supported");
  const int64_t N = x.shape[0], C = x.shape[1], H = x.shape[2], W = x.shape[3];
  const int64_t G = n.get_int("group", 1), Mg = w.shape[1], M = Mg * G, kh = w.shape[2], kw = w.shape[3];
  if (w.shape[0] != C || C % G) fail(n, "weight / channel mismatch");
  const auto st = n.get_ints("strides", {1, 1}), dl = n.get_ints("dilations", {1, 1}), op = n.get_ints("output_padding", {0, 0});
  auto pads = n.get_ints("pads", {0, 0, 0, 0});
  const int64_t k[2] = {kh, kw}, in[2] = {H, W};
  int64_t out[2];
  const auto os = n.get_ints("output_shape");
  const std::string ap = n.get_string("auto_pad", "NOTSET");
  for (int d = 0; d < 2; ++d) {
    const int64_t full = st[d] * (in[d] - 1) + op[d] + (k[d] - 1) * dl[d] + 1;
    if (!os.empty() || ap == "SAME_UPPER" || ap == "SAME_LOWER") {
      out[d] = !os.empty() ? os[os.size() - 2 + d] : in[d] * st[d];
      const int64_t total = full - out[d];
      const bool upper = ap != "SAME_LOWER";  // output_shape without auto_pad: the SAME_UPPER split
      pads[d] = upper ? total / 2 : total - total / 2;
      pads[d + 2] = total - pads[d];
    } else {
      out[d] = full - pads[d] - pads[d + 2];
    }
  }
  auto y = make_f({N, M, out[0], out[1]});
  const int64_t Cg = C / G;
#pragma omp parallel for collapse(2)
  for (int64_t bn = 0; bn < N; ++bn)
    for (int64_t m = 0; m < M; ++m) {
      const int64_t g = m / Mg, mo = m % Mg;
      float* yo = y->f.data() + (bn * M + m) * out[0] * out[1];
      if (b) std::fill(yo, yo + out[0] * out[1], b->f[m]);
      for (int64_t c = g * Cg; c < (g + 1) * Cg; ++c) {
        const float* xi = x.f.data() + (bn * C + c) * H * W;
        const float* wk = w.f.data() + (c * Mg + mo) * kh * kw;
        for (int64_t iy = 0; iy < H; ++iy)
          for (int64_t ix = 0; ix < W; ++ix) {
            const float v = xi[iy * W + ix];
            for (int64_t ky = 0; ky < kh; ++ky) {
              const int64_t oy = iy * st[0] - pads[0] + ky * dl[0];
              if (oy < 0 || oy >= out[0]) continue;
              for (int64_t kx = 0; kx < kw; ++kx) {
                const int64_t ox = ix * st[1] - pads[1] + kx * dl[1];
                if (ox >= 0 && ox < out[1]) yo[oy * out[1] + ox] += v * wk[ky * kw + kx];
              }
            }
          }
      }
    }
  return y;
}

// Resize (opset 10+) / Upsample on [N, C, H, W]: nearest or linear over H, W (N, C scales 1), the
// ONNX coordinate transforms and nearest rounding modes; linear clamps neighbour indices (= the
// specification's edge padding).
CpuValuePtr op_resize(const Node& n, const std::vector<const CpuValue*>& in, int64_t opset) {
  const CpuValue& x = *in[0];
  if (x.shape.size() != 4) fail(n, "only 4-D inputs");
  const bool upsample = n.op_type == "Upsample";
  std::vector<float> scales = n.get_floats("scales");
  std::vector<int64_t> sizes;
  auto floats = [](const CpuValue* v) {
    std::vector<float> f;
    if (v) f = v->is_int ? std::vector<float>(v->i.begin(), v->i.end()) : v->f;
    return f;
  };
  if (scales.empty()) {
    if (upsample || (opset < 11 && in.size() > 1)) scales = floats(in.size() > 1 ? in[1] : nullptr);
    else {
      if (in.size() > 2) scales = floats(in[2]);
      if (scales.empty() && in.size() > 3 && in[3]) sizes = as_ints(*in[3]);
    }
  }
  const int64_t N = x.shape[0], C = x.shape[1], H = x.shape[2], W = x.shape[3];
  int64_t Ho, Wo;
  float sh, sw;
  if (!sizes.empty()) {
    Ho = sizes[2];
    Wo = sizes[3];
    sh = static_cast<float>(Ho) / H;
    sw = static_cast<float>(Wo) / W;
  } else {
    if (scales.size() != 4) fail(n, "expected 4 scales");
    sh = scales[2];
    sw = scales[3];
    Ho = static_cast<int64_t>(std::floor(H * static_cast<double>(sh)));
    Wo = static_cast<int64_t>(std::floor(W * static_cast<double>(sw)));
  }
  const bool legacy = upsample || opset < 11;
  const std::string mode = n.get_string("mode", "nearest");
  const std::string cm = legacy ? "asymmetric" : n.get_string("coordinate_transformation_mode", "half_pixel");
  const std::string nm = legacy ? "floor" : n.get_string("nearest_mode", "round_prefer_floor");
  auto src = [&](int64_t o, float scale, int64_t len, int64_t olen) -> float {
    if (cm == "asymmetric") return o / scale;
    if (cm == "align_corners") return olen > 1 ? o * static_cast<float>(len - 1) / static_cast<float>(olen - 1) : 0.f;
    if (cm == "pytorch_half_pixel") return olen > 1 ? (o + 0.5f) / scale - 0.5f : 0.f;
    if (cm == "tf_half_pixel_for_nn") return (o + 0.5f) / scale;
    if (cm == "half_pixel") return (o + 0.5f) / scale - 0.5f;
    fail(n, "unsupported coordinate_transformation_mode " + cm);
  };
  auto nearest = [&](float v, int64_t len) -> int64_t {
    const float f = std::floor(v);
    int64_t i;
    if (nm == "floor") i = static_cast<int64_t>(f);
    else if (nm == "ceil") i = static_cast<int64_t>(std::ceil(v));
    else if (v - f == 0.5f) i = static_cast<int64_t>(f) + (nm == "round_prefer_ceil" ? 1 : 0);
    else i = static_cast<int64_t>(std::nearbyint(v));
    return std::min(std::max<int64_t>(i, 0), len - 1);
  };
  const bool linear = mode == "linear" || mode == "bilinear";
  if (!linear && mode != "nearest") fail(n, "unsupported mode " + mode);
  auto y = make_f({N, C, Ho, Wo});
#pragma omp parallel for collapse(2)
  for (int64_t p = 0; p < N * C; ++p)
    for (int64_t oy = 0; oy < Ho; ++oy) {
      const float* xi = x.f.data() + p * H * W;
      float* yo = y->f.data() + (p * Ho + oy) * Wo;
      const float fy = src(oy, sh, H, Ho);
      for (int64_t ox = 0; ox < Wo; ++ox) {
        const float fx = src(ox, sw, W, Wo);
        if (!linear) {
          yo[ox] = xi[nearest(fy, H) * W + nearest(fx, W)];
          continue;
        }
        const float y0f = std::floor(fy), x0f = std::floor(fx), ay = fy - y0f, ax = fx - x0f;
        auto cl = [](int64_t v, int64_t len) { return std::min(std::max<int64_t>(v, 0), len - 1); };
        const int64_t y0 = cl(static_cast<int64_t>(y0f), H), y1 = cl(static_cast<int64_t>(y0f) + 1, H);
        const int64_t x0 = cl(static_cast<int64_t>(x0f), W), x1 = cl(static_cast<int64_t>(x0f) + 1, W);
        const float top = xi[y0 * W + x0] * (1.f - ax) + xi[y0 * W + x1] * ax;
        const float bot = xi[y1 * W + x0] * (1.f - ax) + xi[y1 * W + x1] * ax;
        yo[ox] = top * (1.f - ay) + bot * ay;
      }
    }
  return y;
}

// Comparisons -> bool (int 0 / 1); Where(cond, a, b) with broadcasting; Not / And / Or on bools.
CpuValuePtr op_compare(const Node& n, const CpuValue& a, const CpuValue& b) {
  const std::string& op = n.op_type;
  auto os = broadcast_shape(n, a.shape, b.shape);
  auto tof = [](const CpuValue& v) {
    return v.is_int ? std::vector<float>(v.i.begin(), v.i.end()) : v.f;
  };
  const std::vector<float> fa = tof(a), fb = tof(b);
  auto y = make_f(os);
  std::function<float(float, float)> f;
  if (op == "Greater") f = [](float p, float q) { return static_cast<float>(p > q); };
  else if (op == "Less") f = [](float p, float q) { return static_cast<float>(p < q); };
  else if (op == "Equal") f = [](float p, float q) { return static_cast<float>(p == q); };
  else if (op == "GreaterOrEqual") f = [](float p, float q) { return static_cast<float>(p >= q); };
  else if (op == "LessOrEqual") f = [](float p, float q) { return static_cast<float>(p <= q); };
  else if (op == "And") f = [](float p, float q) { return static_cast<float>(p != 0.f && q != 0.f); };
  else if (op == "Or") f = [](float p, float q) { return static_cast<float>(p != 0.f || q != 0.f); };
  else fail(n, "unsupported comparison");
  broadcast_apply<float>(os, fa.data(), a.shape, fb.data(), b.shape, y->f.data(), f);
  auto r = make_i(os);
  for (size_t k = 0; k < r->i.size(); ++k) r->i[k] = y->f[k] != 0.f;
  return r;
}

CpuValuePtr op_where(const Node& n, const CpuValue& c, const CpuValue& a, const CpuValue& b) {
  // select(c, a, b) = a * c + b * (1 - c) would turn inf * 0 into NaN: broadcast c against a, then
  // pick per element
  auto tof = [](const CpuValue& v) { return v.is_int ? std::vector<float>(v.i.begin(), v.i.end()) : v.f; };
  const std::vector<float> fc = tof(c), fa = tof(a), fb = tof(b);
  auto s1 = broadcast_shape(n, c.shape, a.shape);
  auto os = broadcast_shape(n, s1, b.shape);
  auto ca = make_f(os), cb = make_f(os), cc = make_f(os);
  std::vector<float> zeros(1, 0.f);
  const std::vector<int64_t> one = {1};
  broadcast_apply<float>(os, fa.data(), a.shape, zeros.data(), one, ca->f.data(), [](float p, float) { return p; });
  broadcast_apply<float>(os, fb.data(), b.shape, zeros.data(), one, cb->f.data(), [](float p, float) { return p; });
  broadcast_apply<float>(os, fc.data(), c.shape, zeros.data(), one, cc->f.data(), [](float p, float) { return p; });
  for (size_t k = 0; k < ca->f.size(); ++k) ca->f[k] = cc->f[k] != 0.f ? ca->f[k] : cb->f[k];
  return ca;
}

// Split: sizes from the attribute (opset < 13), input 1, or equal parts (the last may be smaller).
std::vector<CpuValuePtr> op_split(const Node& n, const std::vector<const CpuValue*>& in) {
  const CpuValue& x = *in[0];
  const size_t r = x.shape.size();
  const int64_t axis = norm_axis(n.get_int("axis", 0), r);
  std::vector<int64_t> sizes = n.get_ints("split");
  if (sizes.empty() && in.size() > 1 && in[1]) sizes = as_ints(*in[1]);
  const int64_t parts = static_cast<int64_t>(n.outputs.size()), D = x.shape[axis];
  if (sizes.empty()) {
    const int64_t each = (D + parts - 1) / parts;
    for (int64_t k = 0, s = 0; k < parts; ++k, s += each) sizes.push_back(std::min(each, D - s));
  }
  int64_t outer = 1, inner = 1;
  for (int64_t k = 0; k < axis; ++k) outer *= x.shape[k];
  for (size_t k = axis + 1; k < r; ++k) inner *= x.shape[k];
  std::vector<CpuValuePtr> outs;
  int64_t s0 = 0;
  for (int64_t k = 0; k < parts; ++k) {
    auto os = x.shape;
    os[axis] = sizes[k];
    auto y = make_f(os);
    for (int64_t o = 0; o < outer; ++o)
      std::copy_n(x.f.data() + (o * D + s0) * inner, sizes[k] * inner, y->f.data() + o * sizes[k] * inner);
    s0 += sizes[k];
    outs.push_back(y);
  }
  if (s0 != D) fail(n, "split sizes do not cover the axis");
  return outs;
}

// ------------------------------------------------------------------------------------------------

CpuExecutor::CpuExecutor(onnx::Model model) : model_(std::move(model)) {
  for (auto& kv : model_.initializers) {
    auto v = std::make_shared<CpuValue>();
    v->shape = kv.second.dims;
    if (!kv.second.i.empty() || !onnx::is_float_type(kv.second.dtype)) {
      v->is_int = true;
      v->i = kv.second.i;
    } else {
      v->f = kv.second.f;
    }
    consts_[kv.first] = v;
  }
  for (size_t k = 0; k < model_.nodes.size(); ++k)
    for (auto& in : model_.nodes[k].inputs) last_use_[in] = k;
  for (auto& o : model_.outputs) last_use_[o.name] = model_.nodes.size();
}

CpuValuePtr CpuExecutor::run(const CpuValuePtr& input, std::unordered_map<std::string, CpuValuePtr>* trace) {
  if (model_.inputs.empty()) throw std::runtime_error("model has no inputs");
  std::unordered_map<std::string, CpuValuePtr> env;
  env[model_.inputs[0].name] = input;
  const int64_t opset = model_.opset();
  auto get = [&](const std::string& name) -> const CpuValue* {
    if (name.empty()) return nullptr;
    auto it = env.find(name);
    if (it != env.end()) return it->second.get();
    auto c = consts_.find(name);
    if (c != consts_.end()) return c->second.get();
    throw std::runtime_error("cpu executor: undefined value " + name);
  };
  for (size_t k = 0; k < model_.nodes.size(); ++k) {
    const Node& n = model_.nodes[k];
    std::vector<const CpuValue*> in;
    for (auto& s : n.inputs) in.push_back(get(s));
    const std::string& op = n.op_type;
    CpuValuePtr out;
    if (op == "Conv") {
      out = op_conv(n, *in[0], *in[1], in.size() > 2 ? in[2] : nullptr);
    } else if (op == "BatchNormalization") {
      const CpuValue& x = *in[0];
      const float eps = n.get_float("epsilon", 1e-5f);
      out = make_f(x.shape);
      const int64_t N = x.shape[0], C = x.shape[1];
      const int64_t S = x.numel() / (N * C);
#pragma omp parallel for collapse(2)
      for (int64_t b = 0; b < N; ++b)
        for (int64_t c = 0; c < C; ++c) {
          const float sc = in[1]->f[c] / std::sqrt(in[4]->f[c] + eps);
          const float sh = in[2]->f[c] - in[3]->f[c] * sc;
          const float* xi = x.f.data() + (b * C + c) * S;
          float* yo = out->f.data() + (b * C + c) * S;
          for (int64_t s = 0; s < S; ++s) yo[s] = xi[s] * sc + sh;
        }
    } else if (op == "Relu" || op == "Sigmoid" || op == "Tanh" || op == "Erf" || op == "Sqrt" || op == "Exp" ||
               op == "Log" || op == "Neg" || op == "Abs" || op == "Reciprocal" || op == "LeakyRelu" ||
               op == "Gelu" || op == "HardSigmoid" || op == "HardSwish" || op == "Softplus" || op == "Sin" || op == "Cos" ||
               op == "Floor" || op == "Ceil" || op == "Round" || op == "Sign") {
      out = op_unary(n, *in[0]);
    } else if (op == "Clip") {
      float lo = -std::numeric_limits<float>::infinity(), hi = std::numeric_limits<float>::infinity();
      if (opset < 11) {
        lo = n.get_float("min", lo);
        hi = n.get_float("max", hi);
      } else {
        if (in.size() > 1 && in[1]) lo = in[1]->f[0];
        if (in.size() > 2 && in[2]) hi = in[2]->f[0];
      }
      out = make_f(in[0]->shape);
      for (size_t e = 0; e < out->f.size(); ++e) out->f[e] = std::clamp(in[0]->f[e], lo, hi);
    } else if (op == "Add" || op == "Sub" || op == "Mul" || op == "Div" || op == "Pow" || op == "Max" ||
               op == "Min" || (op == "Equal" && in[0]->is_int && in[1]->is_int)) {
      out = op_binary(n, *in[0], *in[1]);
    } else if (op == "MaxPool" || op == "AveragePool") {
      out = op_pool(n, *in[0], op == "MaxPool");
    } else if (op == "GlobalAveragePool" || op == "GlobalMaxPool") {
      out = op_global_pool(*in[0], op == "GlobalMaxPool");
    } else if (op == "Flatten") {
      const int64_t axis = norm_axis(n.get_int("axis", 1), in[0]->shape.size());
      int64_t a = 1, b = 1;
      for (int64_t d = 0; d < static_cast<int64_t>(in[0]->shape.size()); ++d) (d < axis ? a : b) *= in[0]->shape[d];
      out = reshaped(*in[0], {a, b});
    } else if (op == "Reshape") {
      std::vector<int64_t> shape = opset >= 5 ? as_ints(*in[1]) : n.get_ints("shape");
      const bool allowzero = n.get_int("allowzero", 0) != 0;
      int64_t known = 1, neg = -1;
      for (size_t d = 0; d < shape.size(); ++d) {
        if (shape[d] == 0 && !allowzero) shape[d] = in[0]->shape[d];
        if (shape[d] == -1) neg = static_cast<int64_t>(d);
        else known *= shape[d];
      }
      if (neg >= 0) shape[neg] = known ? in[0]->numel() / known : 0;
      int64_t count = 1;
      for (auto d : shape) count *= d;
      if (count != in[0]->numel()) fail(n, "target shape does not match the element count");
      out = reshaped(*in[0], shape);
    } else if (op == "Squeeze" || op == "Unsqueeze") {
      std::vector<int64_t> axes = n.get_ints("axes");
      if (axes.empty() && in.size() > 1 && in[1]) axes = as_ints(*in[1]);
      std::vector<int64_t> s = in[0]->shape;
      if (op == "Squeeze") {
        std::vector<int64_t> o;
        for (size_t d = 0; d < s.size(); ++d) {
          bool sq = axes.empty() ? s[d] == 1 : false;
          for (auto a : axes)
            if (norm_axis(a, s.size()) == static_cast<int64_t>(d)) sq = true;
          if (!sq) o.push_back(s[d]);
        }
        s = o;
      } else {
        const size_t r = s.size() + axes.size();
        std::vector<int64_t> na;
        for (auto a : axes) na.push_back(norm_axis(a, r));
        std::sort(na.begin(), na.end());
        for (auto a : na) s.insert(s.begin() + a, 1);
      }
      out = reshaped(*in[0], s);
    } else if (op == "Transpose") {
      out = op_transpose(n, *in[0]);
    } else if (op == "Concat") {
      out = op_concat(n, in);
    } else if (op == "Gather") {
      out = op_gather(n, *in[0], *in[1]);
    } else if (op == "Slice") {
      out = op_slice(n, in, opset);
    } else if (op == "Shape") {
      out = make_i({static_cast<int64_t>(in[0]->shape.size())});
      out->i = in[0]->shape;
    } else if (op == "Expand") {
      std::vector<int64_t> target = as_ints(*in[1]);
      auto os = broadcast_shape(n, in[0]->shape, target);
      CpuValue zero;
      zero.shape = {1};
      if (in[0]->is_int) {
        zero.is_int = true;
        zero.i = {0};
      } else {
        zero.f = {0.f};
      }
      Node add = n;
      add.op_type = "Add";
      auto tmp = op_binary(add, *in[0], zero);
      // broadcast to os
      CpuValue z2;
      z2.shape = os;
      z2.is_int = in[0]->is_int;
      if (z2.is_int) z2.i.assign(static_cast<size_t>(z2.numel()), 0);
      else z2.f.assign(static_cast<size_t>(z2.numel()), 0.f);
      out = op_binary(add, *tmp, z2);
    } else if (op == "Cast") {
      const int to = static_cast<int>(n.get_int("to", onnx::FLOAT));
      if (to == onnx::BOOL) {
        out = make_i(in[0]->shape);
        for (size_t e = 0; e < out->i.size(); ++e) out->i[e] = in[0]->is_int ? in[0]->i[e] != 0 : in[0]->f[e] != 0.f;
      } else if (onnx::is_float_type(to)) {
        out = make_f(in[0]->shape);
        if (in[0]->is_int) out->f.assign(in[0]->i.begin(), in[0]->i.end());
        else out->f = in[0]->f;
      } else {
        out = make_i(in[0]->shape);
        if (in[0]->is_int) out->i = in[0]->i;
        else
          for (size_t e = 0; e < out->i.size(); ++e) out->i[e] = static_cast<int64_t>(in[0]->f[e]);
      }
    } else if (op == "Identity" || op == "Dropout") {
      out = std::make_shared<CpuValue>(*in[0]);
    } else if (op == "Gemm") {
      out = op_gemm(n, *in[0], *in[1], in.size() > 2 ? in[2] : nullptr);
    } else if (op == "MatMul") {
      out = op_matmul(n, *in[0], *in[1]);
    } else if (op == "Softmax") {
      out = op_softmax(n, *in[0], opset);
    } else if (op == "LayerNormalization") {
      out = op_layernorm(n, *in[0], in.size() > 1 ? in[1] : nullptr, in.size() > 2 ? in[2] : nullptr);
    } else if (op == "ReduceMean" || op == "ReduceSum" || op == "ReduceMax") {
      out = op_reduce(n, in, opset);
    } else if (op == "Pad") {
      out = op_pad(n, in);
    } else if (op == "ConvTranspose") {
      out = op_conv_transpose(n, *in[0], *in[1], in.size() > 2 ? in[2] : nullptr);
    } else if (op == "Resize" || op == "Upsample") {
      out = op_resize(n, in, opset);
    } else if (op == "Greater" || op == "Less" || op == "GreaterOrEqual" || op == "LessOrEqual" || op == "And" ||
               op == "Or" || (op == "Equal" && !(in[0]->is_int && in[1]->is_int))) {
      out = op_compare(n, *in[0], *in[1]);
    } else if (op == "Where") {
      out = op_where(n, *in[0], *in[1], *in[2]);
    } else if (op == "Not") {
      out = make_i(in[0]->shape);
      for (size_t e = 0; e < out->i.size(); ++e) out->i[e] = in[0]->is_int ? in[0]->i[e] == 0 : in[0]->f[e] == 0.f;
    } else if (op == "Split") {
      auto outs = op_split(n, in);
      for (size_t k = 1; k < outs.size(); ++k)
        if (!n.outputs[k].empty()) {
          env[n.outputs[k]] = outs[k];
          if (trace) (*trace)[n.outputs[k]] = outs[k];
        }
      out = outs[0];
    } else {
      throw std::runtime_error("cpu executor: unsupported op " + op + " (" + n.name + ")");
    }
    env[n.outputs[0]] = out;
    if (trace) (*trace)[n.outputs[0]] = out;
    for (auto& s : n.inputs) {
      auto lu = last_use_.find(s);
      if (lu != last_use_.end() && lu->second == k && !trace) env.erase(s);
    }
  }
  auto it = env.find(model_.outputs.at(0).name);
  if (it == env.end()) throw std::runtime_error("cpu executor: output not produced");
  return it->second;
}

}  // namespace die
