// Generic memory-bound kernels that let the HIP planner run graphs beyond the ResNet / ViT patterns
// (VERDICT r2 "model-agnostic device execution"; the reference binds input 0 / output 0 of any
// single-input ONNX model, /root/reference/src/inference_engine.cpp:33-69): rank-2/3 graph inputs,
// channel counts that are not a multiple of 8 (stored padded), concat / slice along the channel
// axis, broadcast binary ops between activations, strided output casts.  All bf16 tensors may be
// split (fp32 mode, common.h): the lo plane follows the hi plane by the tensor's element count at
// batch B (rows x pitch), passed in explicitly.  16-byte vector loads/stores where the pitch and
// column offsets are multiples of 8 (the planner pads every stored row to that).
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

inline int grid_for(long long work, int block = 256, int cap = 8192) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  return static_cast<int>(g > cap ? cap : g);
}

// fp32 [R][F] (dense) -> bf16 / split [R][Fp], pad columns zero.  One thread per 8 output columns.
__global__ void rows_prep_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long long R, int F, int Fp,
                                 int split) {
  const int G = Fp / 8;
  const long long total = R * G, plane = R * Fp;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / G;
    const int c0 = static_cast<int>(i - r * G) * 8;
    const float* src = x + r * F + c0;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = c0 + t < F ? src[t] : 0.f;
    store8v(y + r * Fp + c0, plane, split != 0, v);
  }
}

// fp32 NCHW [B][C][HW] -> (affine) -> bf16 NHWC [B][HW][Cp], any C (Cp % 8 == 0, pad channels 0).
// One thread per (pixel, 8-channel group); the strided NCHW reads of one group are 8 planes apart.
__global__ void input_prep_wide_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                       const float* __restrict__ shift, uint16_t* __restrict__ out, int B, int C,
                                       int HW, int Cp, int split) {
  const int G = Cp / 8;
  const long long total = static_cast<long long>(B) * HW * G, plane = static_cast<long long>(B) * HW * Cp;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i % G);
    const long long pix = i / G;
    const long long b = pix / HW, p = pix - b * HW;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = g * 8 + t;
      if (c < C) {
        const float xv = x[(b * C + c) * HW + p];
        v[t] = scale ? xv * scale[c] + shift[c] : xv;
      } else {
        v[t] = 0.f;
      }
    }
    store8v(out + pix * Cp + g * 8, plane, split != 0, v);
  }
}

// out[r][out_col + j] = in[r][in_col + j], j < ncols (ncols, cols and pitches % 8 == 0).
__global__ void copy_cols_kernel(const uint16_t* __restrict__ x, long long xplane, int ldx, int colx,
                                 uint16_t* __restrict__ y, long long yplane, int ldy, int coly, long long R, int ncols,
                                 int split) {
  const int G = ncols / 8;
  const long long total = R * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / G;
    const int c = static_cast<int>(i - r * G) * 8;
    const uint16_t* s = x + r * ldx + colx + c;
    uint16_t* d = y + r * ldy + coly + c;
    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
    if (split) *reinterpret_cast<uint4*>(d + yplane) = *reinterpret_cast<const uint4*>(s + xplane);
  }
}

// Activation codes (kernels.h unary_rows).  The transcendental ones use the accurate libm forms
// (not the __expf-style intrinsics): they also serve the fp32 (split) mode, whose values carry
// ~16 significant bits.
__device__ __forceinline__ float apply_act(float v, int act, float a, float b) {
  switch (act) {
    case 1: return fmaxf(v, 0.f);
    case 2: return gelu_erf(v);
    case 3: return fminf(fmaxf(v, a), b);
    case 4: return 1.f / (1.f + __expf(-v));
    case 5: return tanhf(v);
    case 6: return v >= 0.f ? v : v * a;
    case 7: return expf(v);
    case 8: return fabsf(v);
    case 9: return sqrtf(v);
    case 10: return -v;
    case 11: return 1.f / v;
    case 12: return logf(v);
    case 13: return erff(v);
    case 14: return a == 2.f ? v * v : a == 0.5f ? sqrtf(v) : a == 1.f ? v : powf(v, a);
    case 15: return fminf(fmaxf(a * v + b, 0.f), 1.f);                   // HardSigmoid(alpha, beta)
    case 16: return v * fminf(fmaxf(v * (1.f / 6.f) + 0.5f, 0.f), 1.f);  // HardSwish
    case 17: return v > 20.f ? v : log1pf(expf(v));                       // Softplus
    case 18: return v > a ? 1.f : 0.f;                                    // comparisons with a constant
    case 19: return v < a ? 1.f : 0.f;
    case 20: return v == a ? 1.f : 0.f;
    case 21: return v >= a ? 1.f : 0.f;
    case 22: return v <= a ? 1.f : 0.f;
    case 23: return v == 0.f ? 1.f : 0.f;                                 // Not (bool as 0 / 1)
    case 24: return v != 0.f ? 1.f : 0.f;                                 // Cast to bool
    default: return v;
  }
}

// out = act(x (op) y) over rows [R][C] (pitch C); y: ymode 0 = same shape, 1 = one row of C per
// sample broadcast over its rows_per_sample rows (squeeze-excitation scales, [B, C, 1, 1] gates).
// op: 0 add, 1 sub, 2 mul, 3 div.
__global__ void binary_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ y, uint16_t* __restrict__ out,
                              long long R, int C, long long rows_per_sample, int ymode, int op, int act, float a,
                              float b, long long plane, long long yplane, const long long* __restrict__ live, int split,
                              int Cl) {
  long long Rl = R;
  if (live) Rl = min(R, *live * rows_per_sample);
  const int G = C / 8;
  const long long total = Rl * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / G;
    const int c = static_cast<int>(i - r * G) * 8;
    float u[8], w[8];
    load8v(x + r * C + c, plane, split != 0, u);
    const long long yr = ymode == 1 ? r / rows_per_sample : r;
    load8v(y + yr * C + c, yplane, split != 0, w);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float v;
      switch (op) {
        case 0: v = u[t] + w[t]; break;
        case 1: v = u[t] - w[t]; break;
        case 2: v = u[t] * w[t]; break;
        case 3: v = u[t] / w[t]; break;
        case 4: v = fmaxf(u[t], w[t]); break;
        case 5: v = fminf(u[t], w[t]); break;
        case 6: v = u[t] > w[t] ? 1.f : 0.f; break;
        case 7: v = u[t] < w[t] ? 1.f : 0.f; break;
        case 8: v = u[t] == w[t] ? 1.f : 0.f; break;
        case 9: v = u[t] >= w[t] ? 1.f : 0.f; break;
        default: v = u[t] <= w[t] ? 1.f : 0.f; break;
      }
      u[t] = c + t < Cl ? apply_act(v, act, a, b) : 0.f;  // pad columns stay 0 (finite)
    }
    store8v(out + r * C + c, plane, split != 0, u);
  }
}

// y[r][c] = act(x[r][c] * scale[c] + shift[c]) with any activation code (affine_act handles the
// common 0/1/3; this one the rest: GELU, sigmoid, tanh, leaky ReLU).
__global__ void unary_kernel(const uint16_t* __restrict__ x, const float* __restrict__ scale,
                             const float* __restrict__ shift, uint16_t* __restrict__ y, long long R, int C, int act,
                             float a, float b, long long rows_per_sample, const long long* __restrict__ live,
                             int split, int Cl) {
  const long long plane = R * C;
  long long Rl = R;
  if (live) Rl = min(R, *live * rows_per_sample);
  const int G = C / 8;
  const long long total = Rl * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / G;
    const int c = static_cast<int>(i - r * G) * 8;
    float v[8];
    load8v(x + r * C + c, plane, split != 0, v);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float s = scale ? scale[c + t] : 1.f, h = scale ? shift[c + t] : 0.f;
      v[t] = c + t < Cl ? apply_act(v[t] * s + h, act, a, b) : 0.f;  // pad columns stay 0 (1/0, log 0)
    }
    store8v(y + r * C + c, plane, split != 0, v);
  }
}

// out = cond != 0 ? a : b over rows [R][C]; a / b null: the scalar av / bv.  Where (bool as 0 / 1).
__global__ void where_kernel(const uint16_t* __restrict__ c, const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                             float av, float bv, uint16_t* __restrict__ out, long long R, int C, long long plane,
                             long long rows_per_sample, const long long* __restrict__ live, int split, int Cl) {
  long long Rl = R;
  if (live) Rl = min(R, *live * rows_per_sample);
  const int G = C / 8;
  const long long total = Rl * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / G;
    const int col = static_cast<int>(i - r * G) * 8;
    float cv[8], x[8], z[8];
    load8v(c + r * C + col, plane, split != 0, cv);
    if (a) load8v(a + r * C + col, plane, split != 0, x);
    if (b) load8v(b + r * C + col, plane, split != 0, z);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float p = a ? x[t] : av, q = b ? z[t] : bv;
      cv[t] = col + t < Cl ? (cv[t] != 0.f ? p : q) : 0.f;
    }
    store8v(out + r * C + col, plane, split != 0, cv);
  }
}

// ONNX Resize / Upsample of an NHWC image (4-D, N and C scales 1).  coord: 0 half_pixel,
// 1 asymmetric, 2 align_corners, 3 pytorch_half_pixel, 4 tf_half_pixel_for_nn; mode 0 nearest
// (nearest: 0 round_prefer_floor, 1 round_prefer_ceil, 2 floor, 3 ceil; a bit copy of the source
// pixel), 1 linear (bilinear, neighbour indices clamped to the image = the spec's edge padding).
__device__ __forceinline__ float resize_src(int o, float scale, int in, int out, int coord) {
  switch (coord) {
    case 1: return o / scale;
    case 2: return out > 1 ? o * static_cast<float>(in - 1) / static_cast<float>(out - 1) : 0.f;
    case 3: return out > 1 ? (o + 0.5f) / scale - 0.5f : 0.f;
    case 4: return (o + 0.5f) / scale;
    default: return (o + 0.5f) / scale - 0.5f;
  }
}

__device__ __forceinline__ int resize_nearest(float s, int nearest, int in) {
  const float f = floorf(s);
  int i;
  switch (nearest) {
    case 1: i = s - f == 0.5f ? static_cast<int>(f) + 1 : static_cast<int>(rintf(s)); break;
    case 2: i = static_cast<int>(f); break;
    case 3: i = static_cast<int>(ceilf(s)); break;
    default: i = s - f == 0.5f ? static_cast<int>(f) : static_cast<int>(rintf(s)); break;
  }
  return min(max(i, 0), in - 1);
}

__global__ void resize_nhwc_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B, int H, int W, int C,
                                   int Ho, int Wo, float sh, float sw, int coord, int mode, int nearest,
                                   long long xplane, long long yplane, const long long* __restrict__ live, int split) {
  if (live) B = min(B, static_cast<int>(*live));
  const int G = C / 8;
  const long long total = static_cast<long long>(B) * Ho * Wo * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int cg = static_cast<int>(i % G);
    long long r = i / G;
    const int w = static_cast<int>(r % Wo);
    r /= Wo;
    const int h = static_cast<int>(r % Ho);
    const long long b = r / Ho;
    const float fy = resize_src(h, sh, H, Ho, coord), fx = resize_src(w, sw, W, Wo, coord);
    uint16_t* d = y + ((b * Ho + h) * Wo + w) * C + cg * 8;
    const uint16_t* xb = x + b * H * W * C + cg * 8;
    if (mode == 0) {
      const uint16_t* s = xb + (static_cast<long long>(resize_nearest(fy, nearest, H)) * W + resize_nearest(fx, nearest, W)) * C;
      *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
      if (split) *reinterpret_cast<uint4*>(d + yplane) = *reinterpret_cast<const uint4*>(s + xplane);
      continue;
    }
    const float y0f = floorf(fy), x0f = floorf(fx);
    const float ay = fy - y0f, ax = fx - x0f;
    const int y0 = min(max(static_cast<int>(y0f), 0), H - 1), y1 = min(max(static_cast<int>(y0f) + 1, 0), H - 1);
    const int x0 = min(max(static_cast<int>(x0f), 0), W - 1), x1 = min(max(static_cast<int>(x0f) + 1, 0), W - 1);
    float p00[8], p01[8], p10[8], p11[8], v[8];
    load8v(xb + (static_cast<long long>(y0) * W + x0) * C, xplane, split != 0, p00);
    load8v(xb + (static_cast<long long>(y0) * W + x1) * C, xplane, split != 0, p01);
    load8v(xb + (static_cast<long long>(y1) * W + x0) * C, xplane, split != 0, p10);
    load8v(xb + (static_cast<long long>(y1) * W + x1) * C, xplane, split != 0, p11);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float top = p00[t] * (1.f - ax) + p01[t] * ax, bot = p10[t] * (1.f - ax) + p11[t] * ax;
      v[t] = top * (1.f - ay) + bot * ay;
    }
    store8v(d, yplane, split != 0, v);
  }
}

// Zero padding of an NHWC image: y [B][Ho][Wo][C] holds x [B][H][W][C] at offset (t, l), zeros
// around it (ONNX Pad, constant mode, value 0, spatial axes only).  Strides sy, sx > 1 also insert
// sy - 1 / sx - 1 zero rows / columns between the input's (ConvTranspose as a stride-1 conv).
__global__ void pad_nhwc_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B, int H, int W, int C,
                                int Ho, int Wo, int t, int l, long long xplane, long long yplane, int split, int sy,
                                int sx) {
  const int G = C / 8;
  const long long total = static_cast<long long>(B) * Ho * Wo * G;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int cg = static_cast<int>(i % G);
    long long r = i / G;
    const int w = static_cast<int>(r % Wo);
    r /= Wo;
    const int h = static_cast<int>(r % Ho);
    const long long b = r / Ho;
    const int dh = h - t, dw = w - l;
    const int sh = dh / sy, sw = dw / sx;
    uint16_t* d = y + ((b * Ho + h) * Wo + w) * C + cg * 8;
    uint4 hi = make_uint4(0, 0, 0, 0), lo = hi;
    if (dh >= 0 && dw >= 0 && dh == sh * sy && dw == sw * sx && sh < H && sw < W) {
      const uint16_t* s = x + ((b * H + sh) * W + sw) * C + cg * 8;
      hi = *reinterpret_cast<const uint4*>(s);
      if (split) lo = *reinterpret_cast<const uint4*>(s + xplane);
    }
    *reinterpret_cast<uint4*>(d) = hi;
    if (split) *reinterpret_cast<uint4*>(d + yplane) = lo;
  }
}

// f32 y[r][0..C) = x[r][0..C) of bf16 / split rows with pitch ld (drops stored pad columns).
__global__ void rows_to_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, long long R, int C, int ld,
                                   long long plane, int split) {
  const long long total = R * C;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = i / C;
    const int c = static_cast<int>(i - r * C);
    y[i] = load1v(x + r * ld + c, plane, split != 0);
  }
}

// fp32 NCHW graph output [B][C][HW] from bf16 NHWC with pitch Cs >= C (drops pad channels).
__global__ void nhwc_to_nchw_strided_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int B, int HW, int C,
                                            int Cs, long long plane, int split) {
  const long long total = static_cast<long long>(B) * HW * C;
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long p = i % HW;
    long long r = i / HW;
    const long long c = r % C;
    const long long b = r / C;
    y[i] = load1v(x + (b * HW + p) * Cs + c, plane, split != 0);
  }
}

}  // namespace

hipError_t pad_nhwc(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, int t, int l,
                    hipStream_t s, int split, int sy, int sx) {
  if (C % 8 || t < 0 || l < 0 || sy < 1 || sx < 1 || Ho < (H - 1) * sy + 1 + t || Wo < (W - 1) * sx + 1 + l)
    return hipErrorInvalidValue;
  const long long work = static_cast<long long>(B) * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(pad_nhwc_kernel, dim3(grid_for(work)), dim3(256), 0, s, x, y, B, H, W, C, Ho, Wo, t, l,
                     static_cast<long long>(B) * H * W * C, static_cast<long long>(B) * Ho * Wo * C, split, sy, sx);
  return hipGetLastError();
}

hipError_t where_rows(const uint16_t* c, const uint16_t* a, const uint16_t* b, float av, float bv, uint16_t* out,
                      long long R, int C, hipStream_t s, const long long* live, long long rows_per_sample, int split,
                      int Cl) {
  if (C % 8 || rows_per_sample <= 0 || Cl < 0 || Cl > C) return hipErrorInvalidValue;
  hipLaunchKernelGGL(where_kernel, dim3(grid_for(R * (C / 8))), dim3(256), 0, s, c, a, b, av, bv, out, R, C, R * C,
                     rows_per_sample, live, split, Cl ? Cl : C);
  return hipGetLastError();
}

hipError_t resize_nhwc(const uint16_t* x, uint16_t* y, int B, int H, int W, int C, int Ho, int Wo, float scale_h,
                       float scale_w, int coord, int mode, int nearest, hipStream_t s, const long long* live, int split) {
  if (C % 8 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || !(scale_h > 0.f) || !(scale_w > 0.f) || coord < 0 || coord > 4 ||
      mode < 0 || mode > 1 || nearest < 0 || nearest > 3)
    return hipErrorInvalidValue;
  const long long work = static_cast<long long>(B) * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(resize_nhwc_kernel, dim3(grid_for(work)), dim3(256), 0, s, x, y, B, H, W, C, Ho, Wo, scale_h,
                     scale_w, coord, mode, nearest, static_cast<long long>(B) * H * W * C,
                     static_cast<long long>(B) * Ho * Wo * C, live, split);
  return hipGetLastError();
}

hipError_t rows_prep(const float* x, uint16_t* y, long long R, int F, int Fp, hipStream_t s, int split) {
  if (Fp % 8 || Fp < F || F <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_prep_kernel, dim3(grid_for(R * (Fp / 8))), dim3(256), 0, s, x, y, R, F, Fp, split);
  return hipGetLastError();
}

hipError_t input_prep_wide(const float* x, const float* scale, const float* shift, uint16_t* out, int B, int C, int H,
                           int W, int Cp, hipStream_t s, int split) {
  if (Cp % 8 || Cp < C) return hipErrorInvalidValue;
  const long long work = static_cast<long long>(B) * H * W * (Cp / 8);
  hipLaunchKernelGGL(input_prep_wide_kernel, dim3(grid_for(work)), dim3(256), 0, s, x, scale, shift, out, B, C, H * W,
                     Cp, split);
  return hipGetLastError();
}

hipError_t copy_cols(const uint16_t* x, long long xplane, int ldx, int colx, uint16_t* y, long long yplane, int ldy,
                     int coly, long long R, int ncols, hipStream_t s, int split) {
  if (ncols % 8 || ldx % 8 || ldy % 8 || colx % 8 || coly % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy_cols_kernel, dim3(grid_for(R * (ncols / 8))), dim3(256), 0, s, x, xplane, ldx, colx, y,
                     yplane, ldy, coly, R, ncols, split);
  return hipGetLastError();
}

hipError_t binary_rows(const uint16_t* x, const uint16_t* y, uint16_t* out, long long R, int C, long long rows_per_sample,
                       int ymode, int op, int act, float a, float b, hipStream_t s, const long long* live, int split,
                       int Cl) {
  if (C % 8 || rows_per_sample <= 0 || op < 0 || op > 10 || Cl < 0 || Cl > C) return hipErrorInvalidValue;
  if (Cl == 0) Cl = C;
  const long long plane = R * C;
  const long long yplane = ymode == 1 ? (R / rows_per_sample) * C : plane;
  hipLaunchKernelGGL(binary_kernel, dim3(grid_for(R * (C / 8))), dim3(256), 0, s, x, y, out, R, C, rows_per_sample,
                     ymode, op, act, a, b, plane, yplane, live, split, Cl);
  return hipGetLastError();
}

hipError_t unary_rows(const uint16_t* x, const float* scale, const float* shift, uint16_t* y, long long R, int C,
                      int act, float a, float b, hipStream_t s, const long long* live, long long rows_per_sample,
                      int split, int Cl) {
  if (C % 8 || (live && rows_per_sample <= 0) || Cl < 0 || Cl > C || act < 0 || act > 24) return hipErrorInvalidValue;
  hipLaunchKernelGGL(unary_kernel, dim3(grid_for(R * (C / 8))), dim3(256), 0, s, x, scale, shift, y, R, C, act, a, b,
                     rows_per_sample, live, split, Cl ? Cl : C);
  return hipGetLastError();
}

hipError_t rows_to_f32(const uint16_t* x, float* y, long long R, int C, int ld, hipStream_t s, int split) {
  if (C > ld) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_to_f32_kernel, dim3(grid_for(R * C)), dim3(256), 0, s, x, y, R, C, ld, R * ld, split);
  return hipGetLastError();
}

hipError_t nhwc_to_nchw_f32_strided(const uint16_t* x, float* y, int B, int H, int W, int C, int Cs, hipStream_t s,
                                    int split) {
  if (C > Cs) return hipErrorInvalidValue;
  const long long plane = static_cast<long long>(B) * H * W * Cs;
  hipLaunchKernelGGL(nhwc_to_nchw_strided_kernel, dim3(grid_for(static_cast<long long>(B) * H * W * C)), dim3(256), 0,
                     s, x, y, B, H * W, C, Cs, plane, split);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
