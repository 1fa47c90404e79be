// Grouped / depthwise convolution for gfx950 (NHWC), e.g. MobileNet's 3x3 depthwise convs
// (ONNX Conv with group > 1; the reference runs any such model through ORT,
// /root/reference/src/inference_engine.cpp:31-69).
//
// A depthwise layer has K = kh*kw per output channel: nothing for the matrix cores to chew on, the
// layer is a stream over the activation.  One thread owns 8 consecutive output channels of one
// pixel and walks the filter taps: for depthwise (one input channel per group, channel multiplier
// 1) each tap is one 16-byte load of the 8 matching input channels (two for split fp32 tensors),
// otherwise the group's input channels are read one by one.  Weights are fp32 [Cout][kh][kw][cpg]
// (BatchNormalization folded), so fp32 mode loses nothing; the epilogue adds the bias, applies
// ReLU / Clip and an optional residual, and stores bf16 or split planes.
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

__device__ __forceinline__ float act_apply(float v, int act, float lo, float hi) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 3) return fminf(fmaxf(v, lo), hi);
  return v;
}

template <bool DW>
__global__ __launch_bounds__(256) void gconv_kernel(const GConvArgs a) {
  const int CG = a.Cout / 8;
  long long total = static_cast<long long>(a.B) * a.Ho * a.Wo * CG;
  if (a.live) total = min(total, *a.live * static_cast<long long>(a.Ho) * a.Wo * CG);
  const long long xplane = static_cast<long long>(a.B) * a.H * a.W * a.Cin;
  const long long oplane = static_cast<long long>(a.B) * a.Ho * a.Wo * a.Cout;
  const bool split = a.split != 0;
  const int cpg = a.Cin / a.groups, opg = a.Cout / a.groups;
  const int KT = a.KH * a.KW * cpg;  // weights per output channel
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int cg = static_cast<int>(i % CG);
    long long r = i / CG;
    const int ow = static_cast<int>(r % a.Wo);
    r /= a.Wo;
    const int oh = static_cast<int>(r % a.Ho);
    const int b = static_cast<int>(r / a.Ho);
    const int co = cg * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint16_t* xb = a.x + static_cast<long long>(b) * a.H * a.W * a.Cin;
    for (int ky = 0; ky < a.KH; ++ky) {
      const int ih = oh * a.stride - a.pad_h + ky * a.dil;
      if (ih < 0 || ih >= a.H) continue;
      for (int kx = 0; kx < a.KW; ++kx) {
        const int iw = ow * a.stride - a.pad_w + kx * a.dil;
        if (iw < 0 || iw >= a.W) continue;
        const uint16_t* px = xb + (static_cast<long long>(ih) * a.W + iw) * a.Cin;
        const int tap = ky * a.KW + kx;
        if constexpr (DW) {  // cpg == 1, opg == 1: output channel c reads input channel c
          float v[8];
          load8v(px + co, xplane, split, v);
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] += v[t] * a.w[static_cast<long long>(co + t) * KT + tap];
        } else {
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int c = co + t, g = c / opg;
            const float* wc = a.w + static_cast<long long>(c) * KT + tap * cpg;
            const uint16_t* xg = px + g * cpg;
            float s = 0.f;
            for (int ci = 0; ci < cpg; ++ci) s += load1v(xg + ci, xplane, split) * wc[ci];
            acc[t] += s;
          }
        }
      }
    }
    const long long o = ((static_cast<long long>(b) * a.Ho + oh) * a.Wo + ow) * a.Cout + co;
    float res[8];
    if (a.res) load8v(a.res + o, oplane, split, res);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float v = acc[t] + (a.bias ? a.bias[co + t] : 0.f);
      v = act_apply(v, a.act, a.clip_lo, a.clip_hi);
      if (a.res) v += res[t];
      acc[t] = v;
    }
    if (a.out) store8v(a.out + o, oplane, split, acc);
    if (a.out_f32) {
#pragma unroll
      for (int t = 0; t < 8; ++t) a.out_f32[o + t] = acc[t];
    }
  }
}

}  // namespace

hipError_t grouped_conv(const GConvArgs& a, hipStream_t s) {
  if (a.groups < 1 || a.Cin % a.groups || a.Cout % a.groups || a.Cout % 8 || !a.w || !a.x || (!a.out && !a.out_f32))
    return hipErrorInvalidValue;
  const long long work = static_cast<long long>(a.B) * a.Ho * a.Wo * (a.Cout / 8);
  long long g = (work + 255) / 256;
  g = g < 1 ? 1 : (g > 8192 ? 8192 : g);
  const bool dw = a.groups == a.Cin && a.groups == a.Cout;
  if (dw) hipLaunchKernelGGL(gconv_kernel<true>, dim3(static_cast<int>(g)), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(gconv_kernel<false>, dim3(static_cast<int>(g)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
