// Transformer (ViT) kernels for gfx950: LayerNorm over rows, token assembly (cls + patches +
// position embedding), row gather, and fused multi-head attention on MFMA.
//
// These replace what ONNX Runtime would run for a ViT-B/16 export (LayerNormalization, the
// MatMul -> Div -> Softmax -> MatMul attention chain with its Reshape/Transpose views, Concat/Add
// of the embeddings, Gather of the cls token).  Layouts: activations are bf16 rows [B*S, C] with the
// head h occupying columns [h*D, (h+1)*D) (no transposes are ever materialised).
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

using namespace die::k;

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One wave per row; each lane holds up to CPL 8-element chunks of the row in registers
// (two-pass mean/variance in fp32).  C % 8 == 0, C <= 64*8*CPL.
template <int CPL>
__global__ __launch_bounds__(256) void layernorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        float eps, long long rows, int C) {
  const int lane = threadIdx.x & 63;
  const long long row = static_cast<long long>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = C / 8;
  const uint16_t* xr = x + row * C;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      const uint4 q = *reinterpret_cast<const uint4*>(xr + c * 8);
      unpack2(q.x, v[i][0], v[i][1]);
      unpack2(q.y, v[i][2], v[i][3]);
      unpack2(q.z, v[i][4], v[i][5]);
      unpack2(q.w, v[i][6], v[i][7]);
#pragma unroll
      for (int t = 0; t < 8; ++t) s += v[i][t];
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[i][t] = 0.f;
    }
  }
  const float mean = wave_sum(s) / C;
  float q2 = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
    if (lane + 64 * i < nch) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float d = v[i][t] - mean;
        q2 += d * d;
      }
    }
  const float inv = rsqrtf(wave_sum(q2) / C + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= nch) continue;
    float o[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] = (v[i][t] - mean) * inv * g[c * 8 + t] + b[c * 8 + t];
    *reinterpret_cast<uint4*>(y + row * C + c * 8) =
        make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
  }
}

// out[b, 0, :] = cls + pos[0];  out[b, 1 + s, :] = patches[b, s, :] + pos[1 + s]
__global__ void tokens_kernel(const uint16_t* __restrict__ patches, const float* __restrict__ cls,
                              const float* __restrict__ pos, uint16_t* __restrict__ out, int B, int S0, int C) {
  const int S = S0 + 1;
  const int CG = C / 8;
  const long long total = static_cast<long long>(B) * S * CG;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int cg = static_cast<int>(i % CG);
    const long long r = i / CG;
    const int s = static_cast<int>(r % S);
    const long long b = r / S;
    float v[8];
    if (s == 0) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = cls ? cls[cg * 8 + t] : 0.f;
    } else {
      const uint4 q = *reinterpret_cast<const uint4*>(patches + ((b * S0 + s - 1) * C + cg * 8));
      unpack2(q.x, v[0], v[1]);
      unpack2(q.y, v[2], v[3]);
      unpack2(q.z, v[4], v[5]);
      unpack2(q.w, v[6], v[7]);
    }
    if (pos) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] += pos[static_cast<long long>(s) * C + cg * 8 + t];
    }
    *reinterpret_cast<uint4*>(out + i * 8) =
        make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
  }
}

__global__ void gather_rows_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int B, int S, int idx,
                                   int C) {
  const int CG = C / 8;
  const long long total = static_cast<long long>(B) * CG;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const long long b = i / CG;
    const int cg = static_cast<int>(i % CG);
    *reinterpret_cast<uint4*>(y + i * 8) =
        *reinterpret_cast<const uint4*>(x + ((b * S + idx) * C + cg * 8));
  }
}

// ---- fused attention ------------------------------------------------------------------------------
// One block = (64 query rows, head h, image b); 4 waves x 16 query rows.  K [S][64] (XOR-swizzled
// 128-B rows), V^T [64][SK+8] and each wave's P [16][SK+8] live in LDS.  QK^T and PV run on
// v_mfma_f32_16x16x32_bf16; softmax in fp32 registers (a row's 16 key columns of a 16x16 tile are
// spread over 16 lanes: max/sum reduce with xor-shuffles 1,2,4,8).
constexpr int AT_D = 64;

template <int SK>
__global__ __launch_bounds__(256) void attention_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                        const uint16_t* __restrict__ v, uint16_t* __restrict__ out,
                                                        int S, int ldq, int ldk, int ldv, int ldo, float scale) {
  constexpr int NT = SK / 16;   // key tiles
  constexpr int NKS = SK / 32;  // PV k-steps
  constexpr int VP = SK + 8;    // padded pitch (conflict-free transposed reads)
  __shared__ __attribute__((aligned(16))) uint16_t lds[SK * AT_D + AT_D * VP + 64 * VP];
  uint16_t* Ks = lds;
  uint16_t* Vt = lds + SK * AT_D;
  uint16_t* P = Vt + AT_D * VP;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long rowbase = static_cast<long long>(b) * S;
  // K -> LDS (swizzled chunks), V -> LDS transposed; rows >= S are zero.
  for (int i = tid; i < SK * 8; i += 256) {
    const int s = i >> 3, c = i & 7;
    uint4 kq = make_uint4(0, 0, 0, 0), vq = make_uint4(0, 0, 0, 0);
    if (s < S) {
      kq = *reinterpret_cast<const uint4*>(k + (rowbase + s) * ldk + h * AT_D + c * 8);
      vq = *reinterpret_cast<const uint4*>(v + (rowbase + s) * ldv + h * AT_D + c * 8);
    }
    *reinterpret_cast<uint4*>(Ks + s * AT_D + ((c ^ ((s >> 1) & 7)) << 3)) = kq;
    const uint32_t w[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      Vt[(c * 8 + 2 * t) * VP + s] = static_cast<uint16_t>(w[t] & 0xFFFF);
      Vt[(c * 8 + 2 * t + 1) * VP + s] = static_cast<uint16_t>(w[t] >> 16);
    }
  }
  __syncthreads();

  const int q0 = blockIdx.x * 64 + wave * 16;
  if (q0 >= S) return;  // whole wave past the end (after the only block barrier)
  // Q fragments (A operand): lane -> row q0 + (lane & 15), k-chunk (lane >> 4) + 4*kk
  bf16x8 qf[2];
  {
    const int qr = q0 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 t = make_uint4(0, 0, 0, 0);
      if (qr < S) t = *reinterpret_cast<const uint4*>(q + (rowbase + qr) * ldq + h * AT_D + ((lane >> 4) + 4 * kk) * 8);
      qf[kk] = __builtin_bit_cast(bf16x8, t);
    }
  }
  f32x4 sc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int key = t * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = (lane >> 4) + 4 * kk;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + key * AT_D + ((c ^ ((key >> 1) & 7)) << 3));
      sc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[kk], kf, sc[t], 0, 0, 0);
    }
  }
  // softmax over keys for the 4 rows this lane holds (rows 4*(lane>>4)+r, key column lane&15)
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const bool valid = t * 16 + (lane & 15) < S;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = valid ? sc[t][r] * scale : -INFINITY;
      sc[t][r] = x;
      mx[r] = fmaxf(mx[r], x);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
  float sm[4] = {0.f, 0.f, 0.f, 0.f};
  uint16_t* Pw = P + wave * 16 * VP;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(sc[t][r] - mx[r]);
      sm[r] += e;
      Pw[(4 * (lane >> 4) + r) * VP + t * 16 + (lane & 15)] = f2bf(e);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) sm[r] += __shfl_xor(sm[r], o, 64);
  // zero P columns [NT*16, SK) never exist (SK multiple of 16); P rows are written by this wave only
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own LDS writes land before the reads below
  // O = P V : A = P [16 q x 32 keys], B = V [32 keys x 16 d]
  f32x4 o[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const bf16x8 pf = *reinterpret_cast<const bf16x8*>(Pw + (lane & 15) * VP + ks * 32 + (lane >> 4) * 8);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vt + (n * 16 + (lane & 15)) * VP + ks * 32 + (lane >> 4) * 8);
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[n], 0, 0, 0);
    }
  }
  // normalise and store: lane holds rows 4*(lane>>4)+r, columns n*16 + (lane&15)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 4 * (lane >> 4) + r;
    if (qr >= S) continue;
    const float inv = 1.f / sm[r];
    uint16_t* orow = out + (rowbase + qr) * ldo + h * AT_D;
#pragma unroll
    for (int n = 0; n < 4; ++n) orow[n * 16 + (lane & 15)] = f2bf(o[n][r] * inv);
  }
}

inline int grid_for(long long work, int cap = 4096) {
  long long g = (work + 255) / 256;
  if (g < 1) g = 1;
  return static_cast<int>(g > cap ? cap : g);
}

}  // namespace

hipError_t layernorm_rows(const uint16_t* x, uint16_t* y, const float* gamma, const float* beta, float eps,
                          long long rows, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int blocks = static_cast<int>((rows + 3) / 4);
  if (C <= 64 * 8) hipLaunchKernelGGL(layernorm_kernel<1>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C);
  else if (C <= 128 * 8) hipLaunchKernelGGL(layernorm_kernel<2>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C);
  else if (C <= 256 * 8) hipLaunchKernelGGL(layernorm_kernel<4>, dim3(blocks), dim3(256), 0, s, x, y, gamma, beta, eps, rows, C);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t tokens_assemble(const uint16_t* patches, const float* cls, const float* pos, uint16_t* out, int B, int S0,
                           int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tokens_kernel, dim3(grid_for(static_cast<long long>(B) * (S0 + 1) * (C / 8))), dim3(256), 0, s,
                     patches, cls, pos, out, B, S0, C);
  return hipGetLastError();
}

hipError_t gather_rows(const uint16_t* x, uint16_t* y, int B, int S, int idx, int C, hipStream_t s) {
  if (C % 8 || idx < 0 || idx >= S) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(static_cast<long long>(B) * (C / 8))), dim3(256), 0, s, x, y, B,
                     S, idx, C);
  return hipGetLastError();
}

hipError_t attention(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* out, int B, int S, int H,
                     int D, int ldq, int ldk, int ldv, int ldo, float scale, hipStream_t s) {
  if (D != AT_D || S <= 0 || S > 256 || ldq % 8 || ldk % 8 || ldv % 8) return hipErrorInvalidValue;
  dim3 grid((S + 63) / 64, H, B);
  if (S <= 64) hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(256), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, scale);
  else if (S <= 128) hipLaunchKernelGGL(attention_kernel<128>, grid, dim3(256), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, scale);
  else if (S <= 224) hipLaunchKernelGGL(attention_kernel<224>, grid, dim3(256), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, scale);
  else hipLaunchKernelGGL(attention_kernel<256>, grid, dim3(256), 0, s, q, k, v, out, S, ldq, ldk, ldv, ldo, scale);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
