// Device-side helpers shared by the CDNA4 (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace die {
namespace k {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

// float -> bf16, round to nearest even (gfx950 lowers this to v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return static_cast<uint32_t>(f2bf(a)) | (static_cast<uint32_t>(f2bf(b)) << 16);
}

__device__ __forceinline__ void unpack2(uint32_t v, float& a, float& b) {
  a = __uint_as_float(v << 16);
  b = __uint_as_float(v & 0xFFFF0000u);
}

}  // namespace k
}  // namespace die
