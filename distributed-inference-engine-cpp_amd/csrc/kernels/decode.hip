// Device-side decode of JSON number lists (the text between '[' and ']' of "input_data").
//
// The serving headline is bound by host CPU, and ~80% of a worker's CPU time went into converting
// ~150k decimal strings per ResNet request.  MI355X has bandwidth to spare, so the worker copies the
// raw text into pinned staging and the GPU converts it (inside the same hipGraph as the forward):
//   (samples uploaded 4-bit packed are expanded to characters in registers as each kernel loads them)
//   1. dec_count : per 4 KiB chunk, count ',' separators and note non-blank bytes
//   2. dec_parse : a chunk is staged in LDS (+ halo); its token index is the sum of the earlier
//                  chunks' counts; token starts are found per 16 bytes and compacted with a block
//                  scan; each lane then converts whole tokens from registers and stores them at
//                  out[sample][token index].  The block holding a sample's last chunk writes its
//                  token count, the "too many values" status and the zero-fill of the padded tail.
// Both kernels run a fixed grid (hipGraph-capturable) that strides over the LIVE chunks only: the
// chunk table is sized for the largest accepted body (24 B per value), ~3.5x a typical request, and
// a grid over the whole table spent most of its blocks on empty chunks.
// Conversion is bit-identical to the host parser: integers up to 2^24 scaled by an exact power of
// ten in fp32 (one rounding), otherwise an exact-power double product/quotient checked for the
// double-rounding hazard.  Anything unusual (exponent overflow, > 19 significant digits, subnormal,
// malformed token, token > 64 bytes) sets status bit 1 and the worker re-parses that request on
// the host with the strict parser, so accepted inputs and error messages match the host path.
#include "common.h"
#include "kernels.h"

namespace die {
namespace kern {

namespace {

constexpr int CHUNK = 4096;  // bytes per block: 256 threads x 16 B
constexpr int HALO = 64;     // max token length converted on the device
constexpr int PRE = 16;

__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {  // 0x80 in each byte of v that is zero
  const uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t eq_bytes(uint32_t v, uint32_t c4) { return zero_bytes(v ^ c4); }
__device__ __forceinline__ bool is_ws(unsigned c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

// bytes of q at or beyond len (q holds [off, off+16)) replaced by ' '
__device__ __forceinline__ uint4 blank_tail(uint4 q, long long off, long long len) {
  if (off + 16 > len) {
    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (off + i >= len) w[i >> 2] = (w[i >> 2] & ~(0xFFu << (8 * (i & 3)))) | (0x20u << (8 * (i & 3)));
    q = make_uint4(w[0], w[1], w[2], w[3]);
  }
  return q;
}

// 4 characters from 2 packed bytes (core/textpack.h: low nibble first).  Symbols 0-7 map through
// one v_perm_b32 table ('0'..'7'), 8-15 through another ('8' '9' ',' '.' '-' '+' 'e' ' '); bit 3 of
// each nibble picks the table.
__device__ __forceinline__ uint32_t nib4(uint32_t p16) {
  const uint32_t t = (p16 & 0xFFu) | ((p16 & 0xFF00u) << 8);
  const uint32_t x = (t & 0x000F000Fu) | ((t & 0x00F000F0u) << 4);  // one nibble per byte
  const uint32_t sel = x & 0x07070707u;
  const uint32_t m = ((x >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t lo = __builtin_amdgcn_perm(0x37363534u, 0x33323130u, sel);
  const uint32_t hi = __builtin_amdgcn_perm(0x20652B2Du, 0x2E2C3938u, sel);
  return (hi & m) | (lo & ~m);
}

// 16 bytes at [off, off+16) of a sample's text (off % 16 == 0), bytes >= len replaced by ' '.  A
// sample uploaded 4-bit packed (pk != nullptr) is expanded from its 8 packed bytes in registers, so
// the character text is never materialised in HBM.  The packed slot is text_cap / 2 bytes and
// off + 16 <= text_cap, so the 8-byte read stays inside it.
__device__ __forceinline__ uint4 load16(const unsigned char* t, const unsigned char* pk, long long off, long long len) {
  uint4 q;
  if (pk) {
    const uint2 p = *reinterpret_cast<const uint2*>(pk + (off >> 1));
    q = make_uint4(nib4(p.x & 0xFFFFu), nib4(p.x >> 16), nib4(p.y & 0xFFFFu), nib4(p.y >> 16));
  } else {
    q = *reinterpret_cast<const uint4*>(t + off);
  }
  return blank_tail(q, off, len);
}

__device__ __forceinline__ int popc_commas(uint4 q) {
  const uint32_t C = 0x2C2C2C2Cu;
  return __popc(eq_bytes(q.x, C)) + __popc(eq_bytes(q.y, C)) + __popc(eq_bytes(q.z, C)) + __popc(eq_bytes(q.w, C));
}

__device__ __forceinline__ bool nonblank(uint4 q) {
  uint32_t w[4] = {q.x, q.y, q.z, q.w};
  bool any = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t ws = eq_bytes(w[i], 0x20202020u) | eq_bytes(w[i], 0x0A0A0A0Au) | eq_bytes(w[i], 0x0D0D0D0Du) |
                        eq_bytes(w[i], 0x09090909u);
    any |= ws != 0x80808080u;
  }
  return any;
}

// true when none of the 16 bytes is ' ', '\n', '\r' or '\t'
__device__ __forceinline__ bool nonblank_all(uint4 q) {
  uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    any |= eq_bytes(w[i], 0x20202020u) | eq_bytes(w[i], 0x0A0A0A0Au) | eq_bytes(w[i], 0x0D0D0D0Du) |
           eq_bytes(w[i], 0x09090909u);
  return any == 0;
}

// exclusive block scan of one int per thread (256 threads)
__device__ __forceinline__ int block_excl_scan(int v, int* red, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) red[w] = x;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += red[i];
  total = red[0] + red[1] + red[2] + red[3];
  return base + x - v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// exclusive scan over the 64 lanes of this wave; total = the wave's sum
__device__ __forceinline__ int wave_excl_scan(int v, int& total) {
  const int lane = threadIdx.x & 63;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  total = __shfl(x, 63, 64);
  return x - v;
}

// This wave's LDS writes are complete and visible to its other lanes (and not reordered by the
// compiler); LDS traffic of one wave needs no workgroup barrier.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

constexpr int kDecMaxB = 1024;  // samples per launch (LDS chunk-prefix table)
constexpr int kDecGrid = 2048;  // blocks (4 waves = 4 work items each) of the grid-stride kernels

// Per block: pre[b] = exclusive prefix over samples of their chunk counts (a sample with text has
// max(1, ceil(len / CHUNK)) chunks -- an empty body still gets one work item; a skipped sample
// none).  Returns the number of work items.
__device__ int chunk_prefix(const long long* __restrict__ lens, int B, int* pre, int* red) {
  int carry = 0;
  for (int i0 = 0; i0 < B; i0 += 256) {
    const int i = i0 + threadIdx.x;
    int v = 0;
    if (i < B) {
      const long long len = lens[i];
      v = len < 0 ? 0 : len == 0 ? 1 : static_cast<int>((len + CHUNK - 1) / CHUNK);
    }
    int tot;
    const int ex = block_excl_scan(v, red, tot);
    if (i < B) pre[i] = carry + ex;
    carry += tot;
  }
  __syncthreads();
  return carry;
}

// work item -> sample: the last b with pre[b] <= item (samples without chunks share their
// successor's prefix and are skipped over)
__device__ __forceinline__ int item_sample(const int* pre, int B, int item) {
  int lo = 0, hi = B;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pre[mid] <= item) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One WAVE per 4 KiB chunk (no workgroup barriers in the loop): lane l counts the separators of
// 16-byte words l, l+64, l+128, l+192 (coalesced), the wave sums them.
__global__ __launch_bounds__(256) void dec_count(const unsigned char* __restrict__ text, long long cap,
                                                 const long long* __restrict__ offs,
                                                 const unsigned char* __restrict__ packed,
                                                 const long long* __restrict__ poffs,
                                                 const long long* __restrict__ lens, int B, int* __restrict__ counts,
                                                 int* __restrict__ blank, int* __restrict__ status,
                                                 int* __restrict__ ntok, int max_chunks) {
  __shared__ int red[4];
  __shared__ int pre[kDecMaxB];
  if (blockIdx.x == 0) {  // per-sample results start clean; dec_parse ORs its bits in
    for (int b = threadIdx.x; b < B; b += 256) {
      status[b] = 0;
      if (lens[b] < 0) ntok[b] = -1;
    }
  }
  const int items = chunk_prefix(lens, B, pre, red);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int it = blockIdx.x * 4 + wave; it < items; it += gridDim.x * 4) {
    const int b = item_sample(pre, B, it), chunk = it - pre[b];
    const long long len = lens[b];
    const long long c0 = static_cast<long long>(chunk) * CHUNK;
    const long long po = poffs ? poffs[b] : -1;
    const unsigned char* t = text + (offs ? offs[b] : b * cap);
    const unsigned char* pk = po >= 0 ? packed + po : nullptr;
    int c = 0, nb = 0;
#pragma unroll
    for (int k = 0; k < CHUNK / 16 / 64; ++k) {
      const long long off = c0 + 16ll * (k * 64 + lane);
      if (off < len) {
        const uint4 q = load16(t, pk, off, len);
        c += popc_commas(q);
        nb |= nonblank(q);
      }
    }
    c = wave_sum(c);
    nb = wave_sum(nb);
    if (lane == 0) {
      counts[b * max_chunks + chunk] = c;
      blank[b * max_chunks + chunk] = nb == 0;
    }
  }
}

__constant__ float kP10f[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
__constant__ double kP10d[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Convert the token s(0..n) (separators excluded).  Returns false -> host fallback.
template <class At>
__device__ bool convert_token(At s, int n, float& out) {  // s(i): byte i of the token
  int i = 0;
  while (i < n && is_ws(s(i))) ++i;
  while (n > i && is_ws(s(n - 1))) --n;
  if (i >= n) return false;
  const bool neg = s(i) == '-';
  i += neg;
  if (i >= n || s(i) - '0' > 9u) return false;
  uint64_t mant = 0;
  int nd = 0, exp10 = 0;
  if (s(i) == '0') {
    ++i;
    if (i < n && s(i) - '0' <= 9u) return false;  // leading zero
  } else {
    while (i < n && s(i) - '0' <= 9u) {
      if (nd >= 19) return false;
      mant = mant * 10 + (s(i) - '0');
      ++nd;
      ++i;
    }
  }
  if (i < n && s(i) == '.') {
    ++i;
    if (i >= n || s(i) - '0' > 9u) return false;
    while (i < n && s(i) - '0' <= 9u) {
      const unsigned d = s(i) - '0';
      if (mant != 0 || d != 0) {
        if (nd >= 19) return false;
        mant = mant * 10 + d;
        ++nd;
      }
      --exp10;
      ++i;
    }
  }
  if (i < n && (s(i) == 'e' || s(i) == 'E')) {
    ++i;
    int es = 1;
    if (i < n && (s(i) == '+' || s(i) == '-')) {
      es = s(i) == '-' ? -1 : 1;
      ++i;
    }
    if (i >= n || s(i) - '0' > 9u) return false;
    int e = 0;
    while (i < n && s(i) - '0' <= 9u) {
      e = e * 10 + (s(i) - '0');
      if (e > 10000) e = 10000;
      ++i;
    }
    exp10 += es * e;
  }
  if (i != n) return false;
  float v;
  if (mant == 0) {
    v = 0.f;
  } else if (mant <= (1u << 24) && exp10 >= -10 && exp10 <= 10) {
    v = exp10 < 0 ? static_cast<float>(mant) / kP10f[-exp10] : static_cast<float>(mant) * kP10f[exp10];
  } else if (exp10 >= -66 && exp10 <= 66) {
    // r <= 4 roundings in double (mantissa > 2^53, then up to three exact powers <= 1e22), so
    // |d - x| < r ulp(d).  The float rounding of d equals that of x unless d lies within r+1 ulp of
    // a float midpoint (low 29 mantissa bits near 0x10000000) -> host fallback in that case.
    double d = static_cast<double>(mant);
    int r = mant > (1ull << 53);
    for (int e = exp10; e != 0; ++r) {
      const int k = e > 0 ? (e > 22 ? 22 : e) : (e < -22 ? 22 : -e);
      d = e > 0 ? d * kP10d[k] : d / kP10d[k];
      e += e > 0 ? -k : k;
    }
    const uint64_t bits = __double_as_longlong(d);
    const long long low = static_cast<long long>(bits & ((1ull << 29) - 1)) - (1ll << 28);
    if (low >= -(r + 1) && low <= r + 1) return false;  // double-rounding hazard
    if (d > 3.4028234663852886e38 || d < 1.1754943508222875e-38) return false;  // overflow / subnormal
    v = static_cast<float>(d);
  } else {
    return false;
  }
  out = __uint_as_float(__float_as_uint(v) | (static_cast<uint32_t>(neg) << 31));
  return true;
}

// 4 bits (one per byte) from a 0x80-per-byte mask
__device__ __forceinline__ uint32_t mask4(uint32_t m) { return (((m >> 7) & 0x01010101u) * 0x01020408u) >> 24; }
__device__ __forceinline__ uint32_t mask16(uint4 q, uint32_t c4) {
  return mask4(eq_bytes(q.x, c4)) | (mask4(eq_bytes(q.y, c4)) << 4) | (mask4(eq_bytes(q.z, c4)) << 8) |
         (mask4(eq_bytes(q.w, c4)) << 12);
}

// Register fast path: the token is in r[] (32 bytes, byte i = r[i/4] >> 8*(i%4)), n in [1, 32], no
// whitespace.  Fully unrolled, so r[] stays in VGPRs.
__device__ __forceinline__ bool convert_token_regs(const uint32_t (&r)[8], int n, float& out) {
  uint64_t mant = 0;
  int nd = 0, exp10 = 0, phase = 0, ndig_int = 0, ndig_frac = 0, ndig_exp = 0, ev = 0, es = 1;
  bool neg = false, lead0 = false, ok = true;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    if (i >= n) break;
    const unsigned c = (r[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    const unsigned d = c - '0';
    if (phase == 0) {  // sign or first integer digit
      if (c == '-' && i == 0) {
        neg = true;
        continue;
      }
      phase = 1;
    }
    if (phase == 1) {
      if (d <= 9u) {
        if (ndig_int == 1 && lead0) ok = false;
        lead0 |= ndig_int == 0 && d == 0;
        ++ndig_int;
        if (mant != 0 || d != 0) {
          ok &= nd < 19;
          mant = mant * 10 + d;
          ++nd;
        }
      } else if (c == '.' && ndig_int > 0) {
        phase = 2;
      } else if ((c | 0x20u) == 'e' && ndig_int > 0) {
        phase = 3;
      } else {
        ok = false;
      }
    } else if (phase == 2) {
      if (d <= 9u) {
        ++ndig_frac;
        --exp10;
        if (mant != 0 || d != 0) {
          ok &= nd < 19;
          mant = mant * 10 + d;
          ++nd;
        }
      } else if ((c | 0x20u) == 'e' && ndig_frac > 0) {
        phase = 3;
      } else {
        ok = false;
      }
    } else {  // exponent
      if ((c == '-' || c == '+') && ndig_exp == 0 && es == 1) {
        es = c == '-' ? -1 : 1;
        if (c == '+') es = 2;  // seen '+': a further sign is invalid
      } else if (d <= 9u) {
        ++ndig_exp;
        ev = ev * 10 + static_cast<int>(d);
        if (ev > 10000) ev = 10000;
      } else {
        ok = false;
      }
    }
  }
  if (!ok || ndig_int == 0 || (phase == 2 && ndig_frac == 0) || (phase == 3 && ndig_exp == 0)) return false;
  exp10 += (es == -1 ? -ev : ev);
  float v;
  if (mant == 0) {
    v = 0.f;
  } else if (mant <= (1u << 24) && exp10 >= -10 && exp10 <= 10) {
    v = exp10 < 0 ? static_cast<float>(mant) / kP10f[-exp10] : static_cast<float>(mant) * kP10f[exp10];
  } else if (exp10 >= -66 && exp10 <= 66) {
    double dd = static_cast<double>(mant);
    int rr = mant > (1ull << 53);
    for (int e = exp10; e != 0; ++rr) {
      const int k = e > 0 ? (e > 22 ? 22 : e) : (e < -22 ? 22 : -e);
      dd = e > 0 ? dd * kP10d[k] : dd / kP10d[k];
      e += e > 0 ? -k : k;
    }
    const uint64_t bits = __double_as_longlong(dd);
    const long long low = static_cast<long long>(bits & ((1ull << 29) - 1)) - (1ll << 28);
    if (low >= -(rr + 1) && low <= rr + 1) return false;
    if (dd > 3.4028234663852886e38 || dd < 1.1754943508222875e-38) return false;
    v = static_cast<float>(dd);
  } else {
    return false;
  }
  out = __uint_as_float(__float_as_uint(v) | (static_cast<uint32_t>(neg) << 31));
  return true;
}

// Common-case fast path: [-](0|[1-9][0-9]*)[.[0-9]+] with at most 8 digits and no exponent, the
// shape every serializer emits for image-like data ("0.1234", "-12.5").  32-bit accumulation over
// at most 10 bytes instead of convert_token_regs' 32-step state machine; the value is computed by
// the same single fp32 rounding (mant <= 2^24, |exp10| <= 8), so it is bit-identical.  Anything
// else (exponent, > 8 digits, malformed) returns false and the caller runs the full converter,
// which decides acceptance and error status exactly as before.
// 10^k for k in [0, 15] without a (lane-divergent) memory lookup; exact in fp32 for k <= 10
__device__ __forceinline__ float pow10f_small(int k) {
  float p = (k & 1) ? 10.f : 1.f;
  p *= (k & 2) ? 100.f : 1.f;
  p *= (k & 4) ? 1e4f : 1.f;
  return (k & 8) ? p * 1e8f : p;
}

__device__ __forceinline__ bool convert_token_fast(const uint32_t (&r)[8], int n, float& out) {
  // SWAR form (no per-byte loop): body = the token after an optional '-', at most 10 bytes; the one
  // optional '.' is squeezed out and the <= 8 digits converted with three multiply-shift steps.
  if (n > 10 || n < 1) return false;
  const bool neg = (r[0] & 0xFFu) == '-';
  const int f = neg ? 1 : 0, L = n - f;  // body length
  const uint32_t d0 = __builtin_amdgcn_alignbyte(r[1], r[0], f), d1 = __builtin_amdgcn_alignbyte(r[2], r[1], f);
  const uint32_t d2 = r[2] >> (8 * f);
  // per-byte flags (0x80) over body bytes [0, L): '.', and "is a digit"
  auto digit = [](uint32_t x) {
    const uint32_t ge0 = (x | 0x80808080u) - 0x30303030u;
    const uint32_t gt9 = (x & 0x7F7F7F7Fu) + 0x46464646u;
    return ge0 & ~gt9 & ~x & 0x80808080u;
  };
  const uint64_t lo = static_cast<uint64_t>(d0) | (static_cast<uint64_t>(d1) << 32);
  const uint64_t in = L >= 8 ? ~0ull : (1ull << (8 * L)) - 1;                    // body bytes 0..7
  const uint32_t in2 = L <= 8 ? 0u : (L >= 12 ? ~0u : (1u << (8 * (L - 8))) - 1);  // body bytes 8..11
  const uint64_t dots = (static_cast<uint64_t>(eq_bytes(d0, 0x2E2E2E2Eu)) | (static_cast<uint64_t>(eq_bytes(d1, 0x2E2E2E2Eu)) << 32)) & in;
  const uint32_t dots2 = eq_bytes(d2, 0x2E2E2E2Eu) & in2;
  const uint64_t digs = (static_cast<uint64_t>(digit(d0)) | (static_cast<uint64_t>(digit(d1)) << 32)) & in;
  const uint32_t digs2 = digit(d2) & in2;
  const uint64_t all = in & 0x8080808080808080ull;
  const uint32_t all2 = in2 & 0x80808080u;
  if (dots2 || (digs2 != all2) || __popcll(dots) > 1 || ((digs | dots) != all)) return false;
  const int dp = dots ? (__builtin_ctzll(dots) >> 3) : -1;  // '.' position in the body
  const int nd = L - (dp >= 0 ? 1 : 0);
  if (nd < 1 || nd > 8 || dp == 0 || dp == L - 1) return false;  // digits before and after a '.'
  const uint32_t b0 = d0 & 0xFFu, b1 = (d0 >> 8) & 0xFFu;
  if (b0 == '0' && L > 1 && b1 != '.') return false;  // a leading '0' must be the whole integer part
  // squeeze the '.' out: digits now fill bytes [0, nd) of w (nd <= 8, so the dot is in bytes 0..7)
  uint64_t w = lo;
  if (dp >= 0) {
    const uint64_t below = (1ull << (8 * dp)) - 1;
    w = (lo & below) | (((lo >> 8) | (static_cast<uint64_t>(d2) << 56)) & ~below);
  }
  // right-align the nd digits at the top, '0'-padded below, then the 8-digit SWAR conversion
  const int sh = 8 * (8 - nd);
  w = sh ? ((w << sh) | (0x3030303030303030ull >> (64 - sh))) : w;
  w -= 0x3030303030303030ull;
  w = (w * 10) + (w >> 8);
  w = (((w & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
       (((w >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
  const uint32_t mant = static_cast<uint32_t>(w);
  if (mant > (1u << 24)) return false;
  const int frac = dp >= 0 ? L - dp - 1 : 0;
  const float v = mant == 0 ? 0.f : (frac > 0 ? static_cast<float>(mant) / pow10f_small(frac) : static_cast<float>(mant));
  out = __uint_as_float(__float_as_uint(v) | (static_cast<uint32_t>(neg) << 31));
  return true;
}

// Per-wave LDS image of the staged bytes: logical byte L (0 = chunk start - PRE) lives at
// L + 4 * ((L + 48) / 64), i.e. every lane's 64-byte region (and the PRE bytes before region 0) is
// followed by a 4-byte gap.  Lane regions then start 17 dwords apart, so the 64 lanes' token-window
// reads (one region each) hit distinct banks instead of 2 (a 16-way conflict on every read).
constexpr int kWaveLds = PRE + CHUNK + HALO + 4 * ((PRE + CHUNK + HALO + 48) / 64 + 1);
__device__ __forceinline__ int lpos(int L) { return L + 4 * ((L + 48) >> 6); }
__device__ __forceinline__ uint32_t ld32(const unsigned char* buf, int L) {  // L % 4 == 0
  return *reinterpret_cast<const uint32_t*>(buf + lpos(L));
}

__global__ __launch_bounds__(256) void dec_parse(const unsigned char* __restrict__ text, long long cap,
                                                 const long long* __restrict__ offs,
                                                 const unsigned char* __restrict__ packed,
                                                 const long long* __restrict__ poffs,
                                                 const long long* __restrict__ lens, int B,
                                                 const int* __restrict__ counts, const int* __restrict__ blank,
                                                 int* __restrict__ status, int* __restrict__ ntok,
                                                 float* __restrict__ out, long long numel, int max_chunks) {
  constexpr int WB = PRE + CHUNK + HALO;  // staged bytes per wave
  __shared__ __attribute__((aligned(16))) unsigned char sbuf[4][kWaveLds];
  __shared__ unsigned short sstarts[4][CHUNK / 2 + 2];
  __shared__ int red[4];
  __shared__ int pre[kDecMaxB];
  const int items = chunk_prefix(lens, B, pre, red);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char* buf = sbuf[wave];
  unsigned short* starts = sstarts[wave];
  for (int it = blockIdx.x * 4 + wave; it < items; it += gridDim.x * 4) {
    const int b = item_sample(pre, B, it), chunk = it - pre[b];
    const long long len = lens[b];
    const long long c0 = static_cast<long long>(chunk) * CHUNK;
    const bool last = c0 + CHUNK >= len;
    // token index of this chunk: the separators of the chunks before it
    const int* crow = counts + static_cast<size_t>(b) * max_chunks;
    int s = 0, nbv = 0;
    for (int c = lane; c < chunk; c += 64) s += crow[c];
    if (last)
      for (int c = lane; c <= chunk; c += 64) nbv |= !blank[static_cast<size_t>(b) * max_chunks + c];
    const int prefix = wave_sum(s);
    const int anynb = last ? wave_sum(nbv) : 0;
    if (c0 < len) {
      const unsigned char* t = text + (offs ? offs[b] : b * cap);
      const long long po = poffs ? poffs[b] : -1;
      const unsigned char* pk = po >= 0 ? packed + po : nullptr;
      const int lim = static_cast<int>(len - c0 < CHUNK + HALO ? len - c0 : CHUNK + HALO) + PRE;  // LDS end of text
      // stage [c0 - 16, c0 + CHUNK + HALO) (bytes outside [0, len) read as ' '; the byte before 0 as ',')
      int wsf = 0;
      for (int i = lane; i < WB / 16; i += 64) {
        const long long off = c0 - PRE + 16ll * i;
        uint4 q;
        if (off < 0) q = make_uint4(0x2C2C2C2Cu, 0x2C2C2C2Cu, 0x2C2C2C2Cu, 0x2C2C2C2Cu);
        else if (off >= len) q = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
        else q = load16(t, pk, off, len);
        uint32_t* d = reinterpret_cast<uint32_t*>(buf + lpos(16 * i));  // a 16-byte word never straddles a gap
        d[0] = q.x;
        d[1] = q.y;
        d[2] = q.z;
        d[3] = q.w;
        if (16 * i >= PRE && 16 * i < lim) wsf |= nonblank_all(q) ? 0 : 1;
      }
      wave_lds_sync();
      const bool anyws = __ballot(wsf) != 0;
      // token starts in my 64 bytes
      const int lo = PRE + 64 * lane;
      uint64_t cm = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        cm |= static_cast<uint64_t>(mask16(make_uint4(ld32(buf, lo + 16 * k), ld32(buf, lo + 16 * k + 4),
                                                       ld32(buf, lo + 16 * k + 8), ld32(buf, lo + 16 * k + 12)),
                                            0x2C2C2C2Cu))
              << (16 * k);
      uint64_t sm = (cm << 1) | (buf[lpos(lo - 1)] == ',' ? 1ull : 0ull);
      if (lo + 64 > lim) sm &= lim > lo ? (1ull << (lim - lo)) - 1ull : 0ull;
      // compact the starts into this wave's list, then take the tokens round-robin (lane l: tokens
      // l, l + 64, ...) so that consecutive lanes store consecutive values
      int total;
      int k = wave_excl_scan(__popcll(sm), total);
      while (sm) {
        starts[k++] = static_cast<unsigned short>(lo + __builtin_ctzll(sm));
        sm &= sm - 1;
      }
      wave_lds_sync();
      const long long base = static_cast<long long>(prefix) + (buf[lpos(PRE - 1)] != ',' ? 1 : 0);
      bool bad = lane == 0 && last && buf[lpos(lim - 1)] == ',';  // trailing comma
      for (int tk = lane; tk < total; tk += 64) {
        const long long idx = base + tk;  // idx >= numel: validated, not stored
        const int p = starts[tk];
        const int rem = lim - p;
        const bool inner = tk + 1 < total;  // the next start bounds the token
        int n = inner ? starts[tk + 1] - 1 - p : 32;
        float v = 0.f;
        bool good = false;
        int slow = -1;  // >= 0: convert bytes [p, p + slow) with the byte-wise converter
        if (inner && n <= 10 && !anyws) {  // hot path: a short token from a 12-byte window
          const int a4 = p & ~3, sh = p & 3;
          const uint32_t x0 = ld32(buf, a4), x1 = ld32(buf, a4 + 4), x2 = ld32(buf, a4 + 8), x3 = ld32(buf, a4 + 12);
          uint32_t r[8] = {__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                           __builtin_amdgcn_alignbyte(x3, x2, sh), 0, 0, 0, 0, 0};
          good = convert_token_fast(r, n, v);
          if (!good) slow = n;  // malformed or unusual: the byte-wise converter decides
        } else if (inner && n > 32) {  // longer than the register window
          slow = n;
        } else {
          const int a4 = p & ~3, sh = p & 3;
          uint32_t x[9];
#pragma unroll
          for (int i = 0; i < 9; ++i) x[i] = ld32(buf, a4 + 4 * i);
          uint32_t r[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) r[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], sh);
          if (!inner) {  // the chunk's last token: first ',' in the 32-byte window
#pragma unroll
            for (int i = 7; i >= 0; --i) {
              const uint32_t c = eq_bytes(r[i], 0x2C2C2C2Cu);
              if (c) n = 4 * i + (__builtin_ctz(c) >> 3);
            }
            if (rem < n) n = rem;
          }
          bool ws = false;
          if (anyws) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const uint32_t w = eq_bytes(r[i], 0x20202020u) | eq_bytes(r[i], 0x0A0A0A0Au) |
                                 eq_bytes(r[i], 0x0D0D0D0Du) | eq_bytes(r[i], 0x09090909u);
              const int lo_b = 4 * i;
              if (w && lo_b < n) ws |= lo_b + static_cast<int>(__builtin_ctz(w) >> 3) < n;
            }
          }
          if (!inner && n == 32 && rem > 32) {  // no ',' in the window: find it in LDS
            int e = p;
            while (e < WB && e < lim && buf[lpos(e)] != ',') ++e;
            if (!(e == WB && e < lim)) slow = e - p;  // else: longer than the halo -> host fallback
          } else if (ws) {
            slow = n;
          } else {
            good = n > 0 && (convert_token_fast(r, n, v) || convert_token_regs(r, n, v));
          }
        }
        if (slow >= 0) good = convert_token([&](int i) -> unsigned { return buf[lpos(p + i)]; }, slow, v);
        if (good && idx < numel) out[b * numel + idx] = v;
        bad |= !good;
      }
      if (bad) atomicOr(status + b, 1);
    }
    if (last) {  // the sample's token count, overflow status and zero-filled tail
      const long long n = anynb ? static_cast<long long>(prefix) + crow[chunk] + 1 : 0;
      if (lane == 0) {
        ntok[b] = static_cast<int>(n);
        if (n > numel) atomicOr(status + b, 2);
      }
      float* o = out + b * numel;
      for (long long i = n + lane; i < numel; i += 64) o[i] = 0.f;
    }
    wave_lds_sync();  // every lane done reading buf before the next item's staging
  }
}


// ------------------------------------------------------------------------------------------------
// 4-bit packed samples, decoded at the symbol (nibble) level.  The worker packs every request text
// it can (core/textpack.cpp): symbols 0-9 digits, 10 ',', 11 '.', 12 '-', 13 '+', 14 'e', 15 ' '
// (also the pad of an odd final symbol); symbol k of a sample = nibble k & 1 of packed byte k >> 1.
// The kernels above expand those nibbles to characters first and then scan bytes (~3.9k VALU
// instructions per 4 KiB chunk item); here separators, token starts and the common number shape
// are found with 8-symbols-per-word SWAR on the nibbles themselves, and the token's digits, already
// values 0-9, become the mantissa by a three-step BCD multiply-add.  Unusual tokens (exponents, > 8
// digits, interior blanks, malformed) take the byte-wise converter through a nibble -> character
// accessor, so acceptance, values and status bits are those of the character path (bit-identical
// to the host parser).  Work item = one wave per PCH symbols, as above.
// ------------------------------------------------------------------------------------------------
constexpr int PCH = 4096;    // symbols per work item (2 KiB packed); = CHUNK: the same scratch layout
constexpr int PHALO = 128;   // symbols past the chunk end the chunk's last token may reach
constexpr int PPRE = 32;     // symbols staged before the chunk (16 bytes)
constexpr int kPkStaged = (PPRE + PCH + PHALO) / 2;  // staged bytes per wave
// LDS position of staged byte L: every lane's 32-byte region (the 64 symbols it scans for starts)
// is followed by a 16-byte gap, so the 16 lanes of a ds_read_b128 group hit distinct banks
__device__ __forceinline__ int ppos(int L) { return L + 16 * ((L + 16) >> 5); }
constexpr int kPkLds = kPkStaged + 16 * ((kPkStaged + 16) / 32) + 16;

// 0x8 in each nibble of x equal to v
__device__ __forceinline__ uint32_t nib_eq(uint32_t x, uint32_t v) {
  const uint32_t t = x ^ (v * 0x11111111u);
  return ~(((t & 0x77777777u) + 0x77777777u) | t) & 0x88888888u;
}
__device__ __forceinline__ uint64_t nib_eq64(uint64_t x, uint64_t v) {
  const uint64_t t = x ^ (v * 0x1111111111111111ull);
  return ~(((t & 0x7777777777777777ull) + 0x7777777777777777ull) | t) & 0x8888888888888888ull;
}
// 8-bit mask (bit i = nibble i) from a 0x8-per-nibble word
__device__ __forceinline__ uint32_t nib_mask8(uint32_t z) {
  uint32_t m = (z >> 3) & 0x11111111u;
  m = (m | (m >> 3)) & 0x03030303u;
  m = (m | (m >> 6)) & 0x000F000Fu;
  return (m | (m >> 12)) & 0xFFu;
}
// nibbles of w at symbol positions >= n (n = valid symbols of this 8-symbol word) set to 15 (blank)
__device__ __forceinline__ uint32_t blank_from(uint32_t w, long long n) {
  if (n >= 8) return w;
  if (n <= 0) return 0xFFFFFFFFu;
  return w | (0xFFFFFFFFu << (4 * static_cast<int>(n)));
}
__device__ __forceinline__ unsigned sym2chr(unsigned v) {
  return v < 10 ? '0' + v : static_cast<unsigned>((0x20652B2D2E2Cull >> (8 * (v - 10))) & 0xFFu);
}

// Common number shape on a 64-bit window (symbol i = nibble i), n symbols before the separator:
// [' '][-](0|[1-9][0-9]*)[.[0-9]+] with <= 8 digits -- one optional leading blank is json.dumps'
// ", " separator.  Same single fp32 rounding as convert_token (mant <= 2^24 scaled by an exact
// power of ten), so the bits equal the character path's.  false: let the byte-wise converter decide.
__device__ __forceinline__ bool pk_fast(uint64_t w, int n, float& out) {
  if (n >= 1 && (w & 0xFu) == 15u) {
    w >>= 4;
    --n;
  }
  const bool neg = n >= 1 && (w & 0xFu) == 12u;
  if (neg) {
    w >>= 4;
    --n;
  }
  if (n < 1 || n > 10) return false;
  const uint64_t in8 = ((1ull << (4 * n)) - 1) & 0x8888888888888888ull;  // bit 3 of the body's nibbles
  const uint64_t ge10 = w & ((w << 1) | (w << 2)) & in8;                 // symbols 10-15
  const uint64_t dots = nib_eq64(w, 11) & in8;
  if (ge10 != dots || __popcll(dots) > 1) return false;  // every non-digit is the one '.'
  const int dp = dots ? (__builtin_ctzll(dots) >> 2) : -1;
  const int nd = n - (dp >= 0 ? 1 : 0);
  if (nd < 1 || nd > 8 || dp == 0 || dp == n - 1) return false;
  if ((w & 0xFu) == 0 && n > 1 && dp != 1) return false;  // a leading 0 is the whole integer part
  uint64_t d = w;
  if (dp >= 0) {
    const uint64_t below = (1ull << (4 * dp)) - 1;
    d = (w & below) | ((w >> 4) & ~below);
  }
  // the nd digits (most significant first = lowest nibble) right-aligned in 8 nibbles, leading zeros
  // below them, then pairs -> hundreds -> the 8-digit value
  uint32_t x = static_cast<uint32_t>(d << (4 * (8 - nd)));
  x = (x & 0x0F0F0F0Fu) * 10u + ((x >> 4) & 0x0F0F0F0Fu);
  x = (x & 0x00FF00FFu) * 100u + ((x >> 8) & 0x00FF00FFu);
  const uint32_t mant = (x & 0xFFFFu) * 10000u + (x >> 16);
  if (mant > (1u << 24)) return false;
  const int frac = dp >= 0 ? n - dp - 1 : 0;
  const float v = mant == 0 ? 0.f : (frac > 0 ? static_cast<float>(mant) / pow10f_small(frac) : static_cast<float>(mant));
  out = __uint_as_float(__float_as_uint(v) | (static_cast<uint32_t>(neg) << 31));
  return true;
}

// Packed sample b: 16 packed bytes at byte offset `bo` of the sample (bo % 16 == 0), symbols at or
// beyond len blank; bytes before the sample read as separators (the symbol before 0 starts token 0).
__device__ __forceinline__ uint4 pk_load16(const unsigned char* pk, long long bo, long long len) {
  if (bo < 0) return make_uint4(0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu);
  const long long s0 = 2 * bo;  // first symbol of these 16 bytes
  if (s0 >= len) return make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  uint4 q = *reinterpret_cast<const uint4*>(pk + bo);
  if (s0 + 32 > len) {
    q.x = blank_from(q.x, len - s0);
    q.y = blank_from(q.y, len - s0 - 8);
    q.z = blank_from(q.z, len - s0 - 16);
    q.w = blank_from(q.w, len - s0 - 24);
  }
  return q;
}

// A raw (unpacked) sample's character as a symbol: the packer's alphabet, plus 'E' as 'e' and
// '\t' '\n' '\r' as ' ' (JSON gives them the same meaning in a number list); any other character is
// `invalid` (the sample then goes to the host parser, which decides and reports).
__device__ __forceinline__ uint32_t chr_to_sym(uint32_t c, bool& invalid) {
  if (c - '0' <= 9u) return c - '0';
  if (c == ',') return 10;
  if (c == '.') return 11;
  if (c == '-') return 12;
  if (c == '+') return 13;
  if ((c | 0x20u) == 'e') return 14;
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r') return 15;
  invalid = true;
  return 15;
}

// 32 symbols of sample b starting at symbol 2 * bo (bo % 16 == 0), packed (pk != nullptr) or
// translated from raw characters at raw + 2 * bo (the rare unpackable texts); the blank /
// separator rules of pk_load16.
__device__ __forceinline__ uint4 sym_load16(const unsigned char* pk, const unsigned char* raw, long long bo,
                                            long long len, bool& invalid) {
  if (pk) return pk_load16(pk, bo, len);
  if (bo < 0) return make_uint4(0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu);
  const long long s0 = 2 * bo;
  if (s0 >= len) return make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  const uint4 a = *reinterpret_cast<const uint4*>(raw + s0), c = *reinterpret_cast<const uint4*>(raw + s0 + 16);
  const uint32_t ch[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    bool inv = false;
    const uint32_t v = chr_to_sym((ch[k >> 2] >> (8 * (k & 3))) & 0xFFu, inv);
    if (inv && s0 + k < len) invalid = true;  // bytes past the text are blanked below
    w[k >> 3] |= v << (4 * (k & 7));
  }
  return make_uint4(blank_from(w[0], len - s0), blank_from(w[1], len - s0 - 8), blank_from(w[2], len - s0 - 16),
                    blank_from(w[3], len - s0 - 24));
}

// the packed bytes of sample b (nullptr: raw characters at its text slot)
__device__ __forceinline__ const unsigned char* pk_ptr(const unsigned char* packed, const long long* poffs, int b) {
  return poffs[b] >= 0 ? packed + poffs[b] : nullptr;
}

// Separator count and "any non-blank" per PCH-symbol chunk of every packed sample; resets status
// (and ntok of skipped samples) for EVERY sample -- this kernel runs first in a packed launch.
__global__ __launch_bounds__(256) void pk_count(const unsigned char* __restrict__ packed,
                                                const long long* __restrict__ poffs,
                                                const unsigned char* __restrict__ text, long long cap,
                                                const long long* __restrict__ offs,
                                                const long long* __restrict__ lens, int B, int* __restrict__ counts,
                                                int* __restrict__ blank, int* __restrict__ status,
                                                int* __restrict__ ntok, int max_chunks) {
  __shared__ int red[4];
  __shared__ int pre[kDecMaxB];
  if (blockIdx.x == 0) {
    for (int b = threadIdx.x; b < B; b += 256) {
      status[b] = 0;
      if (lens[b] < 0) ntok[b] = -1;
    }
  }
  int carry = 0;
  for (int i0 = 0; i0 < B; i0 += 256) {
    const int i = i0 + threadIdx.x;
    int v = 0;
    if (i < B) {
      const long long len = lens[i];
      v = len < 0 ? 0 : len == 0 ? 1 : static_cast<int>((len + PCH - 1) / PCH);
    }
    int tot;
    const int ex = block_excl_scan(v, red, tot);
    if (i < B) pre[i] = carry + ex;
    carry += tot;
  }
  __syncthreads();
  const int items = carry;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int it = blockIdx.x * 4 + wave; it < items; it += gridDim.x * 4) {
    const int b = item_sample(pre, B, it), chunk = it - pre[b];
    const long long len = lens[b];
    const unsigned char* pk = pk_ptr(packed, poffs, b);
    const unsigned char* raw = text + (offs ? offs[b] : b * cap);
    // lane: 64 symbols (32 packed bytes) as two 16-byte words (a misaligned packed slot is not read:
    // pk_parse sends that sample to the host parser)
    const long long bo = static_cast<long long>(chunk) * (PCH / 2) + 32 * lane;
    int c = 0, nb = 0;
    bool inv = false;
#pragma unroll
    for (int k = 0; k < ((pk && (poffs[b] & 15)) ? 0 : 2); ++k) {
      const uint4 q = sym_load16(pk, raw, bo + 16 * k, len, inv);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c += __popc(nib_eq(w[j], 10));
        nb |= nib_eq(w[j], 15) != 0x88888888u;
      }
    }
    c = wave_sum(c);
    nb = wave_sum(nb);
    if (lane == 0) {
      counts[b * max_chunks + chunk] = c;
      blank[b * max_chunks + chunk] = nb == 0;
    }
  }
}

__global__ __launch_bounds__(256) void pk_parse(const unsigned char* __restrict__ packed,
                                                const long long* __restrict__ poffs,
                                                const unsigned char* __restrict__ text, long long cap,
                                                const long long* __restrict__ offs,
                                                const long long* __restrict__ lens, int B,
                                                const int* __restrict__ counts, const int* __restrict__ blank,
                                                int* __restrict__ status, int* __restrict__ ntok,
                                                float* __restrict__ out, long long numel, int max_chunks) {
  __shared__ __attribute__((aligned(16))) unsigned char sbuf[4][kPkLds];
  __shared__ int red[4];
  __shared__ int pre[kDecMaxB];
  int carry = 0;
  for (int i0 = 0; i0 < B; i0 += 256) {
    const int i = i0 + threadIdx.x;
    int v = 0;
    if (i < B) {
      const long long len = lens[i];
      v = len < 0 ? 0 : len == 0 ? 1 : static_cast<int>((len + PCH - 1) / PCH);
    }
    int tot;
    const int ex = block_excl_scan(v, red, tot);
    if (i < B) pre[i] = carry + ex;
    carry += tot;
  }
  __syncthreads();
  const int items = carry;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char* buf = sbuf[wave];
  // symbol j of the staged window (j = chunk symbol + PPRE)
  auto sym = [&](int j) -> unsigned { return (buf[ppos(j >> 1)] >> (4 * (j & 1))) & 0xFu; };
  auto word = [&](int L) -> uint32_t { return *reinterpret_cast<const uint32_t*>(buf + ppos(L)); };  // L % 4 == 0
  constexpr int kNone = 1 << 30;
  for (int it = blockIdx.x * 4 + wave; it < items; it += gridDim.x * 4) {
    const int b = item_sample(pre, B, it), chunk = it - pre[b];
    const long long len = lens[b];
    const long long c0 = static_cast<long long>(chunk) * PCH;
    const bool last = c0 + PCH >= len;
    const int* crow = counts + static_cast<size_t>(b) * max_chunks;
    int s = 0, nbv = 0;
    for (int c = lane; c < chunk; c += 64) s += crow[c];
    if (last)
      for (int c = lane; c <= chunk; c += 64) nbv |= !blank[static_cast<size_t>(b) * max_chunks + c];
    const int prefix = wave_sum(s);
    const int anynb = last ? wave_sum(nbv) : 0;
    const unsigned char* pk = pk_ptr(packed, poffs, b);
    const unsigned char* raw = text + (offs ? offs[b] : b * cap);
    bool bad = false;
    if (pk && (poffs[b] & 15) != 0) {  // the kernels read 16-byte words: a misaligned slot goes to the host parser
      bad = lane == 0;
    } else if (c0 < len) {
      const int lim = static_cast<int>(len - c0 < PCH + PHALO ? len - c0 : PCH + PHALO);  // chunk symbols of text
      // stage the symbols [c0 - 32, c0 + PCH + PHALO) (packed bytes; raw samples translated on load)
      bool inv = false;
      for (int i = lane; i < kPkStaged / 16; i += 64) {
        const uint4 q = sym_load16(pk, raw, c0 / 2 - PPRE / 2 + 16ll * i, len, inv);
        *reinterpret_cast<uint4*>(buf + ppos(16 * i)) = q;
      }
      bad = inv;  // a character outside the number alphabet: the host parser decides (and reports it)
      wave_lds_sync();
      // Token starts among my 64 symbols [64 lane, 64 lane + 64) of the chunk (the symbol after a ','),
      // kept in a register mask: each lane converts the tokens that start in its own region, in order,
      // so no start list is compacted through LDS.  A token ends at the next start (mine, or the first
      // one of a later lane: a suffix minimum over the lanes); the chunk's last token at the next ','
      // in the staged halo or the end of the text.
      const int L0 = PPRE / 2 + 32 * lane;  // staged byte of my first symbol
      const uint4 q0 = *reinterpret_cast<const uint4*>(buf + ppos(L0));
      const uint4 q1 = *reinterpret_cast<const uint4*>(buf + ppos(L0 + 16));
      const uint64_t cm = static_cast<uint64_t>(nib_mask8(nib_eq(q0.x, 10)) | (nib_mask8(nib_eq(q0.y, 10)) << 8) |
                                                (nib_mask8(nib_eq(q0.z, 10)) << 16) | (nib_mask8(nib_eq(q0.w, 10)) << 24)) |
                          (static_cast<uint64_t>(nib_mask8(nib_eq(q1.x, 10)) | (nib_mask8(nib_eq(q1.y, 10)) << 8) |
                                                 (nib_mask8(nib_eq(q1.z, 10)) << 16) | (nib_mask8(nib_eq(q1.w, 10)) << 24))
                           << 32);
      const int lo = 64 * lane;  // chunk symbol of bit 0
      uint64_t sm = (cm << 1) | (sym(PPRE + lo - 1) == 10u ? 1ull : 0ull);
      if (lo + 64 > lim) sm &= lim > lo ? (1ull << (lim - lo)) - 1ull : 0ull;
      if (lo + 64 > PCH) sm &= lo < PCH ? (1ull << (PCH - lo)) - 1ull : 0ull;  // starts past the chunk: next item's
      int total;
      const int k0 = wave_excl_scan(__popcll(sm), total);
      // first start of the lanes after me
      int nxt = sm ? lo + __builtin_ctzll(sm) : kNone;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_down(nxt, o, 64);
        if (lane + o < 64) nxt = min(nxt, y);
      }
      nxt = __shfl_down(nxt, 1, 64);
      if (lane == 63) nxt = kNone;
      const long long base = static_cast<long long>(prefix) + (sym(PPRE - 1) != 10u ? 1 : 0) + k0;
      bad |= lane == 0 && last && len > 0 && sym(PPRE + static_cast<int>(len - c0) - 1) == 10u;  // trailing ','
      float* orow = out + b * numel;
      for (long long idx = base; sm; ++idx) {  // idx >= numel: validated, not stored
        const int p = lo + __builtin_ctzll(sm);
        sm &= sm - 1;
        const int e_start = sm ? lo + __builtin_ctzll(sm) : nxt;  // the next token's start
        int n;
        bool too_long = false;
        if (e_start != kNone) {
          n = e_start - 1 - p;
        } else {  // the chunk's last token: up to the next ',' in the staged halo, or the end of the text
          int e = p;
          while (e < lim && sym(PPRE + e) != 10u) ++e;
          n = e - p;
          too_long = e == lim && lim == PCH + PHALO && len - c0 > PCH + PHALO;  // runs past the halo
        }
        float v = 0.f;
        bool good = false;
        if (!too_long) {
          if (n <= 16) {  // 64-bit window from three staged words
            const int j = PPRE + p, L = j >> 1, a4 = L & ~3;
            const uint64_t w01 = static_cast<uint64_t>(word(a4)) | (static_cast<uint64_t>(word(a4 + 4)) << 32);
            const uint64_t w2 = word(a4 + 8);
            const int sh = 8 * (L & 3) + 4 * (j & 1);
            const uint64_t w = sh ? (w01 >> sh) | (w2 << (64 - sh)) : w01;
            good = pk_fast(w, n, v);
          }
          if (!good) good = convert_token([&](int i) -> unsigned { return sym2chr(sym(PPRE + p + i)); }, n, v);
        }
        if (good && idx < numel) orow[idx] = v;
        bad |= !good;
      }
    }
    if (bad) atomicOr(status + b, 1);
    if (last) {  // the sample's token count, overflow status and zero-filled tail
      const long long n = anynb ? static_cast<long long>(prefix) + crow[chunk] + 1 : 0;
      if (lane == 0) {
        ntok[b] = static_cast<int>(n);
        if (n > numel) atomicOr(status + b, 2);
      }
      float* o = out + b * numel;
      for (long long i = n + lane; i < numel; i += 64) o[i] = 0.f;
    }
    wave_lds_sync();  // every lane done reading buf before the next item's staging
  }
}
int g_decode_variant = 0;

}  // namespace

void set_decode_variant(int v) { g_decode_variant = v; }

size_t decode_scratch_bytes(int max_batch, size_t text_cap) {
  const size_t chunks = (text_cap + CHUNK - 1) / CHUNK;
  return static_cast<size_t>(max_batch) * chunks * 2 * sizeof(int);
}

hipError_t decode_json_numbers(const unsigned char* text, const long long* offs, size_t text_cap,
                               const long long* lens, int B, float* out, long long numel, int* status, int* ntok,
                               void* scratch, hipStream_t s, const unsigned char* packed, const long long* poffs) {
  if (text_cap % CHUNK || B < 1) return hipErrorInvalidValue;
  const int max_chunks = static_cast<int>(text_cap / CHUNK);
  int* counts = static_cast<int*>(scratch);
  // batches above the kernels' per-launch sample table run in passes of kDecMaxB samples (the
  // scratch is sized for the whole batch; each pass uses its front)
  for (int b0 = 0; b0 < B; b0 += kDecMaxB) {
    const int nb = std::min(B - b0, kDecMaxB);
    int* blank = counts + static_cast<size_t>(nb) * max_chunks;
    const unsigned char* t = offs ? text : text + static_cast<size_t>(b0) * text_cap;  // contiguous: slot b at b * cap
    const long long* o = offs ? offs + b0 : nullptr;
    const long long* po = poffs ? poffs + b0 : nullptr;
    const int grid = static_cast<int>(std::min<long long>((static_cast<long long>(max_chunks) * nb + 3) / 4, kDecGrid));
    if (packed && po && g_decode_variant == 0) {
      // the symbol-level kernels: packed samples read as nibbles, raw ones translated on load
      hipLaunchKernelGGL(pk_count, dim3(grid), dim3(256), 0, s, packed, po, t, static_cast<long long>(text_cap), o,
                         lens + b0, nb, counts, blank, status + b0, ntok + b0, max_chunks);
      hipLaunchKernelGGL(pk_parse, dim3(grid), dim3(256), 0, s, packed, po, t, static_cast<long long>(text_cap), o,
                         lens + b0, nb, counts, blank, status + b0, ntok + b0, out + static_cast<size_t>(b0) * numel, numel,
                         max_chunks);
      continue;
    }
    hipLaunchKernelGGL(dec_count, dim3(grid), dim3(256), 0, s, t, static_cast<long long>(text_cap), o, packed, po,
                       lens + b0, nb, counts, blank, status + b0, ntok + b0, max_chunks);
    hipLaunchKernelGGL(dec_parse, dim3(grid), dim3(256), 0, s, t, static_cast<long long>(text_cap), o, packed, po,
                       lens + b0, nb, counts, blank, status + b0, ntok + b0, out + static_cast<size_t>(b0) * numel, numel,
                       max_chunks);
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace die
