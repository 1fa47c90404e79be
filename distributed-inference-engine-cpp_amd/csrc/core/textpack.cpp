#include "textpack.h"

#include <immintrin.h>

namespace die {

namespace {

constexpr char kSym2Chr[16] = {'0', '1', '2', '3', '4', '5', '6', '7', '8', '9', ',', '.', '-', '+', 'e', ' '};

struct Chr2Sym {
  int8_t t[256];
  constexpr Chr2Sym() : t() {
    for (int i = 0; i < 256; ++i) t[i] = -1;
    for (int s = 0; s < 16; ++s) t[static_cast<unsigned char>(kSym2Chr[s])] = static_cast<int8_t>(s);
  }
};
constexpr Chr2Sym kChr2Sym{};

inline bool pack_scalar(const unsigned char* s, size_t n, uint8_t* d) {
  size_t k = 0;
  for (; k + 1 < n; k += 2) {
    const int a = kChr2Sym.t[s[k]], b = kChr2Sym.t[s[k + 1]];
    if ((a | b) < 0) return false;
    d[k >> 1] = static_cast<uint8_t>(a | (b << 4));
  }
  if (k < n) {
    const int a = kChr2Sym.t[s[k]];
    if (a < 0) return false;
    d[k >> 1] = static_cast<uint8_t>(a | (15 << 4));
  }
  return true;
}

// 32 text bytes -> 32 symbols (0..15) and an all-valid mask
inline __m256i classify(__m256i c, __m256i& ok) {
  // indexed by the low nibble: symbol / the one non-digit byte with that low nibble.  Unused
  // entries hold 0x00, whose low nibble differs from the index, so they never compare equal.
  const __m256i sym_tab = _mm256_setr_epi8(15, 0, 0, 0, 0, 14, 0, 0, 0, 0, 0, 13, 10, 12, 11, 0,
                                           15, 0, 0, 0, 0, 14, 0, 0, 0, 0, 0, 13, 10, 12, 11, 0);
  const __m256i chr_tab = _mm256_setr_epi8(' ', 0, 0, 0, 0, 'e', 0, 0, 0, 0, 0, '+', ',', '-', '.', 0,
                                           ' ', 0, 0, 0, 0, 'e', 0, 0, 0, 0, 0, '+', ',', '-', '.', 0);
  const __m256i low = _mm256_and_si256(c, _mm256_set1_epi8(0x0F));
  const __m256i d = _mm256_sub_epi8(c, _mm256_set1_epi8('0'));
  const __m256i is_digit = _mm256_cmpeq_epi8(_mm256_min_epu8(d, _mm256_set1_epi8(9)), d);
  const __m256i other = _mm256_cmpeq_epi8(_mm256_shuffle_epi8(chr_tab, low), c);
  ok = _mm256_and_si256(ok, _mm256_or_si256(is_digit, other));
  return _mm256_blendv_epi8(_mm256_shuffle_epi8(sym_tab, low), d, is_digit);
}

}  // namespace

bool pack_nibbles(const char* src, size_t n, uint8_t* dst) {
  const auto* s = reinterpret_cast<const unsigned char*>(src);
  const __m256i pair = _mm256_set1_epi16(0x1001);  // even byte * 1 + odd byte * 16
  size_t i = 0;
  __m256i ok = _mm256_set1_epi8(-1);
  for (; i + 64 <= n; i += 64) {
    const __m256i a = classify(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)), ok);
    const __m256i b = classify(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32)), ok);
    const __m256i pa = _mm256_maddubs_epi16(a, pair), pb = _mm256_maddubs_epi16(b, pair);
    const __m256i packed = _mm256_permute4x64_epi64(_mm256_packus_epi16(pa, pb), 0xD8);
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + (i >> 1)), packed);
    if ((i & 4095) == 0 && _mm256_movemask_epi8(ok) != -1) return false;  // early out on raw text
  }
  if (_mm256_movemask_epi8(ok) != -1) return false;
  return pack_scalar(s + i, n - i, dst + (i >> 1));
}

void unpack_nibbles(const uint8_t* src, size_t n, char* dst) {
  for (size_t k = 0; k < n; ++k) {
    const uint8_t b = src[k >> 1];
    dst[k] = kSym2Chr[(k & 1) ? (b >> 4) : (b & 15)];
  }
}

}  // namespace die
