#include "json.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>

namespace die {

// ------------------------------------------------------------------------------------------------
// DOM
// ------------------------------------------------------------------------------------------------

Json::Json(const std::vector<float>& v) : type_(Type::Array) {
  a_.reserve(v.size());
  for (float f : v) a_.emplace_back(f);
}

bool Json::as_bool() const {
  if (type_ != Type::Bool) throw JsonError("type must be boolean");
  return b_;
}
int64_t Json::as_int() const {
  if (type_ == Type::Int) return i_;
  if (type_ == Type::Float) return static_cast<int64_t>(d_);
  throw JsonError("type must be number");
}
double Json::as_double() const {
  if (type_ == Type::Float) return d_;
  if (type_ == Type::Int) return static_cast<double>(i_);
  throw JsonError("type must be number");
}
const std::string& Json::as_string() const {
  if (type_ != Type::String) throw JsonError("type must be string");
  return s_;
}
const Json::Array& Json::as_array() const {
  if (type_ != Type::Array) throw JsonError("type must be array");
  return a_;
}
Json::Array& Json::as_array() {
  if (type_ != Type::Array) throw JsonError("type must be array");
  return a_;
}
const Json::Object& Json::as_object() const {
  if (type_ != Type::Object) throw JsonError("type must be object");
  return o_;
}

Json& Json::operator[](const std::string& key) {
  if (type_ == Type::Null) type_ = Type::Object;
  if (type_ != Type::Object) throw JsonError("cannot use operator[] with a string argument");
  for (auto& kv : o_)
    if (kv.first == key) return kv.second;
  o_.emplace_back(key, Json());
  return o_.back().second;
}
const Json* Json::find(const std::string& key) const {
  if (type_ != Type::Object) return nullptr;
  for (auto& kv : o_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}
const Json& Json::at(const std::string& key) const {
  const Json* j = find(key);
  if (!j) throw JsonError("key '" + key + "' not found");
  return *j;
}
void Json::push_back(Json v) {
  if (type_ == Type::Null) type_ = Type::Array;
  if (type_ != Type::Array) throw JsonError("cannot use push_back() with non-array");
  a_.push_back(std::move(v));
}
const Json& Json::operator[](size_t i) const {
  if (type_ != Type::Array) throw JsonError("cannot use operator[] with a numeric argument");
  return a_.at(i);
}
size_t Json::size() const {
  if (type_ == Type::Array) return a_.size();
  if (type_ == Type::Object) return o_.size();
  if (type_ == Type::Null) return 0;
  return 1;
}

void append_json_string(std::string& out, std::string_view s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

static inline void append_double(std::string& out, double d, bool f32) {
  if (!std::isfinite(d)) {
    out += "null";
    return;
  }
  char buf[40];
  std::to_chars_result r = f32 ? std::to_chars(buf, buf + sizeof buf, static_cast<float>(d))
                               : std::to_chars(buf, buf + sizeof buf, d);
  // Keep a visible fraction/exponent so the value reads back as a float, like nlohmann does.
  bool has_dot = false;
  for (char* q = buf; q < r.ptr; ++q)
    if (*q == '.' || *q == 'e' || *q == 'n' || *q == 'i') has_dot = true;
  out.append(buf, r.ptr);
  if (!has_dot) out += ".0";
}

void append_float_array(std::string& out, const float* v, size_t n) {
  out.reserve(out.size() + n * 12 + 2);
  out.push_back('[');
  char buf[32];
  for (size_t i = 0; i < n; ++i) {
    if (i) out.push_back(',');
    float f = v[i];
    if (!std::isfinite(f)) {
      out += "null";
      continue;
    }
    auto r = std::to_chars(buf, buf + sizeof buf, f);
    out.append(buf, r.ptr);
  }
  out.push_back(']');
}

void Json::dump_to(std::string& out) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: {
      char buf[24];
      auto r = std::to_chars(buf, buf + sizeof buf, i_);
      out.append(buf, r.ptr);
      break;
    }
    case Type::Float: append_double(out, d_, is_f32_); break;
    case Type::String: append_json_string(out, s_); break;
    case Type::Array: {
      out.push_back('[');
      for (size_t i = 0; i < a_.size(); ++i) {
        if (i) out.push_back(',');
        a_[i].dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      for (size_t i = 0; i < o_.size(); ++i) {
        if (i) out.push_back(',');
        append_json_string(out, o_[i].first);
        out.push_back(':');
        o_[i].second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump() const {
  std::string s;
  dump_to(s);
  return s;
}

// ------------------------------------------------------------------------------------------------
// Parser
// ------------------------------------------------------------------------------------------------

namespace {

struct Cursor {
  const char* p;
  const char* end;
  const char* begin;

  [[noreturn]] void fail(const char* what) const {
    throw JsonError(std::string("[json.exception.parse_error] syntax error at byte ") +
                    std::to_string(p - begin + 1) + ": " + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  char peek() {
    ws();
    if (p >= end) fail("unexpected end of input");
    return *p;
  }
  void expect(char c) {
    if (peek() != c) {
      char msg[64];
      std::snprintf(msg, sizeof msg, "expected '%c'", c);
      fail(msg);
    }
    ++p;
  }
};

void append_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back(static_cast<char>(cp));
  } else if (cp < 0x800) {
    out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  } else {
    out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
  }
}

uint32_t parse_hex4(Cursor& c) {
  if (c.end - c.p < 4) c.fail("bad \\u escape");
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) {
    char h = *c.p++;
    v <<= 4;
    if (h >= '0' && h <= '9') v |= h - '0';
    else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
    else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
    else c.fail("bad \\u escape");
  }
  return v;
}

std::string parse_string(Cursor& c) {
  c.expect('"');
  std::string out;
  const char* run = c.p;
  while (true) {
    if (c.p >= c.end) c.fail("unterminated string");
    char ch = *c.p;
    if (ch == '"') {
      out.append(run, c.p);
      ++c.p;
      return out;
    }
    if (static_cast<unsigned char>(ch) < 0x20) c.fail("control character in string");
    if (ch == '\\') {
      out.append(run, c.p);
      ++c.p;
      if (c.p >= c.end) c.fail("unterminated escape");
      char e = *c.p++;
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = parse_hex4(c);
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (c.end - c.p >= 6 && c.p[0] == '\\' && c.p[1] == 'u') {
              c.p += 2;
              uint32_t lo = parse_hex4(c);
              if (lo < 0xDC00 || lo > 0xDFFF) c.fail("bad surrogate pair");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              c.fail("bad surrogate pair");
            }
          }
          append_utf8(out, cp);
          break;
        }
        default: c.fail("bad escape");
      }
      run = c.p;
    } else {
      ++c.p;
    }
  }
}

// Skip a string without materialising it.
void skip_string(Cursor& c) {
  c.expect('"');
  while (true) {
    const char* q = static_cast<const char*>(std::memchr(c.p, '"', c.end - c.p));
    if (!q) c.fail("unterminated string");
    // count preceding backslashes
    const char* b = q;
    while (b > c.p && b[-1] == '\\') --b;
    c.p = q + 1;
    if (((q - b) & 1) == 0) return;
  }
}

const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
const float kPow10f[] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};

// Scan a JSON number; returns mantissa digits etc.  Used by both float and DOM paths.
struct NumScan {
  uint64_t mant = 0;
  int digits = 0;      // significant digits accumulated into mant (<= 19)
  int exp10 = 0;       // value = mant * 10^exp10 (when !overflow)
  bool neg = false;
  bool is_int = true;  // no fraction / exponent
  bool truncated = false;
  const char* start = nullptr;
  const char* stop = nullptr;
};

inline bool scan_number(const char*& p, const char* end, NumScan& s) {
  s.start = p;
  if (p < end && *p == '-') {
    s.neg = true;
    ++p;
  }
  if (p >= end) return false;
  if (*p == '0') {
    ++p;
  } else if (*p >= '1' && *p <= '9') {
    while (p < end && static_cast<unsigned>(*p - '0') < 10u) {
      if (s.digits < 19) {
        s.mant = s.mant * 10 + static_cast<unsigned>(*p - '0');
        if (s.mant) ++s.digits;
      } else {
        ++s.exp10;
        s.truncated = true;
      }
      ++p;
    }
  } else {
    return false;
  }
  if (p < end && *p == '.') {
    s.is_int = false;
    ++p;
    if (p >= end || static_cast<unsigned>(*p - '0') >= 10u) return false;
    while (p < end && static_cast<unsigned>(*p - '0') < 10u) {
      if (s.digits < 19) {
        s.mant = s.mant * 10 + static_cast<unsigned>(*p - '0');
        if (s.mant) ++s.digits;
        --s.exp10;
      } else {
        s.truncated = true;
      }
      ++p;
    }
  }
  if (p < end && (*p == 'e' || *p == 'E')) {
    s.is_int = false;
    ++p;
    bool eneg = false;
    if (p < end && (*p == '+' || *p == '-')) {
      eneg = *p == '-';
      ++p;
    }
    if (p >= end || static_cast<unsigned>(*p - '0') >= 10u) return false;
    int e = 0;
    while (p < end && static_cast<unsigned>(*p - '0') < 10u) {
      if (e < 100000) e = e * 10 + (*p - '0');
      ++p;
    }
    s.exp10 += eneg ? -e : e;
  }
  s.stop = p;
  return true;
}

float slow_float(const char* b, const char* e) {
  float v = 0.f;
  auto r = std::from_chars(b, e, v);
  if (r.ec == std::errc::result_out_of_range) {
    // from_chars leaves v untouched on range errors: mirror strtof (inf / 0).
    std::string tmp(b, e);
    v = std::strtof(tmp.c_str(), nullptr);
  }
  return v;
}

double slow_double(const char* b, const char* e) {
  std::string tmp(b, e);
  return std::strtod(tmp.c_str(), nullptr);
}

inline float scan_to_float(const NumScan& s) {
  if (s.mant == 0) return s.neg ? -0.f : 0.f;
  if (!s.truncated) {
    // Clinger fast path in float: exact mantissa and exact power of ten -> one rounding.
    if (s.mant <= (1u << 24) && s.exp10 >= -10 && s.exp10 <= 10) {
      float m = static_cast<float>(s.mant);
      float v = s.exp10 < 0 ? m / kPow10f[-s.exp10] : m * kPow10f[s.exp10];
      return s.neg ? -v : v;
    }
    // Clinger in double (one correct rounding), then to float.  Double rounding can only go
    // wrong when the double lands exactly on a float halfway point: detect that and fall back.
    if (s.mant <= (1ull << 53) && s.exp10 >= -22 && s.exp10 <= 22) {
      double m = static_cast<double>(s.mant);
      double d = s.exp10 < 0 ? m / kPow10[-s.exp10] : m * kPow10[s.exp10];
      uint64_t bits;
      std::memcpy(&bits, &d, sizeof bits);
      const uint64_t low = bits & ((1ull << 29) - 1);
      const int bexp = static_cast<int>((bits >> 52) & 0x7FF) - 1023;
      if (low != (1ull << 28) && bexp > -126 && bexp < 127) {
        float v = static_cast<float>(d);
        return s.neg ? -v : v;
      }
    }
  }
  return slow_float(s.start, s.stop);
}

// ---- SWAR fast path for the common "-?d{1,8}(.d{1,8})?" numbers ----------------------------------

inline uint64_t load8(const char* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
// Number of leading ASCII digits (0..8) in the 8 bytes at p (little-endian: first char = low byte).
inline int leading_digits(uint64_t v) {
  const uint64_t x = (v & 0xF0F0F0F0F0F0F0F0ull) | (((v + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) >> 4);
  const uint64_t nd = x ^ 0x3333333333333333ull;
  if (nd == 0) return 8;
  return __builtin_ctzll(nd) >> 3;
}
// Value of the first k (1..8) digits of v.
inline uint32_t swar_digits(uint64_t v, int k) {
  uint64_t val = (v & 0x0F0F0F0F0F0F0F0Full) << (8 * (8 - k));
  val = (val * 2561) >> 8;
  val = ((val & 0x00FF00FF00FF00FFull) * 6553601) >> 16;
  return static_cast<uint32_t>(((val & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32);
}
const uint32_t kPow10u[] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000};

// Returns true and advances p if the number has the simple form; false leaves p untouched.
inline bool fast_simple_float(const char*& p, const char* end, float& out) {
  const char* q = p;
  if (end - q < 20) return false;
  const bool neg = *q == '-';
  q += neg;
  const uint64_t vi = load8(q);
  const int ki = leading_digits(vi);
  if (ki == 0 || ki == 8) return false;
  if (ki > 1 && *q == '0') return false;  // leading zero: let the strict scanner reject it
  uint64_t mant = swar_digits(vi, ki);
  q += ki;
  int exp10 = 0;
  if (*q == '.') {
    ++q;
    const uint64_t vf = load8(q);
    const int kf = leading_digits(vf);
    if (kf == 0 || kf == 8) return false;
    mant = mant * kPow10u[kf] + swar_digits(vf, kf);
    exp10 = -kf;
    q += kf;
  }
  if (*q == 'e' || *q == 'E') return false;
  float v;
  if (mant <= (1u << 24)) {
    const float m = static_cast<float>(mant);
    v = m / kPow10f[-exp10];
  } else {
    // <= 16 significant digits: exact in double; one correctly rounded division, then the
    // halfway check of scan_to_float.
    const double d = static_cast<double>(mant) / kPow10[-exp10];
    uint64_t bits;
    std::memcpy(&bits, &d, sizeof bits);
    if ((bits & ((1ull << 29) - 1)) == (1ull << 28)) return false;
    v = static_cast<float>(d);
  }
  out = neg ? -v : v;
  p = q;
  return true;
}

// ---- SSE token converter ---------------------------------------------------------------------
// For a token "d+" or "d+.d+" of length L <= 16 (sign already stripped): one pshufb removes the dot
// and right-aligns the digits into 16 lanes, pmaddubsw/pmaddwd fold them into two 8-digit halves.
// The shuffle masks depend only on (L, dot position) and are built once.
struct ShufTable {
  alignas(16) uint8_t m[17][17][16];  // [L][dot index or 16 = none][lane]
  ShufTable() {
    for (int L = 0; L <= 16; ++L)
      for (int d = 0; d <= 16; ++d) {
        // source positions of the digits, in order
        int src[16], n = 0;
        for (int i = 0; i < L && i < 16; ++i)
          if (i != d) src[n++] = i;
        for (int k = 0; k < 16; ++k) {
          const int from_right = 15 - k;  // lane k holds the digit `from_right` places from the end
          m[L][d][k] = from_right < n ? static_cast<uint8_t>(src[n - 1 - from_right]) : 0x80;  // 0x80 -> zero
        }
      }
  }
};
const ShufTable kShuf;

// Returns false (caller falls back) for anything but plain decimal digits with at most one dot.
inline bool parse_token_sse(const char* b, long len, float& out, bool neg) {
  const __m128i raw = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b));
  const __m128i dotm = _mm_cmpeq_epi8(raw, _mm_set1_epi8('.'));
  const uint32_t lenmask = (1u << len) - 1u;
  const uint32_t dots = static_cast<uint32_t>(_mm_movemask_epi8(dotm)) & lenmask;
  const __m128i dig = _mm_sub_epi8(raw, _mm_set1_epi8('0'));
  // digit lanes: (unsigned) dig <= 9
  const __m128i isdig = _mm_cmpeq_epi8(_mm_min_epu8(dig, _mm_set1_epi8(9)), dig);
  const uint32_t digs = static_cast<uint32_t>(_mm_movemask_epi8(isdig)) & lenmask;
  if ((digs | dots) != lenmask || (dots & (dots - 1))) return false;  // bad char or >1 dot
  const int d = dots ? __builtin_ctz(dots) : 16;
  const int ndig = static_cast<int>(len) - (dots ? 1 : 0);
  if (d == 0 || d == len - 1) return false;  // ".5" / "5." are not JSON
  if (b[0] == '0' && (d == 16 ? len > 1 : d > 1)) return false;  // leading zero
  const int frac = dots ? static_cast<int>(len) - 1 - d : 0;
  if (ndig > 16 || frac > 10) return false;
  const __m128i aligned = _mm_shuffle_epi8(dig, _mm_load_si128(reinterpret_cast<const __m128i*>(kShuf.m[len][d])));
  // pairs -> 2-digit, quads -> 4-digit, octets -> 8-digit values
  const __m128i t1 = _mm_maddubs_epi16(aligned, _mm_setr_epi8(10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1, 10, 1));
  const __m128i t2 = _mm_madd_epi16(t1, _mm_setr_epi16(100, 1, 100, 1, 100, 1, 100, 1));
  const __m128i t3 = _mm_packus_epi32(t2, t2);
  const __m128i t4 = _mm_madd_epi16(t3, _mm_setr_epi16(10000, 1, 10000, 1, 10000, 1, 10000, 1));
  const uint64_t hi = static_cast<uint32_t>(_mm_cvtsi128_si32(t4));
  const uint64_t lo = static_cast<uint32_t>(_mm_extract_epi32(t4, 1));
  const uint64_t mant = hi * 100000000ull + lo;
  float v;
  if (mant <= (1u << 24) && frac <= 10) {
    v = static_cast<float>(static_cast<uint32_t>(mant)) / kPow10f[frac];
  } else {
    if (mant > (1ull << 53)) return false;
    const double dv = static_cast<double>(mant) / kPow10[frac];
    uint64_t bits;
    std::memcpy(&bits, &dv, sizeof bits);
    if ((bits & ((1ull << 29) - 1)) == (1ull << 28)) return false;
    v = static_cast<float>(dv);
  }
  uint32_t vb;
  std::memcpy(&vb, &v, 4);
  vb |= static_cast<uint32_t>(neg) << 31;
  std::memcpy(&out, &vb, 4);
  return true;
}

// Parse one token [b, e) known to be delimited by separators (no whitespace inside).  Independent
// of every other token, so consecutive calls overlap in the out-of-order core.
bool g_token_simd = true;  // A/B switch for benchmarks (set_json_simd)

// mantissa (<= 16 digits) and fraction digits -> float with the same rounding rules as above.
inline bool finish_float(uint64_t mant, int frac, bool neg, float& out) {
  float v;
  if (mant <= (1u << 24)) {
    v = static_cast<float>(static_cast<uint32_t>(mant)) / kPow10f[frac];
  } else {
    if (mant > (1ull << 53)) return false;
    const double dv = static_cast<double>(mant) / kPow10[frac];
    uint64_t bits;
    std::memcpy(&bits, &dv, sizeof bits);
    if ((bits & ((1ull << 29) - 1)) == (1ull << 28)) return false;
    v = static_cast<float>(dv);
  }
  uint32_t vb;
  std::memcpy(&vb, &v, 4);
  vb |= static_cast<uint32_t>(neg) << 31;
  std::memcpy(&out, &vb, 4);
  return true;
}

// Two tokens per AVX2 pass: pshufb / maddubs / madd work within 128-bit lanes, so lane 0 converts
// token a and lane 1 token b with the same instruction stream (the per-token work of
// parse_token_sse at half the instructions).  Tokens are sign-stripped, 1..16 chars.
inline bool parse_token_pair_avx2(const char* a, long la, bool na, const char* b, long lb, bool nb, float& oa,
                                  float& ob) {
  const __m256i raw = _mm256_loadu2_m128i(reinterpret_cast<const __m128i*>(b), reinterpret_cast<const __m128i*>(a));
  const uint32_t lenmask = ((1u << la) - 1u) | (((1u << lb) - 1u) << 16);
  const uint32_t dots = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(raw, _mm256_set1_epi8('.')))) & lenmask;
  const __m256i dig = _mm256_sub_epi8(raw, _mm256_set1_epi8('0'));
  const __m256i isdig = _mm256_cmpeq_epi8(_mm256_min_epu8(dig, _mm256_set1_epi8(9)), dig);
  const uint32_t digs = static_cast<uint32_t>(_mm256_movemask_epi8(isdig)) & lenmask;
  const uint32_t da = dots & 0xFFFFu, db = dots >> 16;
  if ((digs | dots) != lenmask || (da & (da - 1)) || (db & (db - 1))) return false;
  const int pa = da ? __builtin_ctz(da) : 16, pb = db ? __builtin_ctz(db) : 16;
  if (pa == 0 || pb == 0 || (da && pa == la - 1) || (db && pb == lb - 1)) return false;
  if ((a[0] == '0' && (da ? pa > 1 : la > 1)) || (b[0] == '0' && (db ? pb > 1 : lb > 1))) return false;
  const int fa = da ? static_cast<int>(la) - 1 - pa : 0, fb = db ? static_cast<int>(lb) - 1 - pb : 0;
  if (fa > 10 || fb > 10) return false;
  const __m256i shuf = _mm256_loadu2_m128i(reinterpret_cast<const __m128i*>(kShuf.m[lb][pb]),
                                           reinterpret_cast<const __m128i*>(kShuf.m[la][pa]));
  const __m256i aligned = _mm256_shuffle_epi8(dig, shuf);
  const __m256i t1 = _mm256_maddubs_epi16(aligned, _mm256_set1_epi16(0x010A));  // bytes (10, 1)
  const __m256i t2 = _mm256_madd_epi16(t1, _mm256_set1_epi32(0x00010064));      // words (100, 1)
  const __m256i t3 = _mm256_packus_epi32(t2, t2);
  const __m256i t4 = _mm256_madd_epi16(t3, _mm256_set1_epi32(0x00012710));      // words (10000, 1)
  const uint64_t ma = static_cast<uint64_t>(static_cast<uint32_t>(_mm256_extract_epi32(t4, 0))) * 100000000ull +
                      static_cast<uint32_t>(_mm256_extract_epi32(t4, 1));
  const uint64_t mb = static_cast<uint64_t>(static_cast<uint32_t>(_mm256_extract_epi32(t4, 4))) * 100000000ull +
                      static_cast<uint32_t>(_mm256_extract_epi32(t4, 5));
  return finish_float(ma, fa, na, oa) && finish_float(mb, fb, nb, ob);
}

inline bool parse_token(const char* b, const char* e, float& out) {
  if (g_token_simd) {
    const bool neg = *b == '-';
    const long len = e - b - neg;
    if (len > 0 && len <= 16 && parse_token_sse(b + neg, len, out, neg)) return true;
  }
  const bool neg = *b == '-';
  b += neg;
  const long len = e - b;
  if (len <= 0 || len > 17) return false;
  const uint64_t vi = load8(b);
  int ki = leading_digits(vi);
  if (ki > len) ki = static_cast<int>(len);
  if (ki == 0 || ki == 8) return false;
  if (ki > 1 && *b == '0') return false;
  uint64_t mant = swar_digits(vi, ki);
  int exp10 = 0;
  if (ki != len) {
    if (b[ki] != '.') return false;
    const int kf = static_cast<int>(len) - ki - 1;
    if (kf <= 0 || kf > 8) return false;
    const uint64_t vf = load8(b + ki + 1);
    if (leading_digits(vf) < kf) return false;
    mant = mant * kPow10u[kf] + swar_digits(vf, kf);
    exp10 = -kf;
  }
  float v;
  if (mant <= (1u << 24)) {
    v = static_cast<float>(mant) / kPow10f[-exp10];
  } else {
    const double d = static_cast<double>(mant) / kPow10[-exp10];
    uint64_t bits;
    std::memcpy(&bits, &d, sizeof bits);
    if ((bits & ((1ull << 29) - 1)) == (1ull << 28)) return false;
    v = static_cast<float>(d);
  }
  // Branch-free sign: random signs would otherwise mispredict half the time.
  uint32_t bits;
  std::memcpy(&bits, &v, 4);
  bits |= static_cast<uint32_t>(neg) << 31;
  std::memcpy(&out, &bits, 4);
  return true;
}

// 64-bit masks of ',' and ']' in the 64 bytes at p (SSE2).
inline void sep_masks(const char* p, uint64_t& comma, uint64_t& close) {
  const __m128i c1 = _mm_set1_epi8(',');
  const __m128i c2 = _mm_set1_epi8(']');
  comma = 0;
  close = 0;
  for (int i = 0; i < 4; ++i) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * i));
    comma |= static_cast<uint64_t>(static_cast<uint32_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(v, c1)))) << (16 * i);
    close |= static_cast<uint64_t>(static_cast<uint32_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(v, c2)))) << (16 * i);
  }
}

// Bulk path for the body of a float array starting right after '['.  Consumes whole tokens while
// they are "simple" and complete 64-byte blocks are available; returns the position of the first
// unconsumed byte (the start of a token, or one past the closing ']' when *done is set).
inline const char* bulk_float_array(const char* p, const char* end, float* dst, size_t cap, size_t& n,
                                    bool& done) {
  done = false;
  const char* tok = p;
  const char* base = p;
  while (end - base >= 64 + 24) {  // 24 bytes of slack so token loads stay in bounds
    uint64_t comma, close;
    sep_masks(base, comma, close);
    uint64_t m = comma | close;
    while (m) {
      const uint64_t m2 = m & (m - 1);
      if (m2 && g_token_simd && !((close >> __builtin_ctzll(m)) & 1)) {
        // two complete tokens in this block: convert them together
        const char* sep1 = base + __builtin_ctzll(m);
        const char* sep2 = base + __builtin_ctzll(m2);
        const char* t2 = sep1 + 1;
        const bool n1 = *tok == '-', n2 = *t2 == '-';
        const long l1 = sep1 - tok - n1, l2 = sep2 - t2 - n2;
        float f1, f2;
        if (l1 > 0 && l1 <= 16 && l2 > 0 && l2 <= 16 &&
            parse_token_pair_avx2(tok + n1, l1, n1, t2 + n2, l2, n2, f1, f2)) {
          if (n < cap) dst[n] = f1;
          if (n + 1 < cap) dst[n + 1] = f2;
          n += 2;
          tok = sep2 + 1;
          if ((close >> (sep2 - base)) & 1) {
            done = true;
            return tok;
          }
          m = m2 & (m2 - 1);
          continue;
        }
      }
      const int s = __builtin_ctzll(m);
      const char* sep = base + s;
      float v;
      if (sep == tok || !parse_token(tok, sep, v)) return tok;  // let the strict path decide
      if (n < cap) dst[n] = v;
      ++n;
      tok = sep + 1;
      if ((close >> s) & 1) {
        done = true;
        return tok;
      }
      m &= m - 1;
    }
    base += 64;
  }
  return tok;
}

Json parse_value(Cursor& c, int depth);

Json parse_number(Cursor& c) {
  NumScan s;
  const char* p = c.p;
  if (!scan_number(p, c.end, s)) c.fail("invalid number");
  c.p = p;
  if (s.is_int && !s.truncated && s.mant <= static_cast<uint64_t>(INT64_MAX)) {
    int64_t v = static_cast<int64_t>(s.mant);
    return Json(static_cast<long long>(s.neg ? -v : v));
  }
  return Json(slow_double(s.start, s.stop));
}

Json parse_value(Cursor& c, int depth) {
  if (depth > 512) c.fail("nesting too deep");
  char ch = c.peek();
  switch (ch) {
    case '{': {
      ++c.p;
      Json obj = Json::object();
      if (c.peek() == '}') {
        ++c.p;
        return obj;
      }
      while (true) {
        std::string key = parse_string(c);
        c.expect(':');
        obj[key] = parse_value(c, depth + 1);
        char n = c.peek();
        if (n == ',') {
          ++c.p;
          continue;
        }
        if (n == '}') {
          ++c.p;
          return obj;
        }
        c.fail("expected ',' or '}'");
      }
    }
    case '[': {
      ++c.p;
      Json arr = Json::array();
      if (c.peek() == ']') {
        ++c.p;
        return arr;
      }
      while (true) {
        arr.push_back(parse_value(c, depth + 1));
        char n = c.peek();
        if (n == ',') {
          ++c.p;
          continue;
        }
        if (n == ']') {
          ++c.p;
          return arr;
        }
        c.fail("expected ',' or ']'");
      }
    }
    case '"': return Json(parse_string(c));
    case 't':
      if (c.end - c.p >= 4 && std::memcmp(c.p, "true", 4) == 0) {
        c.p += 4;
        return Json(true);
      }
      c.fail("invalid literal");
    case 'f':
      if (c.end - c.p >= 5 && std::memcmp(c.p, "false", 5) == 0) {
        c.p += 5;
        return Json(false);
      }
      c.fail("invalid literal");
    case 'n':
      if (c.end - c.p >= 4 && std::memcmp(c.p, "null", 4) == 0) {
        c.p += 4;
        return Json();
      }
      c.fail("invalid literal");
    default:
      if (ch == '-' || (ch >= '0' && ch <= '9')) return parse_number(c);
      c.fail("invalid literal");
  }
}

void skip_value(Cursor& c, int depth) {
  if (depth > 512) c.fail("nesting too deep");
  char ch = c.peek();
  if (ch == '"') {
    skip_string(c);
    return;
  }
  if (ch == '{' || ch == '[') {
    char close = ch == '{' ? '}' : ']';
    ++c.p;
    if (c.peek() == close) {
      ++c.p;
      return;
    }
    while (true) {
      if (ch == '{') {
        skip_string(c);
        c.expect(':');
      }
      skip_value(c, depth + 1);
      char n = c.peek();
      if (n == ',') {
        ++c.p;
        continue;
      }
      if (n == close) {
        ++c.p;
        return;
      }
      c.fail("expected separator");
    }
  }
  if (ch == '-' || (ch >= '0' && ch <= '9')) {
    NumScan s;
    const char* p = c.p;
    if (!scan_number(p, c.end, s)) c.fail("invalid number");
    c.p = p;
    return;
  }
  parse_value(c, depth);  // literals
}

}  // namespace

Json Json::parse(std::string_view text) {
  Cursor c{text.data(), text.data() + text.size(), text.data()};
  Json v = parse_value(c, 0);
  c.ws();
  if (c.p != c.end) c.fail("unexpected trailing characters");
  return v;
}

bool parse_json_float(const char*& p, const char* end, float& out) {
  if (fast_simple_float(p, end, out)) return true;
  NumScan s;
  if (!scan_number(p, end, s)) return false;
  out = scan_to_float(s);
  return true;
}

int parse_infer_body(std::string_view body, InferBodySink& sink) {
  Cursor c{body.data(), body.data() + body.size(), body.data()};
  int seen = 0;
  c.expect('{');
  if (c.peek() == '}') {
    ++c.p;
  } else {
    while (true) {
      std::string key = parse_string(c);
      c.expect(':');
      if (key == "input_data") {
        if (c.peek() != '[') throw JsonError("[json.exception.type_error.302] type must be array, but is " +
                                             std::string(c.peek() == '"' ? "string" : "other"));
        ++c.p;
        if (sink.defer_input_text()) {
          const char* q = static_cast<const char*>(std::memchr(c.p, ']', static_cast<size_t>(c.end - c.p)));
          if (!q) c.fail("unexpected end of input; expected ']'");
          sink.on_input_text(c.p, static_cast<size_t>(q - c.p));
          c.p = q + 1;
          seen |= 2 | 4;
          goto next_member;
        }
        float* dst = sink.input_buffer();
        const size_t cap = sink.input_capacity();
        size_t n = 0;
        c.ws();
        if (c.p < c.end && *c.p == ']') {
          ++c.p;
        } else {
          const char* p = c.p;
          const char* end = c.end;
          bool done = false;
          p = bulk_float_array(p, end, dst, cap, n, done);
          while (!done) {
            while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
            float fv;
            if (fast_simple_float(p, end, fv)) {
              if (n < cap) dst[n] = fv;
              ++n;
              if (*p == ',') {
                ++p;
                continue;
              }
              while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
              if (p < end && *p == ',') {
                ++p;
                continue;
              }
              if (p < end && *p == ']') {
                ++p;
                break;
              }
              c.p = p;
              c.fail("expected ',' or ']'");
            }
            NumScan s;
            const char* q = p;
            if (!scan_number(q, end, s)) {
              c.p = p;
              if (p < end && (*p == '"' || *p == 't' || *p == 'f' || *p == 'n' || *p == '[' || *p == '{'))
                throw JsonError("[json.exception.type_error.302] type must be number");
              c.fail("invalid number in input_data");
            }
            if (n < cap) dst[n] = scan_to_float(s);
            ++n;
            p = q;
            while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
            if (p >= end) {
              c.p = p;
              c.fail("unexpected end of input");
            }
            if (*p == ',') {
              ++p;
              continue;
            }
            if (*p == ']') {
              ++p;
              break;
            }
            c.p = p;
            c.fail("expected ',' or ']'");
          }
          c.p = p;
        }
        sink.on_input_count(n);
        seen |= 2;
      } else if (key == "request_id") {
        if (c.peek() != '"') throw JsonError("[json.exception.type_error.302] type must be string");
        std::string id = parse_string(c);
        sink.on_request_id(id);
        seen |= 1;
      } else {
        Json v = parse_value(c, 1);
        sink.on_other_key(key, v);
      }
    next_member:
      char n = c.peek();
      if (n == ',') {
        ++c.p;
        continue;
      }
      if (n == '}') {
        ++c.p;
        break;
      }
      c.fail("expected ',' or '}'");
    }
  }
  c.ws();
  if (c.p != c.end) c.fail("unexpected trailing characters");
  return seen;
}

bool find_top_level_string(std::string_view body, std::string_view key, std::string& out) {
  try {
    Cursor c{body.data(), body.data() + body.size(), body.data()};
    c.expect('{');
    if (c.peek() == '}') return false;
    while (true) {
      std::string k = parse_string(c);
      c.expect(':');
      if (k == key) {
        if (c.peek() != '"') return false;
        out = parse_string(c);
        return true;
      }
      skip_value(c, 1);
      char n = c.peek();
      if (n == ',') {
        ++c.p;
        continue;
      }
      return false;
    }
  } catch (const JsonError&) {
    return false;
  }
}

}  // namespace die

namespace die {
void set_json_simd(bool on) { g_token_simd = on; }
}  // namespace die
