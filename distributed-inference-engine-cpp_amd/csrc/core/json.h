// Minimal JSON DOM + fast float-array paths for the /infer hot path.
//
// The reference uses nlohmann::json for everything (src/worker_node.cpp:54,176,179;
// src/gateway.cpp:107,178,181).  That parses every float of `input_data` into a DOM node and
// prints floats as 17-significant-digit doubles.  Here the DOM is only used for small control
// documents (/health, /stats, errors); request bodies go through `parse_infer_body`, which
// writes the floats straight into caller memory (pinned staging), and responses go through
// `append_float_array`, which prints the shortest string that round-trips the float32.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace die {

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type { Null, Bool, Int, Float, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::vector<std::pair<std::string, Json>>;  // insertion ordered

  Json() = default;
  Json(std::nullptr_t) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(long v) : type_(Type::Int), i_(v) {}
  Json(long long v) : type_(Type::Int), i_(v) {}
  Json(unsigned v) : type_(Type::Int), i_(v) {}
  Json(unsigned long v) : type_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(unsigned long long v) : type_(Type::Int), i_(static_cast<int64_t>(v)) {}
  Json(double v) : type_(Type::Float), d_(v) {}
  Json(float v) : type_(Type::Float), d_(v), is_f32_(true) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Json(std::string_view s) : type_(Type::String), s_(s) {}
  Json(const std::vector<float>& v);

  static Json array() { Json j; j.type_ = Type::Array; return j; }
  static Json object() { Json j; j.type_ = Type::Object; return j; }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Float; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_int() const;
  double as_double() const;
  const std::string& as_string() const;
  const Array& as_array() const;
  Array& as_array();
  const Object& as_object() const;

  // Object access.  operator[] on a non-const object inserts; `at` throws on a missing key
  // (the reference's const operator[] on a missing key is UB: SURVEY §5.2).
  Json& operator[](const std::string& key);
  const Json& at(const std::string& key) const;
  const Json* find(const std::string& key) const;
  bool contains(const std::string& key) const { return find(key) != nullptr; }
  // Array access.
  void push_back(Json v);
  const Json& operator[](size_t i) const;
  size_t size() const;

  std::string dump() const;
  void dump_to(std::string& out) const;
  static Json parse(std::string_view text);

 private:
  Type type_ = Type::Null;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0.0;
  bool is_f32_ = false;
  std::string s_;
  Array a_;
  Object o_;
};

// ---- fast paths --------------------------------------------------------------------------------

// Append `"..."` with JSON escaping.
void append_json_string(std::string& out, std::string_view s);
// Append `[v0,v1,...]` using the shortest float32 round-trip representation; non-finite -> null
// (nlohmann prints NaN/inf as null too).
void append_float_array(std::string& out, const float* v, size_t n);

// Parse one JSON number at `p` as float32 (correctly rounded).  Advances p.  Returns false on
// malformed input.
bool parse_json_float(const char*& p, const char* end, float& out);

// Receives the fields of a /infer body.  `floats(n_hint)` must return a buffer with room for at
// least `cap` floats; the parser writes values there and calls `float_count(n)` at the end.
struct InferBodySink {
  virtual ~InferBodySink() = default;
  virtual void on_request_id(std::string_view id) = 0;
  // Destination for input_data; the parser never writes more than `capacity()` values.
  virtual float* input_buffer() = 0;
  virtual size_t input_capacity() const = 0;
  virtual void on_input_count(size_t n) = 0;  // n may exceed capacity (values beyond are dropped)
  virtual void on_other_key(std::string_view key, const Json& value) { (void)key; (void)value; }
  // Device decode: when true, input_data is not converted here; its raw text (between '[' and the
  // first ']') goes to on_input_text and the engine converts it (malformed tokens are caught there).
  virtual bool defer_input_text() const { return false; }
  virtual void on_input_text(const char* b, size_t n) { (void)b; (void)n; }
};

// Parse a top-level object {"request_id": str, "input_data": [numbers...], ...}.  Throws JsonError
// (message mirrors nlohmann's where it matters) on malformed JSON or wrong types.  Returns a bit
// mask: 1 = request_id seen, 2 = input_data seen, 4 = input_data deferred as text.
int parse_infer_body(std::string_view body, InferBodySink& sink);

// Locate the top-level string member `key` without building a DOM (gateway routing).  Values of
// other members are skipped.  Returns false if the key is absent or not a string.
bool find_top_level_string(std::string_view body, std::string_view key, std::string& out);

// Benchmark switch: false disables the SSE token converter (scalar SWAR path only).
void set_json_simd(bool on);

}  // namespace die
