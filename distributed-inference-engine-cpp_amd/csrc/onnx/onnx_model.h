// ONNX model IR and an in-tree protobuf wire-format reader.
//
// The reference hands the .onnx path to ONNX Runtime (src/inference_engine.cpp:31) and only reads
// back input/output 0 (:35-69).  No onnx/protoc is available offline, so the ModelProto is decoded
// here directly from the wire format (varint / fixed32 / fixed64 / length-delimited fields).
// Supported: IR v3+ (initializers listed as graph inputs or not), raw_data and typed *_data
// fields, Constant nodes, dynamic dims (dim_param).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace die {
namespace onnx {

enum DataType : int {
  UNDEFINED = 0, FLOAT = 1, UINT8 = 2, INT8 = 3, UINT16 = 4, INT16 = 5, INT32 = 6, INT64 = 7,
  STRING = 8, BOOL = 9, FLOAT16 = 10, DOUBLE = 11, UINT32 = 12, UINT64 = 13, BFLOAT16 = 16
};

inline bool is_float_type(int t) { return t == FLOAT || t == FLOAT16 || t == DOUBLE || t == BFLOAT16; }

// Host tensor.  Float-like element types are widened to f32 in `f`; integer/bool types to int64 in
// `i`.  Exactly one of the two vectors is populated.
struct Tensor {
  std::string name;
  int dtype = FLOAT;
  std::vector<int64_t> dims;
  std::vector<float> f;
  std::vector<int64_t> i;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
};

struct Attribute {
  enum Type { UNDEF = 0, FLOAT_ = 1, INT_ = 2, STRING_ = 3, TENSOR_ = 4, GRAPH_ = 5, FLOATS = 6, INTS = 7, STRINGS = 8 };
  std::string name;
  int type = UNDEF;
  float f = 0.f;
  int64_t i = 0;
  std::string s;
  std::vector<float> floats;
  std::vector<int64_t> ints;
  std::vector<std::string> strings;
  std::shared_ptr<Tensor> t;
};

struct Node {
  std::string name, op_type, domain;
  std::vector<std::string> inputs, outputs;
  std::map<std::string, Attribute> attrs;

  bool has(const std::string& k) const { return attrs.count(k) != 0; }
  int64_t get_int(const std::string& k, int64_t d) const;
  float get_float(const std::string& k, float d) const;
  std::string get_string(const std::string& k, const std::string& d) const;
  std::vector<int64_t> get_ints(const std::string& k, const std::vector<int64_t>& d = {}) const;
  std::vector<float> get_floats(const std::string& k, const std::vector<float>& d = {}) const;
  // Input i or "" when absent/optional.
  const std::string& in(size_t i) const;
};

struct ValueInfo {
  std::string name;
  int elem_type = FLOAT;
  std::vector<int64_t> dims;          // -1 for a symbolic/unknown dim
  std::vector<std::string> dim_params;
};

struct Model {
  int64_t ir_version = 0;
  std::vector<std::pair<std::string, int64_t>> opsets;
  std::string producer_name, graph_name;
  std::vector<Node> nodes;                               // topologically sorted on load
  std::unordered_map<std::string, Tensor> initializers;  // includes Constant node outputs
  std::vector<ValueInfo> inputs;                         // real inputs (initializers removed)
  std::vector<ValueInfo> outputs;
  std::unordered_map<std::string, ValueInfo> value_info;

  int64_t opset(const std::string& domain = "") const;
  size_t param_bytes_f32() const;
};

class OnnxError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

Model load_onnx(const std::string& path);
Model parse_onnx(const uint8_t* data, size_t size);

}  // namespace onnx
}  // namespace die
