#include "onnx_model.h"

#include <cstring>
#include <fstream>
#include <queue>
#include <unordered_set>

namespace die {
namespace onnx {

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* end;

  bool eof() const { return p >= end; }
  [[noreturn]] static void fail(const char* m) { throw OnnxError(std::string("onnx protobuf: ") + m); }
  uint64_t varint() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end) fail("truncated varint");
      uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7F) << shift;
      if (!(b & 0x80)) return v;
      shift += 7;
      if (shift > 63) fail("varint too long");
    }
  }
  uint32_t fixed32() {
    if (end - p < 4) fail("truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (end - p < 8) fail("truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  Reader sub() {
    uint64_t n = varint();
    if (static_cast<uint64_t>(end - p) < n) fail("truncated length-delimited field");
    Reader r{p, p + n};
    p += n;
    return r;
  }
  std::string str() {
    Reader r = sub();
    return std::string(reinterpret_cast<const char*>(r.p), r.end - r.p);
  }
  bool next(uint32_t& field, uint32_t& wt) {
    if (eof()) return false;
    uint64_t key = varint();
    field = static_cast<uint32_t>(key >> 3);
    wt = static_cast<uint32_t>(key & 7);
    return true;
  }
  void skip(uint32_t wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: fixed64(); break;
      case 2: sub(); break;
      case 5: fixed32(); break;
      default: fail("unsupported wire type");
    }
  }
};

// Repeated scalar fields may be packed (wt 2) or not.
void read_int64s(Reader& r, uint32_t wt, std::vector<int64_t>& out) {
  if (wt == 2) {
    Reader s = r.sub();
    while (!s.eof()) out.push_back(static_cast<int64_t>(s.varint()));
  } else {
    out.push_back(static_cast<int64_t>(r.varint()));
  }
}
void read_floats(Reader& r, uint32_t wt, std::vector<float>& out) {
  auto one = [&](Reader& s) {
    uint32_t b = s.fixed32();
    float f;
    std::memcpy(&f, &b, 4);
    out.push_back(f);
  };
  if (wt == 2) {
    Reader s = r.sub();
    while (!s.eof()) one(s);
  } else {
    one(r);
  }
}
void read_doubles(Reader& r, uint32_t wt, std::vector<double>& out) {
  auto one = [&](Reader& s) {
    uint64_t b = s.fixed64();
    double d;
    std::memcpy(&d, &b, 8);
    out.push_back(d);
  };
  if (wt == 2) {
    Reader s = r.sub();
    while (!s.eof()) one(s);
  } else {
    one(r);
  }
}

float half_to_float(uint16_t h) {
  uint32_t sign = (h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1F;
  uint32_t mant = h & 0x3FF;
  uint32_t bits;
  if (exp == 0) {
    if (mant == 0) {
      bits = sign;
    } else {
      int e = -1;
      do {
        ++e;
        mant <<= 1;
      } while (!(mant & 0x400));
      bits = sign | static_cast<uint32_t>(127 - 15 - e) << 23 | (mant & 0x3FF) << 13;
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (mant << 13);
  } else {
    bits = sign | (exp - 15 + 127) << 23 | (mant << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

float bf16_to_float(uint16_t h) {
  uint32_t bits = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

Tensor parse_tensor(Reader r) {
  Tensor t;
  std::vector<float> float_data;
  std::vector<int64_t> int32_data, int64_data;
  std::vector<double> double_data;
  const uint8_t* raw = nullptr;
  size_t raw_n = 0;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    switch (f) {
      case 1: read_int64s(r, wt, t.dims); break;
      case 2: t.dtype = static_cast<int>(r.varint()); break;
      case 4: read_floats(r, wt, float_data); break;
      case 5: read_int64s(r, wt, int32_data); break;
      case 7: read_int64s(r, wt, int64_data); break;
      case 8: t.name = r.str(); break;
      case 9: {
        Reader s = r.sub();
        raw = s.p;
        raw_n = s.end - s.p;
        break;
      }
      case 10: read_doubles(r, wt, double_data); break;
      case 11: read_int64s(r, wt, int64_data); break;  // uint64_data
      case 14:
        if (r.varint() == 1) throw OnnxError("external tensor data is not supported (tensor " + t.name + ")");
        break;
      default: r.skip(wt);
    }
  }
  const int64_t n = t.numel();
  auto need = [&](size_t have) {
    if (static_cast<int64_t>(have) != n)
      throw OnnxError("tensor " + t.name + ": expected " + std::to_string(n) + " elements, got " + std::to_string(have));
  };
  switch (t.dtype) {
    case FLOAT:
      if (raw) {
        need(raw_n / 4);
        t.f.resize(n);
        std::memcpy(t.f.data(), raw, n * 4);
      } else {
        need(float_data.size());
        t.f = std::move(float_data);
      }
      break;
    case DOUBLE:
      if (raw) {
        need(raw_n / 8);
        t.f.resize(n);
        for (int64_t k = 0; k < n; ++k) {
          double d;
          std::memcpy(&d, raw + 8 * k, 8);
          t.f[k] = static_cast<float>(d);
        }
      } else {
        need(double_data.size());
        t.f.assign(double_data.begin(), double_data.end());
      }
      break;
    case FLOAT16:
    case BFLOAT16: {
      t.f.resize(n);
      if (raw) {
        need(raw_n / 2);
        for (int64_t k = 0; k < n; ++k) {
          uint16_t h;
          std::memcpy(&h, raw + 2 * k, 2);
          t.f[k] = t.dtype == FLOAT16 ? half_to_float(h) : bf16_to_float(h);
        }
      } else {
        need(int32_data.size());
        for (int64_t k = 0; k < n; ++k) {
          uint16_t h = static_cast<uint16_t>(int32_data[k]);
          t.f[k] = t.dtype == FLOAT16 ? half_to_float(h) : bf16_to_float(h);
        }
      }
      break;
    }
    case INT64:
    case UINT64:
      if (raw) {
        need(raw_n / 8);
        t.i.resize(n);
        std::memcpy(t.i.data(), raw, n * 8);
      } else {
        need(int64_data.size());
        t.i = std::move(int64_data);
      }
      break;
    case INT32:
    case INT16:
    case INT8:
    case UINT8:
    case UINT16:
    case BOOL:
    case UINT32: {
      if (raw) {
        size_t es = (t.dtype == INT32 || t.dtype == UINT32) ? 4 : (t.dtype == INT16 || t.dtype == UINT16) ? 2 : 1;
        need(raw_n / es);
        t.i.resize(n);
        for (int64_t k = 0; k < n; ++k) {
          const uint8_t* q = raw + es * k;
          int64_t v = 0;
          switch (t.dtype) {
            case INT32: { int32_t x; std::memcpy(&x, q, 4); v = x; break; }
            case UINT32: { uint32_t x; std::memcpy(&x, q, 4); v = x; break; }
            case INT16: { int16_t x; std::memcpy(&x, q, 2); v = x; break; }
            case UINT16: { uint16_t x; std::memcpy(&x, q, 2); v = x; break; }
            case INT8: v = static_cast<int8_t>(*q); break;
            default: v = *q; break;
          }
          t.i[k] = v;
        }
      } else {
        need(int32_data.size());
        t.i = std::move(int32_data);
      }
      break;
    }
    default:
      throw OnnxError("tensor " + t.name + ": unsupported data type " + std::to_string(t.dtype));
  }
  return t;
}

ValueInfo parse_value_info(Reader r) {
  ValueInfo vi;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    if (f == 1) {
      vi.name = r.str();
    } else if (f == 2) {  // TypeProto
      Reader tp = r.sub();
      uint32_t f2, w2;
      while (tp.next(f2, w2)) {
        if (f2 != 1) {
          tp.skip(w2);
          continue;
        }
        Reader tt = tp.sub();  // TypeProto.Tensor
        uint32_t f3, w3;
        while (tt.next(f3, w3)) {
          if (f3 == 1) {
            vi.elem_type = static_cast<int>(tt.varint());
          } else if (f3 == 2) {
            Reader sh = tt.sub();
            uint32_t f4, w4;
            while (sh.next(f4, w4)) {
              if (f4 != 1) {
                sh.skip(w4);
                continue;
              }
              Reader dim = sh.sub();
              int64_t dv = -1;
              std::string dp;
              uint32_t f5, w5;
              while (dim.next(f5, w5)) {
                if (f5 == 1) dv = static_cast<int64_t>(dim.varint());
                else if (f5 == 2) dp = dim.str();
                else dim.skip(w5);
              }
              vi.dims.push_back(dv);
              vi.dim_params.push_back(dp);
            }
          } else {
            tt.skip(w3);
          }
        }
      }
    } else {
      r.skip(wt);
    }
  }
  return vi;
}

Attribute parse_attribute(Reader r) {
  Attribute a;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    switch (f) {
      case 1: a.name = r.str(); break;
      case 2: {
        uint32_t b = r.fixed32();
        std::memcpy(&a.f, &b, 4);
        break;
      }
      case 3: a.i = static_cast<int64_t>(r.varint()); break;
      case 4: a.s = r.str(); break;
      case 5: a.t = std::make_shared<Tensor>(parse_tensor(r.sub())); break;
      case 7: read_floats(r, wt, a.floats); break;
      case 8: read_int64s(r, wt, a.ints); break;
      case 9: a.strings.push_back(r.str()); break;
      case 20: a.type = static_cast<int>(r.varint()); break;
      default: r.skip(wt);
    }
  }
  if (a.type == Attribute::UNDEF) {  // very old files: infer from content
    if (a.t) a.type = Attribute::TENSOR_;
    else if (!a.ints.empty()) a.type = Attribute::INTS;
    else if (!a.floats.empty()) a.type = Attribute::FLOATS;
    else if (!a.s.empty()) a.type = Attribute::STRING_;
  }
  return a;
}

Node parse_node(Reader r) {
  Node n;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    switch (f) {
      case 1: n.inputs.push_back(r.str()); break;
      case 2: n.outputs.push_back(r.str()); break;
      case 3: n.name = r.str(); break;
      case 4: n.op_type = r.str(); break;
      case 5: {
        Attribute a = parse_attribute(r.sub());
        n.attrs[a.name] = std::move(a);
        break;
      }
      case 7: n.domain = r.str(); break;
      default: r.skip(wt);
    }
  }
  return n;
}

void parse_graph(Reader r, Model& m) {
  std::vector<ValueInfo> inputs;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    switch (f) {
      case 1: m.nodes.push_back(parse_node(r.sub())); break;
      case 2: m.graph_name = r.str(); break;
      case 5: {
        Tensor t = parse_tensor(r.sub());
        std::string name = t.name;
        m.initializers.emplace(name, std::move(t));
        break;
      }
      case 11: inputs.push_back(parse_value_info(r.sub())); break;
      case 12: m.outputs.push_back(parse_value_info(r.sub())); break;
      case 13: {
        ValueInfo vi = parse_value_info(r.sub());
        m.value_info[vi.name] = vi;
        break;
      }
      default: r.skip(wt);
    }
  }
  for (auto& vi : inputs)
    if (!m.initializers.count(vi.name)) m.inputs.push_back(vi);
}

void toposort_and_fold_constants(Model& m) {
  // Constant nodes become initializers.
  std::vector<Node> rest;
  for (auto& n : m.nodes) {
    if (n.op_type == "Constant" && n.outputs.size() == 1) {
      Tensor t;
      if (n.has("value") && n.attrs.at("value").t) {
        t = *n.attrs.at("value").t;
      } else if (n.has("value_float")) {
        t.dtype = FLOAT;
        t.f = {n.get_float("value_float", 0.f)};
      } else if (n.has("value_floats")) {
        t.dtype = FLOAT;
        t.f = n.attrs.at("value_floats").floats;
        t.dims = {static_cast<int64_t>(t.f.size())};
      } else if (n.has("value_int")) {
        t.dtype = INT64;
        t.i = {n.get_int("value_int", 0)};
      } else if (n.has("value_ints")) {
        t.dtype = INT64;
        t.i = n.get_ints("value_ints");
        t.dims = {static_cast<int64_t>(t.i.size())};
      } else {
        throw OnnxError("unsupported Constant node " + n.name);
      }
      t.name = n.outputs[0];
      m.initializers[t.name] = std::move(t);
    } else {
      rest.push_back(std::move(n));
    }
  }
  // Kahn's algorithm, stable with respect to file order.
  std::unordered_set<std::string> avail;
  for (auto& kv : m.initializers) avail.insert(kv.first);
  for (auto& vi : m.inputs) avail.insert(vi.name);
  avail.insert("");
  std::vector<Node> sorted;
  std::vector<bool> done(rest.size(), false);
  size_t remaining = rest.size();
  while (remaining) {
    bool progress = false;
    for (size_t k = 0; k < rest.size(); ++k) {
      if (done[k]) continue;
      bool ready = true;
      for (auto& in : rest[k].inputs)
        if (!avail.count(in)) {
          ready = false;
          break;
        }
      if (!ready) continue;
      for (auto& o : rest[k].outputs) avail.insert(o);
      sorted.push_back(std::move(rest[k]));
      done[k] = true;
      --remaining;
      progress = true;
    }
    if (!progress) {
      for (size_t k = 0; k < rest.size(); ++k)
        if (!done[k]) throw OnnxError("graph has a cycle or an undefined input at node " + rest[k].name);
    }
  }
  m.nodes = std::move(sorted);
}

}  // namespace

int64_t Node::get_int(const std::string& k, int64_t d) const {
  auto it = attrs.find(k);
  return it == attrs.end() ? d : it->second.i;
}
float Node::get_float(const std::string& k, float d) const {
  auto it = attrs.find(k);
  return it == attrs.end() ? d : it->second.f;
}
std::string Node::get_string(const std::string& k, const std::string& d) const {
  auto it = attrs.find(k);
  return it == attrs.end() ? d : it->second.s;
}
std::vector<int64_t> Node::get_ints(const std::string& k, const std::vector<int64_t>& d) const {
  auto it = attrs.find(k);
  return it == attrs.end() ? d : it->second.ints;
}
std::vector<float> Node::get_floats(const std::string& k, const std::vector<float>& d) const {
  auto it = attrs.find(k);
  return it == attrs.end() ? d : it->second.floats;
}
const std::string& Node::in(size_t i) const {
  static const std::string empty;
  return i < inputs.size() ? inputs[i] : empty;
}

int64_t Model::opset(const std::string& domain) const {
  for (auto& o : opsets)
    if (o.first == domain || (domain.empty() && o.first == "ai.onnx")) return o.second;
  return 0;
}

size_t Model::param_bytes_f32() const {
  size_t n = 0;
  for (auto& kv : initializers) n += kv.second.f.size() * 4;
  return n;
}

Model parse_onnx(const uint8_t* data, size_t size) {
  Model m;
  Reader r{data, data + size};
  bool have_graph = false;
  uint32_t f, wt;
  while (r.next(f, wt)) {
    switch (f) {
      case 1: m.ir_version = static_cast<int64_t>(r.varint()); break;
      case 2: m.producer_name = r.str(); break;
      case 7:
        parse_graph(r.sub(), m);
        have_graph = true;
        break;
      case 8: {
        Reader o = r.sub();
        std::string dom;
        int64_t ver = 0;
        uint32_t f2, w2;
        while (o.next(f2, w2)) {
          if (f2 == 1) dom = o.str();
          else if (f2 == 2) ver = static_cast<int64_t>(o.varint());
          else o.skip(w2);
        }
        m.opsets.emplace_back(dom, ver);
        break;
      }
      default: r.skip(wt);
    }
  }
  if (!have_graph) throw OnnxError("model has no graph");
  toposort_and_fold_constants(m);
  return m;
}

Model load_onnx(const std::string& path) {
  std::ifstream in(path, std::ios::binary | std::ios::ate);
  if (!in) throw OnnxError("cannot open model file: " + path);
  std::streamsize n = in.tellg();
  in.seekg(0);
  std::vector<uint8_t> buf(static_cast<size_t>(n));
  if (!in.read(reinterpret_cast<char*>(buf.data()), n)) throw OnnxError("cannot read model file: " + path);
  return parse_onnx(buf.data(), buf.size());
}

}  // namespace onnx
}  // namespace die
