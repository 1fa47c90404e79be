#include "metrics.h"

#include <cmath>
#include <cstdio>

namespace die {

namespace {

std::string sanitize(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  for (char c : s) o += (std::isalnum(static_cast<unsigned char>(c)) || c == '_') ? c : '_';
  if (!o.empty() && std::isdigit(static_cast<unsigned char>(o[0]))) o.insert(o.begin(), '_');
  return o;
}

std::string escape_label(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '\\' || c == '"') o += '\\';
    if (c == '\n') {
      o += "\\n";
      continue;
    }
    o += c;
  }
  return o;
}

void emit(std::string& out, const std::string& name, const std::string& labels, double v) {
  char num[64];
  if (std::isnan(v)) std::snprintf(num, sizeof num, "NaN");
  else if (std::isinf(v)) std::snprintf(num, sizeof num, v > 0 ? "+Inf" : "-Inf");
  else std::snprintf(num, sizeof num, "%.17g", v);
  out += name;
  if (!labels.empty()) {
    out += '{';
    out += labels;
    out += '}';
  }
  out += ' ';
  out += num;
  out += '\n';
}

// name: metric name (array levels become an `index` label); lname: the same path with array
// indices spelled out, used when a string leaf turns into an info label (unique per element).
void walk(const Json& j, const std::string& name, const std::string& lname, const std::string& labels,
          std::string& out, std::string& info) {
  if (j.is_number()) {
    emit(out, name, labels, j.as_double());
  } else if (j.is_bool()) {
    emit(out, name, labels, j.as_bool() ? 1.0 : 0.0);
  } else if (j.is_string()) {
    if (!info.empty()) info += ',';
    info += lname + "=\"" + escape_label(j.as_string()) + "\"";
  } else if (j.is_object()) {
    for (const auto& kv : j.as_object()) {
      const std::string k = sanitize(kv.first);
      walk(kv.second, name + "_" + k, lname + "_" + k, labels, out, info);
    }
  } else if (j.is_array()) {
    const auto& a = j.as_array();
    for (size_t i = 0; i < a.size(); ++i) {
      std::string l = labels;
      if (!l.empty()) l += ',';
      l += "index=\"" + std::to_string(i) + "\"";
      walk(a[i], name, lname + "_" + std::to_string(i), l, out, info);
    }
  }
}

}  // namespace

std::string prometheus_text(const Json& stats, const std::string& prefix, const std::string& labels) {
  std::string out, info;
  const std::string p = sanitize(prefix);
  if (stats.is_object()) {
    for (const auto& kv : stats.as_object()) {
      const std::string k = sanitize(kv.first);
      walk(kv.second, p + "_" + k, k, labels, out, info);
    }
  } else {
    walk(stats, p, "value", labels, out, info);
  }
  // string leaves: one info sample carrying them as labels
  std::string il = labels;
  if (!info.empty()) {
    if (!il.empty()) il += ',';
    il += info;
  }
  emit(out, p + "_info", il, 1.0);
  return out;
}

}  // namespace die
