// Tiny `--name value` / `--name=value` / `--flag` parser that leaves positionals in order, so the
// binaries keep the reference's positional CLIs (src/worker_node.cpp:145-168,
// src/gateway.cpp:161-171) and add optional flags whose defaults equal the reference constants.
#pragma once

#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace die {

class Flags {
 public:
  Flags(int argc, char** argv, const std::vector<std::string>& boolean_flags = {}) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
        std::string k = a.substr(2), v;
        size_t eq = k.find('=');
        if (eq != std::string::npos) {
          v = k.substr(eq + 1);
          k = k.substr(0, eq);
        } else {
          bool is_bool = false;
          for (auto& b : boolean_flags) is_bool |= b == k;
          if (is_bool || i + 1 >= argc) v = "1";
          else v = argv[++i];
        }
        kv_[k] = v;
      } else {
        pos_.push_back(a);
      }
    }
  }
  const std::vector<std::string>& positional() const { return pos_; }
  bool has(const std::string& k) const { return kv_.count(k) != 0; }
  std::string str(const std::string& k, const std::string& d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : it->second;
  }
  long long i(const std::string& k, long long d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : std::stoll(it->second);
  }
  double f(const std::string& k, double d) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? d : std::stod(it->second);
  }
  bool b(const std::string& k) const {
    auto it = kv_.find(k);
    return it != kv_.end() && it->second != "0" && it->second != "false";
  }

 private:
  std::map<std::string, std::string> kv_;
  std::vector<std::string> pos_;
};

}  // namespace die
