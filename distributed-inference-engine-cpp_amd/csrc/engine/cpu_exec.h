// Reference fp32 ONNX interpreter on the CPU (OpenMP).
//
// Plays the role of the reference's ORT CPU execution provider fallback
// (src/inference_engine.cpp:26-29) and is the correctness oracle for the HIP engine's graph
// passes: it executes the graph node by node with no fusion, NCHW, fp32.
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../onnx/onnx_model.h"

namespace die {

struct CpuValue {
  std::vector<int64_t> shape;
  bool is_int = false;
  std::vector<float> f;
  std::vector<int64_t> i;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    return n;
  }
};
using CpuValuePtr = std::shared_ptr<CpuValue>;

class CpuExecutor {
 public:
  explicit CpuExecutor(onnx::Model model);
  // Run with the first graph input bound to `input` (shape includes batch).  Returns the first
  // graph output.
  CpuValuePtr run(const CpuValuePtr& input, std::unordered_map<std::string, CpuValuePtr>* trace = nullptr);
  const onnx::Model& model() const { return model_; }

 private:
  onnx::Model model_;
  std::unordered_map<std::string, CpuValuePtr> consts_;
  std::unordered_map<std::string, size_t> last_use_;
};

// Exposed for unit tests.
void cpu_gemm(int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
              bool accumulate);

}  // namespace die
