// Placeholder until the HIP engine lands.
#include <hip/hip_runtime.h>
#include "engine.h"
namespace die {
std::unique_ptr<Engine> create_hip_engine(const std::string&, const EngineOptions&, std::string* why) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    if (why) *why = "no HIP device visible";
    return nullptr;
  }
  if (why) *why = "HIP engine not built yet";
  return nullptr;
}
}  // namespace die
