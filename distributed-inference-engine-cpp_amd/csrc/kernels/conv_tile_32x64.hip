// Instantiates the 32x64-tile launch configurations of the implicit-GEMM conv (conv_igemm_impl.h;
// configs CFG_SMALL_BASE + variant).
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {

hipError_t launch_tile_32x64(const ConvArgs& a, hipStream_t s, int variant) { return launch_cfg<32, 64>(a, s, variant); }

}  // namespace igemm
}  // namespace kern
}  // namespace die
