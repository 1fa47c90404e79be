// Instantiates the 64x128-tile launch configurations of the implicit-GEMM conv (conv_igemm_impl.h).
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {

hipError_t launch_tile_64x128(const ConvArgs& a, hipStream_t s, int variant) { return launch_cfg<64, 128>(a, s, variant); }

}  // namespace igemm
}  // namespace kern
}  // namespace die
