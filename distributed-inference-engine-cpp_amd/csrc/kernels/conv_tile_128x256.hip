// Instantiates the 128 x 256 (wide) tile launch configurations of the implicit-GEMM conv
// (conv_igemm_impl.h launch_wide_cfg; configs CFG_WIDE_BASE..).
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {

hipError_t launch_tile_128x256(const ConvArgs& a, hipStream_t s, int variant) { return launch_wide_cfg<128, 256>(a, s, variant); }

}  // namespace igemm
}  // namespace kern
}  // namespace die
