// Instantiates the wide-tile (256-row, 8-wave) launch configurations of the GEMM (conv_igemm_impl.h
// gemm_wide_kernel): variant 7 of the config space, tile 0 = 256 x 128.
#include "conv_igemm_impl.h"

namespace die {
namespace kern {
namespace igemm {

hipError_t launch_tile_wide(const ConvArgs& a, hipStream_t s, int tile) {
  return tile == TILE_128x128 ? launch_wide(a, s) : hipErrorInvalidValue;
}

}  // namespace igemm
}  // namespace kern
}  // namespace die
