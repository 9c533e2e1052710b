// Detector instances of the implicit-GEMM conv kernel (conv_mfma_impl.h): no pre-BN,
// conv + BN + ReLU (zero PReLU slopes) and BasicBlock conv2 + BN + residual + ReLU,
// on the tiles the SCRFD layer shapes use (detector.cpp).  f32 only.
#include "conv_mfma_impl.h"

namespace frhip {

hipError_t launch_conv_det(const ConvParams& p, ConvTile tile, Epi epi, int nsplit, hipStream_t s) {
  switch (tile) {
    case TILE_128x64_W8: return launch_tile<128, 64, 4, 2, false, 1>(p, false, epi, nsplit, s);
    case TILE_128x128_W8: return launch_tile<128, 128, 2, 4, false, 1>(p, false, epi, nsplit, s);
    case TILE_256x128_W8: return launch_tile<256, 128, 4, 2, false, 1>(p, false, epi, nsplit, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frhip
