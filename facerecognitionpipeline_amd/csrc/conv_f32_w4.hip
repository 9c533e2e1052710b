// Instantiations of the implicit-GEMM conv kernel (conv_mfma_impl.h), split across
// translation units so hipcc builds them in parallel.
#include "conv_mfma_impl.h"

namespace frhip {

hipError_t launch_conv_f32_w4(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s) {
  switch (tile) {
    case TILE_256x64: return launch_tile<256, 64, 4, 1, false>(p, pre, epi, nsplit, s);
    case TILE_128x128: return launch_tile<128, 128, 2, 2, false>(p, pre, epi, nsplit, s);
    case TILE_128x64: return launch_tile<128, 64, 4, 1, false>(p, pre, epi, nsplit, s);
    case TILE_64x128: return launch_tile<64, 128, 1, 4, false>(p, pre, epi, nsplit, s);
    case TILE_256x128: return launch_tile<256, 128, 2, 2, false>(p, pre, epi, nsplit, s);
    case TILE_128x256: return launch_tile<128, 256, 2, 2, false>(p, pre, epi, nsplit, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frhip
