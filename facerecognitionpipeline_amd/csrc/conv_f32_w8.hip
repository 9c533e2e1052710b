// Instantiations of the implicit-GEMM conv kernel (conv_mfma_impl.h), split across
// translation units so hipcc builds them in parallel.
#include "conv_mfma_impl.h"

namespace frhip {

hipError_t launch_conv_f32_w8(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s) {
  switch (tile) {
    case TILE_128x128_W8: return launch_tile<128, 128, 2, 4, false>(p, pre, epi, nsplit, s);
    case TILE_256x128_W8: return launch_tile<256, 128, 4, 2, false>(p, pre, epi, nsplit, s);
    case TILE_128x64_W8: return launch_tile<128, 64, 4, 2, false>(p, pre, epi, nsplit, s);
    case TILE_64x256_W8: return launch_tile<64, 256, 2, 4, false>(p, pre, epi, nsplit, s);
    case TILE_256x64_W8: return launch_tile<256, 64, 4, 2, false>(p, pre, epi, nsplit, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frhip
