// Conv dispatch: validates a launch and routes it to the translation unit holding the
// (tile, precision) instantiation.  Kernel: conv_mfma_impl.h.
#include "frhip_kernels.h"

namespace frhip {

hipError_t launch_conv_f32_w4(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s);
hipError_t launch_conv_f32_w8(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s);
hipError_t launch_conv_bf16x3(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s);
hipError_t launch_conv_det(const ConvParams& p, ConvTile tile, Epi epi, int nsplit, hipStream_t s);

hipError_t launch_conv(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s,
                       Precision prec) {
  const int main_steps = p.KH * p.KW * p.Cin / 32;
  if (p.Cin % 32 != 0 || p.Cin2 < 0 || p.Cin2 % 32 != 0 || p.steps_total != main_steps + p.Cin2 / 32 || nsplit < 1 ||
      (long long)p.steps_per_split * nsplit < p.steps_total || p.M <= 0 || p.Cout <= 0 ||
      (long long)p.B * p.H * p.W * p.Cin * 4 >= (1ll << 31) ||
      (long long)p.Cout * (p.KH * p.KW * p.Cin + p.Cin2) * 4 >= (1ll << 31) || (p.sk_cus > 0 && nsplit != 1) ||
      (long long)p.M * p.Cout * 4 >= (1ll << 31))  // 32-bit output offsets (the epilogue's buffer stores)
    return hipErrorInvalidValue;
  // fused 1x1 shortcut: its own input, no pre-BN, not on the detector's instances
  if (p.Cin2 > 0 && (!p.x2 || pre || p.steps1 != main_steps || (long long)p.B * p.H * p.W * p.Cin2 * 4 >= (1ll << 31) ||
                     epi == EPI_AFFINE_RES_PRELU || epi == EPI_AFFINE_PRELU))
    return hipErrorInvalidValue;
  // detector instances (f32 only, whatever the handle's precision)
  if (epi == EPI_AFFINE_RES_PRELU || (epi == EPI_AFFINE_PRELU && !pre)) {
    if (pre) return hipErrorInvalidValue;
    return launch_conv_det(p, tile, epi, nsplit, s);
  }
  if (prec == PREC_BF16X3) return launch_conv_bf16x3(p, tile, pre, epi, nsplit, s);
  if (tile >= TILE_128x128_W8) return launch_conv_f32_w8(p, tile, pre, epi, nsplit, s);
  return launch_conv_f32_w4(p, tile, pre, epi, nsplit, s);
}

int conv_tile_bm(ConvTile t) {
  switch (t) {
    case TILE_256x64: case TILE_256x128: case TILE_256x128_W8: case TILE_256x64_W8: return 256;
    case TILE_64x128: case TILE_64x256_W8: return 64;
    default: return 128;
  }
}

int conv_tile_bn(ConvTile t) {
  switch (t) {
    case TILE_256x64: case TILE_128x64: case TILE_128x64_W8: case TILE_256x64_W8: return 64;
    case TILE_128x256: case TILE_64x256_W8: return 256;
    default: return 128;
  }
}

}  // namespace frhip
