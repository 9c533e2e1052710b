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

// Split-K finish of a serving-sized direct conv: y[m][n] = epilogue(sum over the S raw slabs
// part[s][m][n], in split order: deterministic), the epilogue exactly as conv_mfma_kernel's
// (v * scale + shift, then the residual: same row / the MaxPool2d(1, 2) shortcut pixel).  One
// thread per output; every slab load of a thread is in flight at once (S <= 32).
template <int EPI>
__global__ __launch_bounds__(256) void conv_split_fixup_kernel(ConvParams p, const float* __restrict__ part, int S,
                                                               long long stride) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)p.M * p.Cout) return;
  float a[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) a[k] = k < S ? part[k * stride + i] : 0.f;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 32; ++k)
    if (k < S) v += a[k];
  const int n = (int)(i % p.Cout);
  const int m = (int)(i / p.Cout);
  v = v * p.post_scale[n] + p.post_shift[n];
  if constexpr (EPI == EPI_AFFINE_RES) v += p.res[i];
  if constexpr (EPI == EPI_AFFINE_RES_SUB) {
    const int HoWo = p.Ho * p.Wo;
    const int b = m / HoWo, rem = m - b * HoWo, oy = rem / p.Wo, ox = rem - oy * p.Wo;
    v += p.res[(((long long)b * p.res_H + 2 * oy) * p.res_W + 2 * ox) * p.Cout + n];
  }
  p.y[i] = v;
}

hipError_t launch_conv_split_fixup(const ConvParams& p, Epi epi, const float* part, int S, long long stride,
                                   hipStream_t s) {
  if (S < 1 || S > 32) return hipErrorInvalidValue;
  const long long n = (long long)p.M * p.Cout;
  const dim3 grid((unsigned)((n + 255) / 256));
  switch (epi) {
    case EPI_AFFINE: hipLaunchKernelGGL(conv_split_fixup_kernel<EPI_AFFINE>, grid, dim3(256), 0, s, p, part, S, stride); break;
    case EPI_AFFINE_RES:
      hipLaunchKernelGGL(conv_split_fixup_kernel<EPI_AFFINE_RES>, grid, dim3(256), 0, s, p, part, S, stride);
      break;
    case EPI_AFFINE_RES_SUB:
      hipLaunchKernelGGL(conv_split_fixup_kernel<EPI_AFFINE_RES_SUB>, grid, dim3(256), 0, s, p, part, S, stride);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
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
