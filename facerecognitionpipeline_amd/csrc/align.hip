// Face alignment and blur quality on gfx950: the reference's FaceAligner.align
// (face_recognition.py:64-74: cv2.warpAffine INTER_LINEAR, BORDER_CONSTANT 0) and
// FaceQualityFilter.compute_blur_score (face_recognition.py:94-99: RGB2GRAY ->
// Laplacian CV_64F ksize 1 -> var), so crops go from the frame in HBM straight
// into fr_embed without a host round trip.
//
// Both kernels are integer-exact restatements of OpenCV's uint8 arithmetic
// (oracle/align_ref.py): the warp's map is AB_BITS=10 fixed point with
// cvRound (round-half-even) of double products, 5-bit sub-pixel positions and
// 15-bit bilinear weights; gray is 14-bit fixed point; the Laplacian sums are
// exact in int64, so the variance is the correctly rounded double of an exact
// rational.  HBM-bound gathers (a 112x112x3 crop reads ~4x its size at most).
#include "frhip_kernels.h"

// The map arithmetic must round exactly like OpenCV (separate double mul and add).
#pragma clang fp contract(off)

namespace frhip {

// One thread per output pixel (all channels); blockIdx.y = face.
// Maps come from device memory (minv) or, for up to WARP_MAPS_BY_VALUE faces, by value in the
// kernel arguments (no H2D copy, so the caller needs no stream sync to keep a host buffer alive).
__global__ __launch_bounds__(256) void warp_affine_kernel(const uint8_t* __restrict__ frame, int H, int W,
                                                          const double* __restrict__ minv, WarpMaps maps,
                                                          int S, uint8_t* __restrict__ out) {
  const int face = blockIdx.y;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= S * S) return;
  const int oy = pix / S, ox = pix - oy * S;
  const double* m = minv ? minv + face * 6 : maps.m[face];
  const long long X0 = (long long)__builtin_rint((m[1] * oy + m[2]) * 1024.0) + 16;
  const long long Y0 = (long long)__builtin_rint((m[4] * oy + m[5]) * 1024.0) + 16;
  const long long adx = (long long)__builtin_rint(m[0] * ox * 1024.0);
  const long long bdx = (long long)__builtin_rint(m[3] * ox * 1024.0);
  const long long X = (X0 + adx) >> 5, Y = (Y0 + bdx) >> 5;
  const int sx = (int)(X >> 5), sy = (int)(Y >> 5);
  const int fx = (int)(X & 31), fy = (int)(Y & 31);
  const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32;
  const int w10 = (32 - fx) * fy * 32, w11 = fx * fy * 32;
  const bool in_x0 = (unsigned)sx < (unsigned)W, in_x1 = (unsigned)(sx + 1) < (unsigned)W;
  const bool in_y0 = (unsigned)sy < (unsigned)H, in_y1 = (unsigned)(sy + 1) < (unsigned)H;
  uint8_t* o = out + ((long long)face * S * S + pix) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int p00 = (in_y0 && in_x0) ? frame[((long long)sy * W + sx) * 3 + c] : 0;
    const int p01 = (in_y0 && in_x1) ? frame[((long long)sy * W + sx + 1) * 3 + c] : 0;
    const int p10 = (in_y1 && in_x0) ? frame[((long long)(sy + 1) * W + sx) * 3 + c] : 0;
    const int p11 = (in_y1 && in_x1) ? frame[((long long)(sy + 1) * W + sx + 1) * 3 + c] : 0;
    int v = (p00 * w00 + p01 * w01 + p10 * w10 + p11 * w11 + (1 << 14)) >> 15;
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

hipError_t launch_warp_affine(const uint8_t* frame, int H, int W, const double* minv, int n, int S, uint8_t* out,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(warp_affine_kernel, dim3((S * S + 255) / 256, n), dim3(256), 0, s, frame, H, W, minv,
                     WarpMaps{}, S, out);
  return hipGetLastError();
}

hipError_t launch_warp_affine_by_value(const uint8_t* frame, int H, int W, const double* host_minv, int n, int S,
                                       uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n > WARP_MAPS_BY_VALUE) return hipErrorInvalidValue;
  WarpMaps maps{};
  for (int f = 0; f < n; ++f)
    for (int j = 0; j < 6; ++j) maps.m[f][j] = host_minv[f * 6 + j];
  hipLaunchKernelGGL(warp_affine_kernel, dim3((S * S + 255) / 256, n), dim3(256), 0, s, frame, H, W,
                     (const double*)nullptr, maps, S, out);
  return hipGetLastError();
}

// One block per crop: gray into LDS, 4-neighbour Laplacian with reflect-101 borders,
// int64 sums of L and L^2, var = (n*sum(L^2) - sum(L)^2) / n^2.
__global__ __launch_bounds__(256) void blur_kernel(const uint8_t* __restrict__ crops, int S, double* __restrict__ var) {
  extern __shared__ uint8_t s_gray[];
  __shared__ long long red[2][4];
  const uint8_t* img = crops + (long long)blockIdx.x * S * S * 3;
  for (int i = threadIdx.x; i < S * S; i += 256) {
    const int r = img[i * 3], g = img[i * 3 + 1], b = img[i * 3 + 2];
    s_gray[i] = (uint8_t)((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14);
  }
  __syncthreads();
  long long s1 = 0, s2 = 0;
  for (int i = threadIdx.x; i < S * S; i += 256) {
    const int y = i / S, x = i - y * S;
    const int ym = y > 0 ? y - 1 : 1, yp = y < S - 1 ? y + 1 : S - 2;
    const int xm = x > 0 ? x - 1 : 1, xp = x < S - 1 ? x + 1 : S - 2;
    const int L = s_gray[ym * S + x] + s_gray[yp * S + x] + s_gray[y * S + xm] + s_gray[y * S + xp] - 4 * s_gray[i];
    s1 += L;
    s2 += (long long)L * L;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long t1 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const long long t2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const long long n = (long long)S * S;
    var[blockIdx.x] = (double)(n * t2 - t1 * t1) / ((double)n * (double)n);
  }
}

hipError_t launch_blur(const uint8_t* crops, int n, int S, double* var, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(blur_kernel, dim3(n), dim3(256), S * S, s, crops, S, var);
  return hipGetLastError();
}

}  // namespace frhip
