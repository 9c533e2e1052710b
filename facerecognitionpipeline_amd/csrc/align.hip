// Face alignment and blur quality on gfx950: the reference's FaceAligner.align
// (face_recognition.py:64-74: cv2.warpAffine INTER_LINEAR, BORDER_CONSTANT 0) and
// FaceQualityFilter.compute_blur_score (face_recognition.py:94-99: RGB2GRAY ->
// Laplacian CV_64F ksize 1 -> var), so crops go from the frame in HBM straight
// into fr_embed without a host round trip.
//
// Both kernels are integer-exact restatements of OpenCV's uint8 arithmetic
// (oracle/align_ref.py): the warp's map is AB_BITS=10 fixed point with
// cvRound (round-half-even) of double products, 5-bit sub-pixel positions and
// 15-bit bilinear weights; gray is 14-bit fixed point; the Laplacian's variance
// is summed in numpy's order (ndarray.var, below), so it is bitwise the
// reference's.  HBM-bound gathers (a 112x112x3 crop reads ~4x its size at most).
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

// numpy's order for a float64 add-reduction over a contiguous array (numpy 2.x: the buffered
// reduction iterator hands the loop chunks of NPY_BUFSIZE = 8192 elements, and the loop adds each
// chunk's pairwise_sum -- loops_utils.h.src -- to the running value, which starts at 0):
//   sum = ((0 + pw(chunk 0)) + pw(chunk 1)) + ...
//   pw(n) = n <= 128 ? leaf(n) : pw(n2) + pw(n - n2),   n2 = n/2 - (n/2) % 8
//   leaf(n) = n < 8: sequential from 0; else 8 interleaved accumulators over the first n - n % 8,
//             ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the rest sequentially.
// ndarray.var() (face_recognition.py:99 calls it on cv2.Laplacian's float64 image) is
//   m = sum(L) / n;  var = sum((L - m) * (L - m)) / n      (numpy/_core/_methods.py _var)
// with both sums in that order; fp contraction is off in this file, so every operation rounds
// as numpy's does and the result is bitwise numpy's (tests/test_align.py).
constexpr int NP_BUFSIZE = 8192, NP_PW_BLOCK = 128;

// calls f(leaf index, start, length) for the pairwise_sum leaves of [0, n), left to right
template <typename F>
__device__ void np_sum_leaves(int n, F&& f) {
  int li = 0;
  for (int c0 = 0; c0 < n; c0 += NP_BUFSIZE) {
    int st[24], ln[24], sp = 1;
    st[0] = c0;
    ln[0] = min(NP_BUFSIZE, n - c0);
    while (sp) {
      --sp;
      const int s = st[sp], m = ln[sp];
      if (m <= NP_PW_BLOCK) {
        f(li++, s, m);
        continue;
      }
      int m2 = m / 2;
      m2 -= m2 % 8;
      st[sp] = s + m2;  // right half below the left, so the left pops first
      ln[sp] = m - m2;
      st[sp + 1] = s;
      ln[sp + 1] = m2;
      sp += 2;
    }
  }
}

// pw(m) over the leaf values part[li ..] (consumed in order); a chunk of <= 8192 is <= 7 levels deep
template <int D>
__device__ __noinline__ double np_pw_eval(int m, const double* part, int& li) {
  if (m <= NP_PW_BLOCK) return part[li++];
  if constexpr (D > 0) {
    int m2 = m / 2;
    m2 -= m2 % 8;
    const double a = np_pw_eval<D - 1>(m2, part, li);
    const double b = np_pw_eval<D - 1>(m - m2, part, li);
    return a + b;
  } else {
    __builtin_trap();
  }
}

// One block per crop: gray into LDS, 4-neighbour Laplacian with reflect-101 borders (integers,
// exact in double), sum(L) exactly in int64 (so its float64 value does not depend on the order),
// then the squared deviations summed in numpy's order: each thread sums whole pairwise leaves,
// thread 0 combines them in the tree's order.
__global__ __launch_bounds__(256) void blur_kernel(const uint8_t* __restrict__ crops, int S, double* __restrict__ var) {
  extern __shared__ __align__(8) uint8_t s_dyn[];
  double* part = reinterpret_cast<double*>(s_dyn);               // [leaves]
  const int n = S * S;
  uint8_t* s_gray = s_dyn + 8 * (n / 64 + 2 * ((n + NP_BUFSIZE - 1) / NP_BUFSIZE));
  __shared__ long long red[4];
  __shared__ double s_mean;
  const uint8_t* img = crops + (long long)blockIdx.x * n * 3;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int r = img[i * 3], g = img[i * 3 + 1], b = img[i * 3 + 2];
    s_gray[i] = (uint8_t)((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14);
  }
  __syncthreads();
  auto lap = [&](int i) {
    const int y = i / S, x = i - y * S;
    const int ym = y > 0 ? y - 1 : 1, yp = y < S - 1 ? y + 1 : S - 2;
    const int xm = x > 0 ? x - 1 : 1, xp = x < S - 1 ? x + 1 : S - 2;
    return s_gray[ym * S + x] + s_gray[yp * S + x] + s_gray[y * S + xm] + s_gray[y * S + xp] - 4 * s_gray[i];
  };
  long long s1 = 0;
  for (int i = threadIdx.x; i < n; i += 256) s1 += lap(i);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s1 += __shfl_xor(s1, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s1;
  __syncthreads();
  if (threadIdx.x == 0) s_mean = (double)(red[0] + red[1] + red[2] + red[3]) / (double)n;
  __syncthreads();
  const double m = s_mean;
  auto dev2 = [&](int i) {
    const double d = (double)lap(i) - m;
    return d * d;
  };
  np_sum_leaves(n, [&](int li, int s, int len) {
    if (li % 256 != (int)threadIdx.x) return;
    double res;
    if (len < 8) {
      res = 0.0;
      for (int i = 0; i < len; ++i) res = res + dev2(s + i);
    } else {
      double r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = dev2(s + j);
      int i = 8;
      for (; i < len - (len % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = r[j] + dev2(s + i + j);
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; i < len; ++i) res = res + dev2(s + i);
    }
    part[li] = res;
  });
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    int li = 0;
    for (int c0 = 0; c0 < n; c0 += NP_BUFSIZE) acc = acc + np_pw_eval<10>(min(NP_BUFSIZE, n - c0), part, li);
    var[blockIdx.x] = acc / (double)n;
  }
}

// dynamic LDS of blur_kernel: the leaf sums (<= n / 64 + 2 per chunk) + the gray crop
static size_t blur_lds_bytes(int S) {
  const size_t n = (size_t)S * S;
  return 8 * (n / 64 + 2 * ((n + NP_BUFSIZE - 1) / NP_BUFSIZE)) + n;
}

hipError_t launch_blur(const uint8_t* crops, int n, int S, double* var, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const size_t lds = blur_lds_bytes(S);
  if (S < 2 || lds > 160 * 1024) return hipErrorInvalidValue;  // crops up to 357 x 357
  hipLaunchKernelGGL(blur_kernel, dim3(n), dim3(256), lds, s, crops, S, var);
  return hipGetLastError();
}

}  // namespace frhip
