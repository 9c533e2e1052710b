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

// numpy's order for a float64 add-reduction over a contiguous array (derived from numpy 2.2's
// sources and checked bitwise against numpy 2.2.6, the version in the build image; numpy 2.x: the
// buffered reduction iterator hands the loop chunks of NPY_BUFSIZE = 8192 elements, and the loop
// adds each chunk's pairwise_sum -- loops_utils.h.src -- to the running value, which starts at 0):
//   sum = ((0 + pw(chunk 0)) + pw(chunk 1)) + ...
//   pw(n) = n <= 128 ? leaf(n) : pw(n2) + pw(n - n2),   n2 = n/2 - (n/2) % 8
//   leaf(n) = n < 8: sequential from 0; else 8 interleaved accumulators over the first n - n % 8,
//             ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the rest sequentially.
// ndarray.var() (face_recognition.py:99 calls it on cv2.Laplacian's float64 image) is
//   m = sum(L) / n;  var = sum((L - m) * (L - m)) / n      (numpy/_core/_methods.py _var)
// with both sums in that order; fp contraction is off in this file, so every operation rounds
// as numpy's does and the result is bitwise numpy's (tests/test_align.py).
constexpr int NP_BUFSIZE = 8192, NP_PW_BLOCK = 128;
// The pairwise tree of a chunk of <= 8192 elements is at most 7 splits deep (each split leaves
// parts of at most half + 8 elements; checked for every chunk length): 128 leaf-level slots and
// 255 tree nodes per chunk.
constexpr int NP_DEPTH = 7, NP_SLOTS = 1 << NP_DEPTH, NP_NODES = 2 * NP_SLOTS - 1;

// One image of a blur batch: uint8 [H][W][C], C = 3 or 4 (cv2 COLOR_RGB2GRAY: 14-bit fixed
// point, alpha ignored) or 1 (the reference's 2-D gray branch, face_recognition.py:95-98), and
// cv2.Laplacian ksize 1 = the 4-neighbour kernel with BORDER_REFLECT_101 (an axis of length 1
// reflects onto itself).  Integer-exact.
struct BlurImg {
  const uint8_t* p;
  int H, W, C;
  __device__ int gray(int i) const {
    if (C == 1) return p[i];
    const uint8_t* q = p + (long long)i * C;
    return (q[0] * 4899 + q[1] * 9617 + q[2] * 1868 + (1 << 13)) >> 14;
  }
  template <typename G>
  __device__ static int lap(int i, int H, int W, G g) {
    const int y = i / W, x = i - y * W;
    const int ym = y > 0 ? y - 1 : (H > 1 ? 1 : 0), yp = y < H - 1 ? y + 1 : (H > 1 ? H - 2 : 0);
    const int xm = x > 0 ? x - 1 : (W > 1 ? 1 : 0), xp = x < W - 1 ? x + 1 : (W > 1 ? W - 2 : 0);
    return g(ym * W + x) + g(yp * W + x) + g(y * W + xm) + g(y * W + xp) - 4 * g(i);
  }
};

// Top-down split of nch chunk trees (chunk c's root = node c * 255 with range [lo, lo + len)):
// node k of level l of chunk c lives at c * 255 + 2^l - 1 + k; its children are nodes 2k and
// 2k + 1 of level l + 1 (a leaf is carried down to 2k alone), so every level keeps the
// left-to-right order.  Ranges are split as pairwise_sum splits them.
__device__ void np_tree_split(int* lo, int* len, int nch, int tid, int nthr) {
  for (int l = 0; l < NP_DEPTH; ++l) {
    for (int j = tid; j < (nch << l); j += nthr) {
      const int c = j >> l, k = j & ((1 << l) - 1);
      const int src = c * NP_NODES + (1 << l) - 1 + k;
      const int dst = c * NP_NODES + (2 << l) - 1 + 2 * k;
      const int s0 = lo[src], m = len[src];
      int m2 = m;  // a leaf (or nothing) is carried down alone
      if (m > NP_PW_BLOCK) {
        m2 = m / 2;
        m2 -= m2 % 8;
      }
      lo[dst] = s0;
      len[dst] = m2;
      lo[dst + 1] = s0 + m2;
      len[dst + 1] = m - m2;
    }
    __syncthreads();
  }
}

// Leaves (pairwise_sum's n <= 128 branch, one per thread), then bottom-up: a split node = left +
// right, a carried leaf passes its value up.  val: [2][nch * 128]; chunk c's value ends in
// val[c * 128].
template <typename F>
__device__ void np_tree_sum(const int* lo, const int* len, double* val, int nch, int tid, int nthr, F dev2) {
  for (int j = tid; j < nch * NP_SLOTS; j += nthr) {
    const int c = j / NP_SLOTS, k = j % NP_SLOTS;
    const int nd = c * NP_NODES + NP_SLOTS - 1 + k;
    const int s = lo[nd], m = len[nd];
    double res = 0.0;
    if (m < 8) {
      for (int i = 0; i < m; ++i) res = res + dev2(s + i);
    } else {
      double r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = dev2(s + q);
      int i = 8;
      for (; i < m - (m % 8); i += 8)
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = r[q] + dev2(s + i + q);
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; i < m; ++i) res = res + dev2(s + i);
    }
    val[(NP_DEPTH & 1) * nch * NP_SLOTS + j] = res;
  }
  __syncthreads();
  for (int l = NP_DEPTH - 1; l >= 0; --l) {
    const double* vc = val + ((l + 1) & 1) * nch * NP_SLOTS;
    double* vp = val + (l & 1) * nch * NP_SLOTS;
    for (int j = tid; j < (nch << l); j += nthr) {
      const int c = j >> l, k = j & ((1 << l) - 1);
      const int ch = c * NP_SLOTS + 2 * k;
      vp[c * NP_SLOTS + k] = len[c * NP_NODES + (1 << l) - 1 + k] > NP_PW_BLOCK ? vc[ch] + vc[ch + 1] : vc[ch];
    }
    __syncthreads();
  }
}

__device__ long long block_sum_i64(long long v, long long* red, int tid) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  const long long t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// Images whose gray copy and chunk trees fit in LDS: one block per image.  Gray into LDS,
// sum(L) exactly in int64 (so its float64 value does not depend on the order), then the squared
// deviations summed in numpy's order, every chunk's tree evaluated level by level in parallel;
// thread 0 adds the chunks' values to a running 0.  (The first form walked the tree per thread
// and combined it in one thread through recursive calls: 1.23 ms for 256 crops, on the C4 step's
// critical path; this one 0.06 ms.)
__global__ __launch_bounds__(256) void blur_kernel(const uint8_t* __restrict__ crops, int H, int W, int C,
                                                   double* __restrict__ var) {
  extern __shared__ __align__(8) uint8_t s_dyn[];
  const int n = H * W;
  const int nch = (n + NP_BUFSIZE - 1) / NP_BUFSIZE;
  double* val = reinterpret_cast<double*>(s_dyn);   // [2][nch * 128]: two adjacent levels' values
  int* lo = reinterpret_cast<int*>(val + 2 * nch * NP_SLOTS);  // [nch * 255]: node starts
  int* len = lo + nch * NP_NODES;                               // [nch * 255]: node lengths
  uint8_t* s_gray = reinterpret_cast<uint8_t*>(len + nch * NP_NODES);
  __shared__ long long red[4];
  const int tid = threadIdx.x;
  const BlurImg im{crops + (long long)blockIdx.x * n * C, H, W, C};
  for (int i = tid; i < n; i += 256) s_gray[i] = (uint8_t)im.gray(i);
  for (int c = tid; c < nch; c += 256) {  // level 0: the chunks
    lo[c * NP_NODES] = c * NP_BUFSIZE;
    len[c * NP_NODES] = min(NP_BUFSIZE, n - c * NP_BUFSIZE);
  }
  __syncthreads();
  auto g = [&](int i) { return (int)s_gray[i]; };
  long long s1 = 0;
  for (int i = tid; i < n; i += 256) s1 += BlurImg::lap(i, H, W, g);
  const double mean = (double)block_sum_i64(s1, red, tid) / (double)n;
  np_tree_split(lo, len, nch, tid, 256);
  np_tree_sum(lo, len, val, nch, tid, 256, [&](int i) {
    const double d = (double)BlurImg::lap(i, H, W, g) - mean;
    return d * d;
  });
  if (tid == 0) {
    double acc = 0.0;
    for (int c = 0; c < nch; ++c) acc = acc + val[c * NP_SLOTS];  // level 0 in val[0]
    var[blockIdx.x] = acc / (double)n;
  }
}

// Larger images, one block per (chunk, image) in three launches: the chunk's exact int64 sum of
// L; the chunk's pairwise sum of squared deviations (the mean from all chunk sums, added in
// integers, so exactly the one-block value); the chunks' values added in order per image.  Gray
// is recomputed from the image in global memory (L2-resident neighbour rows), so there is no
// size limit.
__global__ __launch_bounds__(256) void blur_lsum_kernel(const uint8_t* __restrict__ crops, int H, int W, int C,
                                                        long long* __restrict__ lsum) {
  __shared__ long long red[4];
  const int n = H * W, nch = gridDim.x, c = blockIdx.x, tid = threadIdx.x;
  const BlurImg im{crops + (long long)blockIdx.y * n * C, H, W, C};
  auto g = [&](int i) { return im.gray(i); };
  long long s1 = 0;
  const int e = min(n, (c + 1) * NP_BUFSIZE);
  for (int i = c * NP_BUFSIZE + tid; i < e; i += 256) s1 += BlurImg::lap(i, H, W, g);
  s1 = block_sum_i64(s1, red, tid);
  if (tid == 0) lsum[(long long)blockIdx.y * nch + c] = s1;
}

__global__ __launch_bounds__(256) void blur_chunk_kernel(const uint8_t* __restrict__ crops, int H, int W, int C,
                                                         const long long* __restrict__ lsum,
                                                         double* __restrict__ cval) {
  __shared__ double val[2 * NP_SLOTS];
  __shared__ int lo[NP_NODES], len[NP_NODES];
  __shared__ double s_mean;
  const int n = H * W, nch = gridDim.x, c = blockIdx.x, tid = threadIdx.x;
  const BlurImg im{crops + (long long)blockIdx.y * n * C, H, W, C};
  if (tid == 0) {
    long long t = 0;
    for (int k = 0; k < nch; ++k) t += lsum[(long long)blockIdx.y * nch + k];
    s_mean = (double)t / (double)n;
    lo[0] = c * NP_BUFSIZE;
    len[0] = min(NP_BUFSIZE, n - c * NP_BUFSIZE);
  }
  __syncthreads();
  const double mean = s_mean;
  auto g = [&](int i) { return im.gray(i); };
  np_tree_split(lo, len, 1, tid, 256);
  np_tree_sum(lo, len, val, 1, tid, 256, [&](int i) {
    const double d = (double)BlurImg::lap(i, H, W, g) - mean;
    return d * d;
  });
  if (tid == 0) cval[(long long)blockIdx.y * nch + c] = val[0];
}

__global__ __launch_bounds__(256) void blur_final_kernel(const double* __restrict__ cval, int nimg, int nch,
                                                         int npix, double* __restrict__ var) {
  const int img = blockIdx.x * 256 + threadIdx.x;
  if (img >= nimg) return;
  double acc = 0.0;
  for (int c = 0; c < nch; ++c) acc = acc + cval[(long long)img * nch + c];
  var[img] = acc / (double)npix;
}

// dynamic LDS of blur_kernel: two levels of values, the trees' node ranges, the gray image
size_t blur_lds_bytes(int H, int W) {
  const size_t n = (size_t)H * W, nch = (n + NP_BUFSIZE - 1) / NP_BUFSIZE;
  return 2 * nch * NP_SLOTS * 8 + 2 * nch * NP_NODES * 4 + n;
}

size_t blur_workspace_bytes(int n, int H, int W) {
  if (blur_lds_bytes(H, W) <= BLUR_LDS_MAX) return 0;
  const size_t nch = ((size_t)H * W + NP_BUFSIZE - 1) / NP_BUFSIZE;
  return (size_t)n * nch * (sizeof(long long) + sizeof(double));
}

hipError_t launch_blur(const uint8_t* crops, int n, int H, int W, int C, double* var, void* ws, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (H < 1 || W < 1 || (long long)H * W >= (1ll << 31) || (C != 1 && C != 3 && C != 4))
    return hipErrorInvalidValue;
  const size_t lds = blur_lds_bytes(H, W);
  if (lds <= BLUR_LDS_MAX) {
    hipLaunchKernelGGL(blur_kernel, dim3(n), dim3(256), lds, s, crops, H, W, C, var);
    return hipGetLastError();
  }
  const long long npix = (long long)H * W;
  const int nch = (int)((npix + NP_BUFSIZE - 1) / NP_BUFSIZE);
  if (!ws || n > 65535) return hipErrorInvalidValue;
  long long* lsum = static_cast<long long*>(ws);
  double* cval = reinterpret_cast<double*>(lsum + (size_t)n * nch);
  hipLaunchKernelGGL(blur_lsum_kernel, dim3(nch, n), dim3(256), 0, s, crops, H, W, C, lsum);
  hipLaunchKernelGGL(blur_chunk_kernel, dim3(nch, n), dim3(256), 0, s, crops, H, W, C, lsum, cval);
  hipLaunchKernelGGL(blur_final_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cval, n, nch, (int)npix, var);
  return hipGetLastError();
}

}  // namespace frhip
