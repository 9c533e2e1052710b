// Stem, head and match-side kernels of the embed + match hot path (gfx950).
//
//   stem_kernel        FaceEmbedder.preprocess (face_embedder.py:97-104: RGB->BGR,
//                      (x/255-0.5)/0.5 in f64 -> f32) fused with net input_layer
//                      (Conv3x3 3->64 + BN2d + PReLU).  uint8 in, NHWC f32 out.
//   head_reduce_kernel split-K sum of the Linear(25088,512) partials + bias ->
//                      BN1d -> x/||x|| (AdaFace net forward tail; ArcFace has none)
//                      -> optional e/(||e||+1e-8) (face_embedder.py:133-134, 177-180).
//   l2norm_rows_kernel q/(||q||+1e-8) (gallery_manager.py:195).
//   topk_kernel        argsort(S)[::-1][:k] (gallery_manager.py:197) with the
//                      documented tie policy: score desc, then index asc.
#include "frhip_kernels.h"

#include <float.h>

namespace frhip {

constexpr int IMG = 112;
constexpr int STEM_C = 64;

// One block per (image, STEM_ROWS output rows).  LDS: STEM_ROWS+2 LUT-normalised input rows
// with a zero halo ([STEM_ROWS+2][IMG+2][3] floats) and the [27][64] weights.  Thread t owns 4
// output channels (t&15) of pixels (t>>4) + 16j of every row; its 27x4 weights live in
// registers for the whole block.  A wave writes 4 pixels x 256 B contiguous.  Per output the
// 27 FMAs run in (ky, kx, c) order, as before the row blocking.
constexpr int STEM_ROWS = 4;
static_assert(IMG % STEM_ROWS == 0, "rows per block must divide the image height");
__global__ __launch_bounds__(256) void stem_kernel(const uint8_t* __restrict__ img, const float* __restrict__ lut,
                                                   const float* __restrict__ w27x64,
                                                   const float* __restrict__ bn_scale,
                                                   const float* __restrict__ bn_shift,
                                                   const float* __restrict__ prelu, float* __restrict__ y) {
  __shared__ float s_lut[256];
  __shared__ __attribute__((aligned(16))) float s_w[27 * STEM_C];
  __shared__ float s_in[STEM_ROWS + 2][IMG + 2][3];
  constexpr int RB = IMG / STEM_ROWS;  // row blocks per image
  const int b = blockIdx.x / RB;
  const int oy0 = (blockIdx.x - b * RB) * STEM_ROWS;
  const int tid = threadIdx.x;
  s_lut[tid] = lut[tid];
  for (int i = tid; i < 27 * STEM_C; i += 256) s_w[i] = w27x64[i];
  __syncthreads();
  for (int i = tid; i < (STEM_ROWS + 2) * (IMG + 2) * 3; i += 256) {
    const int r = i / ((IMG + 2) * 3);
    const int rem = i - r * (IMG + 2) * 3;
    const int xx = rem / 3;
    const int c = rem - xx * 3;
    const int iy = oy0 + r - 1, ix = xx - 1;
    float v = 0.f;
    if ((unsigned)iy < IMG && (unsigned)ix < IMG) v = s_lut[img[(((long long)b * IMG + iy) * IMG + ix) * 3 + c]];
    s_in[r][xx][c] = v;
  }
  __syncthreads();
  const int cg = tid & 15;
  float4 w[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) w[t] = *reinterpret_cast<const float4*>(s_w + t * STEM_C + 4 * cg);
  const float4 sc = *reinterpret_cast<const float4*>(bn_scale + 4 * cg);
  const float4 sh = *reinterpret_cast<const float4*>(bn_shift + 4 * cg);
  const float4 al = *reinterpret_cast<const float4*>(prelu + 4 * cg);
  for (int r = 0; r < STEM_ROWS; ++r) {
    for (int px = tid >> 4; px < IMG; px += 16) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const float v = s_in[r + ky][px + kx][c];
            const float4 wt = w[(ky * 3 + kx) * 3 + c];
            acc.x = fmaf(v, wt.x, acc.x);
            acc.y = fmaf(v, wt.y, acc.y);
            acc.z = fmaf(v, wt.z, acc.z);
            acc.w = fmaf(v, wt.w, acc.w);
          }
      float4 o;
      o.x = acc.x * sc.x + sh.x;
      o.y = acc.y * sc.y + sh.y;
      o.z = acc.z * sc.z + sh.z;
      o.w = acc.w * sc.w + sh.w;
      o.x = o.x > 0.f ? o.x : o.x * al.x;
      o.y = o.y > 0.f ? o.y : o.y * al.y;
      o.z = o.z > 0.f ? o.z : o.z * al.z;
      o.w = o.w > 0.f ? o.w : o.w * al.w;
      *reinterpret_cast<float4*>(y + (((long long)b * IMG + oy0 + r) * IMG + px) * STEM_C + 4 * cg) = o;
    }
  }
}

hipError_t launch_stem(const uint8_t* img, int B, const float* lut, const float* w27x64, const float* bn_scale,
                       const float* bn_shift, const float* prelu, float* y, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(stem_kernel, dim3(B * (IMG / STEM_ROWS)), dim3(256), 0, s, img, lut, w27x64, bn_scale, bn_shift,
                     prelu, y);
  return hipGetLastError();
}

// Block-wide sum over 256 threads (4 waves of 64).
__device__ __forceinline__ float block_sum_256(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wid = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One block (256 threads, 2 columns each) per embedding row, D = 512.
__global__ __launch_bounds__(256) void head_reduce_kernel(const float* __restrict__ partial, int nsplit,
                                                          long long split_stride, const float* __restrict__ fc_bias,
                                                          const float* __restrict__ bn_scale,
                                                          const float* __restrict__ bn_shift, float* __restrict__ emb,
                                                          int normalize, int model_l2) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int c0 = threadIdx.x, c1 = threadIdx.x + 256;
  float v0 = 0.f, v1 = 0.f;
  const float* p = partial + (long long)row * 512;
  // eight splits' loads in flight at a time, summed in split order (deterministic)
  for (int s0 = 0; s0 < nsplit; s0 += 8) {
    float a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = s0 + u < nsplit;
      a0[u] = ok ? p[(long long)(s0 + u) * split_stride + c0] : 0.f;
      a1[u] = ok ? p[(long long)(s0 + u) * split_stride + c1] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < nsplit) {
        v0 += a0[u];
        v1 += a1[u];
      }
  }
  v0 += fc_bias[c0];
  v1 += fc_bias[c1];
  v0 = v0 * bn_scale[c0] + bn_shift[c0];
  v1 = v1 * bn_scale[c1] + bn_shift[c1];
  if (model_l2) {  // AdaFace forward tail x / ||x|| (ArcFace's model has none)
    const float norm = sqrtf(block_sum_256(v0 * v0 + v1 * v1, red));
    v0 = v0 / norm;
    v1 = v1 / norm;
  }
  if (normalize) {
    const float n2 = sqrtf(block_sum_256(v0 * v0 + v1 * v1, red)) + 1e-8f;
    v0 = v0 / n2;
    v1 = v1 / n2;
  }
  emb[(long long)row * 512 + c0] = v0;
  emb[(long long)row * 512 + c1] = v1;
}

hipError_t launch_head_reduce(const float* partial, int nsplit, long long split_stride, const float* fc_bias,
                              const float* bn_scale, const float* bn_shift, float* emb, int n, int normalize,
                              int model_l2, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(head_reduce_kernel, dim3(n), dim3(256), 0, s, partial, nsplit, split_stride, fc_bias, bn_scale,
                     bn_shift, emb, normalize, model_l2);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void l2norm_rows_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                          int d) {
  __shared__ float red[4];
  const float* r = q + (long long)blockIdx.x * d;
  float ss = 0.f;
  for (int c = threadIdx.x; c < d; c += 256) ss += r[c] * r[c];
  const float nrm = sqrtf(block_sum_256(ss, red)) + 1e-8f;
  for (int c = threadIdx.x; c < d; c += 256) out[(long long)blockIdx.x * d + c] = r[c] / nrm;
}

hipError_t launch_l2norm_rows(const float* q, float* out, int n, int d, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3(n), dim3(256), 0, s, q, out, d);
  return hipGetLastError();
}

// (score, index) total order: a before b  <=>  a.s > b.s || (a.s == b.s && a.i > b.i).
// Equal scores rank the HIGHER gallery row first: that is np.argsort(s)[::-1] (the reference,
// gallery_manager.py:197) whenever numpy's sort is stable -- its insertion sort for <= 16
// elements, or kind="stable" -- i.e. a stable ascending sort, reversed.  (numpy's AVX-512
// argsort leaves ties in no defined order)  NO_ROW ranks after any real row.
constexpr int NO_ROW = -1;
__device__ __forceinline__ bool ranks_before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia > ib);
}

// One wave per score row; k selection passes, each a strided scan for the best
// element ranked strictly after the previous pick, then a wave arg-reduction.
// Exact and order-independent (the result never depends on scan order).
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ scores, int n, int G, int k,
                                                   int32_t* __restrict__ idx, float* __restrict__ val) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const int lane = threadIdx.x & 63;
  const float* r = scores + (long long)row * G;
  float prev_s = INFINITY;
  int prev_i = 0x7fffffff;  // ranks before every (score, row), +inf included
  for (int t = 0; t < k; ++t) {
    float bs = -INFINITY;
    int bi = NO_ROW;
    for (int g = lane; g < G; g += 64) {
      const float s = r[g];
      if (s != s) continue;  // NaN never ranks
      if (ranks_before(prev_s, prev_i, s, g) && ranks_before(s, g, bs, bi)) {
        bs = s;
        bi = g;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ranks_before(os, oi, bs, bi)) {
        bs = os;
        bi = oi;
      }
    }
    if (lane == 0) {
      idx[(long long)row * k + t] = bi < 0 ? -1 : bi;
      val[(long long)row * k + t] = bs;
    }
    prev_s = bs;
    prev_i = bi;
  }
}

// Single-pass form for k <= KMAX: one 256-thread block per row.  Each thread keeps its
// best KMAX (score, index) pairs of a strided slice in registers (unrolled insertion, no
// runtime-indexed arrays), then k block-wide arg-max rounds pop the global best in order.
template <int KMAX>
__global__ __launch_bounds__(256) void topk_small_kernel(const float* __restrict__ scores, int G, int k,
                                                         int32_t* __restrict__ idx, float* __restrict__ val) {
  __shared__ float s_s[4];
  __shared__ int s_i[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* r = scores + (long long)row * G;
  float ls[KMAX];
  int li[KMAX];
#pragma unroll
  for (int j = 0; j < KMAX; ++j) {
    ls[j] = -INFINITY;
    li[j] = NO_ROW;
  }
  auto push = [&](float sv, int iv) {
    if (sv != sv || !ranks_before(sv, iv, ls[KMAX - 1], li[KMAX - 1])) return;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {  // bubble the new pair into the sorted list
      if (ranks_before(sv, iv, ls[j], li[j])) {
        const float ts = ls[j];
        const int ti = li[j];
        ls[j] = sv;
        li[j] = iv;
        sv = ts;
        iv = ti;
      }
    }
  };
  const bool vec = (G & 3) == 0 && (((unsigned long long)r) & 15) == 0;
  if (vec) {
    const float4* r4 = reinterpret_cast<const float4*>(r);
    for (int g = tid; g < G / 4; g += 256) {
      const float4 v = r4[g];
      push(v.x, 4 * g);
      push(v.y, 4 * g + 1);
      push(v.z, 4 * g + 2);
      push(v.w, 4 * g + 3);
    }
  } else {
    for (int g = tid; g < G; g += 256) push(r[g], g);
  }
  // k rounds of block arg-max over the list heads; the owning thread pops its head
  for (int t = 0; t < k; ++t) {
    float bs = ls[0];
    int bi = li[0];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ranks_before(os, oi, bs, bi)) {
        bs = os;
        bi = oi;
      }
    }
    if (lane == 0) {
      s_s[wid] = bs;
      s_i[wid] = bi;
    }
    __syncthreads();
    bs = s_s[0];
    bi = s_i[0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
      if (ranks_before(s_s[w], s_i[w], bs, bi)) {
        bs = s_s[w];
        bi = s_i[w];
      }
    __syncthreads();
    if (tid == 0) {
      idx[(long long)row * k + t] = bi < 0 ? -1 : bi;
      val[(long long)row * k + t] = bs;
    }
    if (li[0] == bi && bi >= 0) {  // indices are unique: exactly one owner pops
#pragma unroll
      for (int j = 0; j < KMAX - 1; ++j) {
        ls[j] = ls[j + 1];
        li[j] = li[j + 1];
      }
      ls[KMAX - 1] = -INFINITY;
      li[KMAX - 1] = NO_ROW;
    }
  }
}

hipError_t launch_topk(const float* scores, int n, int G, int k, int32_t* idx, float* val, hipStream_t s) {
  if (n <= 0 || k <= 0) return hipSuccess;
  if (k <= 8) {
    hipLaunchKernelGGL(topk_small_kernel<8>, dim3(n), dim3(256), 0, s, scores, G, k, idx, val);
  } else {
    hipLaunchKernelGGL(topk_kernel, dim3((n + 3) / 4), dim3(256), 0, s, scores, n, G, k, idx, val);
  }
  return hipGetLastError();
}

}  // namespace frhip
