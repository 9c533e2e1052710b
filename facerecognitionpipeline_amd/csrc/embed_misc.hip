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
//                      documented tie policy: score desc, then gallery row desc.
#include "frhip_kernels.h"

#include <float.h>

namespace frhip {

constexpr int IMG = 112;
constexpr int STEM_C = 64;

// One block (4 waves) per (image, STEM_ROWS output rows).  The 3x3x3 -> 64 conv is a GEMM with
// K = 27 (padded to 28 with a zero tap) on v_mfma_f32_16x16x4_f32: the weights are the A operand
// (16 output channels x 4 taps per fragment, 28 registers per lane for all 64 channels, loaded
// once), the im2col of 16 pixels the B operand (one ds_read_b32 per lane and K-step from the
// LUT-normalised input rows staged in LDS with a zero halo), so a lane's accumulator holds 4
// consecutive channels of one pixel and every store is 16 bytes.  An f32 MFMA accumulates its 4
// products as a chain of fmaf (bitwise), so with K in (ky, kx, c) order each output is the same
// fmaf sequence as the scalar 27-tap loop it replaces; the padded tap adds 0 * x.  Per 16 pixels x
// 64 channels: 28 MFMAs (the VALU version's 1,728 FMAs), 7 LDS reads, 4 stores; the kernel is
// bound by its 822 MB (B = 256) output write.
// STEM_ROWS output rows per block: 16 for batches (fewer halo rows re-read), 4 for serving
// batches of <= 8 crops, whose 7 blocks per image would leave the chip idle (batch 1: 26 -> 9 us)
constexpr int STEM_W = IMG + 2;  // staged row width with the halo
typedef float stem_f4 __attribute__((ext_vector_type(4)));
template <int STEM_ROWS>
__global__ __launch_bounds__(256) void stem_kernel(const uint8_t* __restrict__ img, const float* __restrict__ lut,
                                                   const float* __restrict__ w27x64,
                                                   const float* __restrict__ bn_scale,
                                                   const float* __restrict__ bn_shift,
                                                   const float* __restrict__ prelu, float* __restrict__ y) {
  static_assert(IMG % STEM_ROWS == 0 && IMG % 16 == 0, "row blocks and 16-pixel groups must tile the image");
  __shared__ float s_lut[256];
  __shared__ float s_in[(STEM_ROWS + 2) * STEM_W * 3 + 1];  // + one zero cell for the padded tap
  // per-wave output transpose: [16 pixels][64 channels + 4 pad] (MFMA layout in, row-major out)
  __shared__ __attribute__((aligned(16))) float s_out[4][16 * 68];
  constexpr int RB = IMG / STEM_ROWS;  // row blocks per image
  constexpr int NIN = (STEM_ROWS + 2) * STEM_W * 3;
  const int b = blockIdx.x / RB;
  const int oy0 = (blockIdx.x - b * RB) * STEM_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  s_lut[tid] = lut[tid];
  // weights as A fragments: lane (cout m = lane & 15, tap group kk = lane >> 4), K-step s holds
  // tap 4 s + kk of channel 16 cb + m (tap 27 = 0)
  const int m = lane & 15, kk = lane >> 4;
  float wa[4][7];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = 4 * st + kk;
      wa[cb][st] = k < 27 ? w27x64[k * STEM_C + 16 * cb + m] : 0.f;
    }
  // the block's STEM_ROWS + 2 input rows are whole image rows (336 contiguous bytes each): all
  // their dwords are loaded at once (one memory latency, not one per byte), then unpacked
  // through the LUT into the zero-haloed LDS rows
  constexpr int RDW = IMG * 3 / 4;                         // dwords per image row
  constexpr int NDW = (STEM_ROWS + 2) * RDW;
  constexpr int PER = (NDW + 255) / 256;
  const unsigned* src = reinterpret_cast<const unsigned*>(img + (size_t)b * IMG * IMG * 3);
  unsigned raw[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = tid + 256 * k;
    const int r = i / RDW, iy = oy0 + r - 1;
    raw[k] = i < NDW && (unsigned)iy < IMG ? src[iy * RDW + (i - r * RDW)] : 0u;
  }
  for (int i = tid; i < (STEM_ROWS + 2) * 2 * 3 + 1; i += 256) {  // halo columns and the zero cell
    const int r = i / 6, e = i - r * 6;
    s_in[i < (STEM_ROWS + 2) * 6 ? (r * STEM_W + (e < 3 ? 0 : STEM_W - 1)) * 3 + e % 3 : NIN] = 0.f;
  }
  __syncthreads();  // s_lut (the row loads above are already in flight)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = tid + 256 * k;
    if (i < NDW) {
      const int r = i / RDW, q = 4 * (i - r * RDW);  // first byte of the dword within the row
      const bool in = (unsigned)(oy0 + r - 1) < IMG;   // rows above / below the image: zero padding
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int xb = q + e, ix = xb / 3;
        s_in[(r * STEM_W + ix + 1) * 3 + (xb - ix * 3)] = in ? s_lut[(raw[k] >> (8 * e)) & 255u] : 0.f;
      }
    }
  }
  __syncthreads();
  // the lane's im2col offsets: tap k = (ky * 3 + kx) * 3 + c at staged (row ky, column kx, c)
  int koff[7];
#pragma unroll
  for (int st = 0; st < 7; ++st) {
    const int k = 4 * st + kk;
    const int ky = k / 9, kx = (k / 3) % 3, c = k % 3;
    koff[st] = k < 27 ? (ky * STEM_W + kx) * 3 + c : -1;
  }
  const int rg = lane >> 4;  // this lane's output channels: 16 cb + 4 rg .. + 3
  // PReLU as med3(t, a t, c) with c = +inf for a slope a <= 1 (= max(t, a t)) and -inf for
  // a > 1 (= min(t, a t)): t > 0 ? t : a t exactly (med3 returns one of its operands), in two
  // instructions instead of a multiply, a compare and a select
  stem_f4 sc[4], sh[4], al[4], cl[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    sc[cb] = *reinterpret_cast<const stem_f4*>(bn_scale + 16 * cb + 4 * rg);
    sh[cb] = *reinterpret_cast<const stem_f4*>(bn_shift + 16 * cb + 4 * rg);
    al[cb] = *reinterpret_cast<const stem_f4*>(prelu + 16 * cb + 4 * rg);
#pragma unroll
    for (int e = 0; e < 4; ++e) cl[cb][e] = al[cb][e] <= 1.f ? INFINITY : -INFINITY;
  }
  // 16-pixel groups of the block (STEM_ROWS rows x 7), round-robin over the 4 waves
  for (int grp = wv; grp < STEM_ROWS * (IMG / 16); grp += 4) {
    const int r = grp / (IMG / 16), px = (grp - r * (IMG / 16)) * 16 + m;
    const int base = (r * STEM_W + px) * 3;
    float bv[7];
#pragma unroll
    for (int st = 0; st < 7; ++st) bv[st] = s_in[koff[st] < 0 ? NIN : base + koff[st]];
    stem_f4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      acc[cb] = stem_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 7; ++st) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[cb][st], bv[st], acc[cb], 0, 0, 0);
    }
    // through the wave's LDS tile, so each store writes 4 whole 256-byte pixel rows (1 KiB
    // contiguous) instead of 16 scattered 64-byte pieces
    float* so = s_out[wv];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      stem_f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = acc[cb][e] * sc[cb][e] + sh[cb][e];
        o[e] = __builtin_amdgcn_fmed3f(t, t * al[cb][e], cl[cb][e]);
      }
      *reinterpret_cast<stem_f4*>(so + m * 68 + 16 * cb + 4 * rg) = o;
    }
    float* out = y + (((size_t)b * IMG + oy0 + r) * IMG + px - m) * STEM_C;  // the group's first pixel
    // plain stores: nontemporal ones measured 194 -> 191 us on the stem alone but 149 -> 184 us
    // inside the forward
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pp = 4 * j + (lane >> 4);  // pixel of the group, 16-byte channel piece lane & 15
      *reinterpret_cast<stem_f4*>(out + pp * STEM_C + 4 * (lane & 15)) =
          *reinterpret_cast<const stem_f4*>(so + pp * 68 + 4 * (lane & 15));
    }
  }
}

hipError_t launch_stem(const uint8_t* img, int B, const float* lut, const float* w27x64, const float* bn_scale,
                       const float* bn_shift, const float* prelu, float* y, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (B <= 8)
    hipLaunchKernelGGL(stem_kernel<4>, dim3(B * (IMG / 4)), dim3(256), 0, s, img, lut, w27x64, bn_scale, bn_shift,
                       prelu, y);
  else
    hipLaunchKernelGGL(stem_kernel<16>, dim3(B * (IMG / 16)), dim3(256), 0, s, img, lut, w27x64, bn_scale,
                       bn_shift, prelu, y);
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

// Block-wide sum over 1024 threads whose waves 4..15 hold zeros: the same value as
// block_sum_256 over waves 0..3 (the extra terms add exact zeros).
__device__ __forceinline__ float block_sum_1024(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wid = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  float r = (red[0] + red[1]) + (red[2] + red[3]);
#pragma unroll
  for (int w = 4; w < 16; ++w) r += red[w];
  return r;
}

// One block per embedding row, D = 512: 4 groups of 256 threads (2 columns per thread) sum
// split ranges g*nsplit/4 .. (g+1)*nsplit/4 with eight loads in flight each, and the group sums
// are added in group order (deterministic).  One group per row walked all splits in turn: the
// 196-split serving FC's reduce took 15 us at batch 1, a chain of 25 load latencies.
__global__ __launch_bounds__(1024) void head_reduce_kernel(const float* __restrict__ partial, int nsplit,
                                                           long long split_stride, const float* __restrict__ fc_bias,
                                                           const float* __restrict__ bn_scale,
                                                           const float* __restrict__ bn_shift, float* __restrict__ emb,
                                                           int normalize, int model_l2) {
  __shared__ float part[3][512];
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int g = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int c0 = t, c1 = t + 256;
  float v0 = 0.f, v1 = 0.f;
  const float* p = partial + (long long)row * 512;
  const int s_lo = g * nsplit / 4, s_hi = (g + 1) * nsplit / 4;
  for (int s0 = s_lo; s0 < s_hi; s0 += 8) {
    float a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = s0 + u < s_hi;
      a0[u] = ok ? p[(long long)(s0 + u) * split_stride + c0] : 0.f;
      a1[u] = ok ? p[(long long)(s0 + u) * split_stride + c1] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < s_hi) {
        v0 += a0[u];
        v1 += a1[u];
      }
  }
  if (g > 0) {
    part[g - 1][c0] = v0;
    part[g - 1][c1] = v1;
  }
  __syncthreads();
  // group 0 finishes the row; the other groups stay for the block-wide norms with zeros (x + 0
  // is exact, so the sums are those of group 0's four waves)
  if (g == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v0 += part[k][c0];
      v1 += part[k][c1];
    }
    v0 += fc_bias[c0];
    v1 += fc_bias[c1];
    v0 = v0 * bn_scale[c0] + bn_shift[c0];
    v1 = v1 * bn_scale[c1] + bn_shift[c1];
  } else {
    v0 = v1 = 0.f;
  }
  if (model_l2) {  // AdaFace forward tail x / ||x|| (ArcFace's model has none)
    const float norm = sqrtf(block_sum_1024(v0 * v0 + v1 * v1, red));
    v0 = v0 / norm;
    v1 = v1 / norm;
  }
  if (normalize) {
    const float n2 = sqrtf(block_sum_1024(v0 * v0 + v1 * v1, red)) + 1e-8f;
    v0 = v0 / n2;
    v1 = v1 / n2;
  }
  if (g == 0) {
    emb[(long long)row * 512 + c0] = v0;
    emb[(long long)row * 512 + c1] = v1;
  }
}

hipError_t launch_head_reduce(const float* partial, int nsplit, long long split_stride, const float* fc_bias,
                              const float* bn_scale, const float* bn_shift, float* emb, int n, int normalize,
                              int model_l2, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(head_reduce_kernel, dim3(n), dim3(1024), 0, s, partial, nsplit, split_stride, fc_bias, bn_scale,
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
__device__ __forceinline__ void topk_row_small(const float* __restrict__ r, int G, int k, int32_t* __restrict__ idx,
                                               float* __restrict__ val, float* s_s, int* s_i) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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
      idx[t] = bi < 0 ? -1 : bi;
      val[t] = bs;
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

template <int KMAX>
__global__ __launch_bounds__(256) void topk_small_kernel(const float* __restrict__ scores, int G, int k,
                                                         int32_t* __restrict__ idx, float* __restrict__ val) {
  __shared__ float s_s[4];
  __shared__ int s_i[4];
  const int row = blockIdx.x;
  topk_row_small<KMAX>(scores + (long long)row * G, G, k, idx + (long long)row * k, val + (long long)row * k, s_s, s_i);
}

// Serving-sized match scores: block (64 gallery rows, query q) of 256 threads.  The query is
// normalised exactly as l2norm_rows_kernel does it (same per-thread terms, same block reduction),
// kept in LDS, and each group of 4 lanes dots one gallery row, a quarter of the 512 dimensions per
// lane (32 float4 loads, 8 in flight), the quarters summed in a fixed order.  For n <= 16 it
// replaces l2norm + the implicit-GEMM score launch (a stream-K grid over a 1-row M): batch-1
// embed + match 1.823 -> 1.810 ms.  (Taking the top-k in the query's last-arriving block as well
// -- release, arrival ticket, acquire -- measured the same 1.810 ms as the separate top-k launch.)
__global__ __launch_bounds__(256) void scores_small_kernel(const float* __restrict__ q,
                                                           const float* __restrict__ gallery, int G,
                                                           float* __restrict__ scores) {
  __shared__ float red[4];
  __shared__ __attribute__((aligned(16))) float qn[512];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int qi = blockIdx.y;
  const float* r = q + (long long)qi * 512;
  const float r0 = r[tid], r1 = r[tid + 256];
  const float nrm = sqrtf(block_sum_256(r0 * r0 + r1 * r1, red)) + 1e-8f;
  qn[tid] = r0 / nrm;
  qn[tid + 256] = r1 / nrm;
  __syncthreads();
  const int row = blockIdx.x * 64 + w * 16 + (lane & 15), part = lane >> 4;
  float acc = 0.f;
  if (row < G) {
    const float4* g4 = reinterpret_cast<const float4*>(gallery + (long long)row * 512 + part * 128);
    const float4* q4 = reinterpret_cast<const float4*>(qn + part * 128);
    for (int c0 = 0; c0 < 32; c0 += 8) {
      float4 a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = g4[c0 + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 b = q4[c0 + u];
        acc = fmaf(a[u].x, b.x, acc);
        acc = fmaf(a[u].y, b.y, acc);
        acc = fmaf(a[u].z, b.z, acc);
        acc = fmaf(a[u].w, b.w, acc);
      }
    }
  }
  // quarters in order: (p0 + p1) + (p2 + p3)
  const float o1 = __shfl_xor(acc, 16, 64);
  const float s01 = (lane & 16) ? o1 + acc : acc + o1;
  const float o2 = __shfl_xor(s01, 32, 64);
  const float sum = (lane & 32) ? o2 + s01 : s01 + o2;
  if (part == 0 && row < G) scores[(long long)qi * G + row] = sum;
}

hipError_t launch_scores_small(const float* q, const float* gallery, int G, float* scores, int n, hipStream_t s) {
  if (n <= 0 || G <= 0) return hipSuccess;
  if (n > 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scores_small_kernel, dim3((G + 63) / 64, n), dim3(256), 0, s, q, gallery, G, scores);
  return hipGetLastError();
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
