// Gallery template construction on gfx950: GalleryManager._aggregate_embeddings
// (gallery_manager.py:297-317) with its quality filter _filter_quality_embeddings
// (:104-122), for a whole batch of students at once (bulk enrollment, SURVEY.md
// §8(f) rank 3).  One workgroup per student; the student's N sample rows are a
// CSR slice of one [total][512] f32 matrix in HBM.
//
//   N == 1            template = row 0, not normalised (:298-299)
//   N > 2             S = E.E^T, diag := 0, avg_i = mean_j S_ij (over all N),
//                     keep avg_i >= min_similarity, else the two largest avg
//   mean              t = (sum of kept rows, in row order) / n_kept
//   median            per column: middle value, or (a + b) / 2 of the two middle
//   weighted_mean     w_i = mean_j (E_k.E_k^T)_ij (diag kept), w /= sum w,
//                     t = sum_i E_i * w_i
//   then              t / (||t|| + 1e-8)
//
// The element-wise steps round like numpy's float32 ufuncs (separate mul / add,
// row-sequential axis-0 sums, correctly rounded div/sqrt); the Gram dot products
// are f32 wave reductions, so avg_i agrees with numpy's BLAS to ~1e-7, not bit
// for bit (a threshold decision could differ only within that of 0.70).
#include "frhip_kernels.h"

#pragma clang fp contract(off)

namespace frhip {

namespace {

// dot(E[i], E[j]) over 512 floats: lane l holds elements 8l..8l+7 of row i.
__device__ __forceinline__ float wave_dot(const float (&ei)[8], const float* __restrict__ ej, int lane) {
  const float4 a = *reinterpret_cast<const float4*>(ej + lane * 8);
  const float4 b = *reinterpret_cast<const float4*>(ej + lane * 8 + 4);
  float d = ei[0] * a.x + ei[1] * a.y + ei[2] * a.z + ei[3] * a.w + ei[4] * b.x + ei[5] * b.y + ei[6] * b.z +
            ei[7] * b.w;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
  return d;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace

__global__ __launch_bounds__(256) void template_kernel(const float* __restrict__ emb, const int* __restrict__ offsets,
                                                       int method, float min_sim, float* __restrict__ out,
                                                       int* __restrict__ kept_out) {
  __shared__ float avg[TEMPLATE_MAX_SAMPLES];
  __shared__ int keep_idx[TEMPLATE_MAX_SAMPLES];
  __shared__ float red[4];
  __shared__ int s_cnt;
  const int st = blockIdx.x;
  const int r0 = offsets[st];
  const int N = offsets[st + 1] - r0;
  const float* __restrict__ E = emb + (long long)r0 * 512;
  float* __restrict__ T = out + (long long)st * 512;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (N == 1) {  // single sample: the row itself
    T[t] = E[t];
    T[t + 256] = E[t + 256];
    if (kept_out && t == 0) kept_out[st] = 1;
    return;
  }
  // ---- quality filter
  if (N <= 2) {
    if (t < N) keep_idx[t] = t;
    if (t == 0) s_cnt = N;
  } else {
    for (int i = wv; i < N; i += 4) {
      float ei[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ei[e] = E[(long long)i * 512 + lane * 8 + e];
      float acc = 0.f;
      for (int j = 0; j < N; ++j) {
        const float d = j == i ? 0.f : wave_dot(ei, E + (long long)j * 512, lane);
        acc += d;
      }
      if (lane == 0) avg[i] = acc / (float)N;
    }
    __syncthreads();
    if (t == 0) {
      int c = 0;
      for (int i = 0; i < N; ++i)
        if (avg[i] >= min_sim) keep_idx[c++] = i;
      if (c < 2) {  // np.argsort(avg)[-2:]: the two largest; ties take the higher index, as a stable sort
        // would (numpy's default argsort leaves tie order unspecified)
        int a = -1, b = -1;
        for (int i = 0; i < N; ++i) {
          if (a < 0 || avg[i] >= avg[a]) {
            b = a;
            a = i;
          } else if (b < 0 || avg[i] >= avg[b]) {
            b = i;
          }
        }
        keep_idx[0] = b < a ? b : a;  // row order (sums below are order-free for 2 rows)
        keep_idx[1] = b < a ? a : b;
        c = 2;
      }
      s_cnt = c;
    }
  }
  __syncthreads();
  const int cnt = s_cnt;
  if (kept_out && t == 0) kept_out[st] = cnt;
  // ---- aggregate (thread t owns columns t and t + 256)
  float v0 = 0.f, v1 = 0.f;
  if (method == TEMPLATE_MEDIAN) {
    const int m_lo = (cnt - 1) / 2, m_hi = cnt / 2;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int c = t + half * 256;
      float lo = 0.f, hi = 0.f;
      for (int a = 0; a < cnt; ++a) {
        const float va = E[(long long)keep_idx[a] * 512 + c];
        int rank = 0;
        for (int b = 0; b < cnt; ++b) {
          const float vb = E[(long long)keep_idx[b] * 512 + c];
          rank += (vb < va) || (vb == va && b < a);
        }
        if (rank == m_lo) lo = va;
        if (rank == m_hi) hi = va;
      }
      const float v = m_lo == m_hi ? lo : (lo + hi) / 2.0f;
      if (half == 0)
        v0 = v;
      else
        v1 = v;
    }
  } else if (method == TEMPLATE_WEIGHTED_MEAN) {
    // weights over the kept rows, diagonal included
    for (int a = wv; a < cnt; a += 4) {
      float ei[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ei[e] = E[(long long)keep_idx[a] * 512 + lane * 8 + e];
      float acc = 0.f;
      for (int b = 0; b < cnt; ++b) acc += wave_dot(ei, E + (long long)keep_idx[b] * 512, lane);
      if (lane == 0) avg[a] = acc / (float)cnt;
    }
    __syncthreads();
    float wsum = 0.f;
    for (int a = 0; a < cnt; ++a) wsum += avg[a];
    for (int a = 0; a < cnt; ++a) {
      const float w = avg[a] / wsum;
      const float* row = E + (long long)keep_idx[a] * 512;
      v0 = v0 + row[t] * w;
      v1 = v1 + row[t + 256] * w;
    }
  } else {  // mean (also the reference's fallback for unknown methods)
    for (int a = 0; a < cnt; ++a) {
      const float* row = E + (long long)keep_idx[a] * 512;
      v0 += row[t];
      v1 += row[t + 256];
    }
    v0 = v0 / (float)cnt;
    v1 = v1 / (float)cnt;
  }
  const float nrm = sqrtf(block_sum(v0 * v0 + v1 * v1, red)) + 1e-8f;
  T[t] = v0 / nrm;
  T[t + 256] = v1 / nrm;
}

hipError_t launch_templates(const float* emb, const int* offsets, int n_students, int method, float min_sim,
                            float* out, int* kept, hipStream_t s) {
  if (n_students <= 0) return hipSuccess;
  hipLaunchKernelGGL(template_kernel, dim3(n_students), dim3(256), 0, s, emb, offsets, method, min_sim, out, kept);
  return hipGetLastError();
}

}  // namespace frhip
