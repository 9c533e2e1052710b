// Does f32 MFMA on one wave overlap with f32 VALU on another wave of the same SIMD?
// 512-thread workgroups (2 waves per SIMD): waves 0-3 run N MFMAs (v_mfma_f32_16x16x4_f32,
// 4 independent accumulators), waves 4-7 run M independent v_fma_f32 per lane-chain.
// usage: mfma_valu_overlap  (prints us for mfma-only, valu-only, both)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool DO_MFMA, bool DO_VALU, bool PK = false>
__global__ __launch_bounds__(512, 1) void k(float* out, int n_mfma, int n_valu, float s) {
  const int wid = threadIdx.x >> 6;
  if (wid < 4) {
    if (!DO_MFMA) return;
    f4 a0 = {s, s, s, s}, a1 = a0, a2 = a0, a3 = a0;
    float x = s * threadIdx.x, y = s + threadIdx.x;
    for (int i = 0; i < n_mfma; i += 4) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a3, 0, 0, 0);
    }
    const f4 r = a0 + a1 + a2 + a3;
    if (r.x == 1234.5f) out[threadIdx.x] = r.y;
  } else {
    if (!DO_VALU) return;
    if constexpr (PK) {  // the same flops as n_valu scalar fmas, 2 per v_pk_fma_f32
      f2 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = f2{s * (threadIdx.x + j), s + j};
      const f2 m = {s, s}, c = {0.5f, 0.5f};
      for (int i = 0; i < n_valu; i += 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = __builtin_elementwise_fma(v[j], m, c);
      }
      float r = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) r += v[j].x + v[j].y;
      if (r == 1234.5f) out[threadIdx.x] = r;
    } else {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = s * (threadIdx.x + j);
      for (int i = 0; i < n_valu; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = __builtin_fmaf(v[j], s, 0.5f);
      }
      float r = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) r += v[j];
      if (r == 1234.5f) out[threadIdx.x] = r;
    }
  }
}

template <bool A, bool B, bool PK = false>
float run(float* out, int nm, int nv) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k<A, B, PK>), dim3(256), dim3(512), 0, 0, out, nm, nv, 1.0001f);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<A, B, PK>), dim3(256), dim3(512), 0, 0, out, nm, nv, 1.0001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000 / 5;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  const int nm = 8192;  // MFMAs per wave: 8192 * 32 cyc = 262k cyc
  for (int nv : {2048, 8192, 16384, 32768}) {
    const float tm = run<true, false>(out, nm, nv), tv = run<false, true>(out, nm, nv), tb = run<true, true>(out, nm, nv);
    printf("mfma %d/wave: %.1f us | valu %d fma/wave: %.1f us | both: %.1f us (sum %.1f)\n", nm, tm, nv, tv, tb, tm + tv);
    const float pv = run<false, true, true>(out, nm, nv), pb = run<true, true, true>(out, nm, nv);
    printf("   packed: valu %d fma-equivalents/wave: %.1f us | both: %.1f us (sum %.1f)\n", nv, pv, pb, tm + pv);
  }
  return 0;
}
