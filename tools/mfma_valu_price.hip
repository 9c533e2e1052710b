// Price of VALU instructions issued by one wave beside an f32-MFMA wave on the same SIMD, in the
// shape of the F(4x4) kernel's K-step: 512-thread workgroups, one per CU; waves 0-3 issue 144
// v_mfma_f32_16x16x4_f32 per step (36 independent accumulators, as the MFMA waves do), waves 4-7
// issue a per-step VALU mix; both meet at one s_barrier per step (or not, SYNC = 0).
// Prints cycles per step (s_memtime, median wave) for each mix.
// usage: mfma_valu_price
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int STEPS = 64;

// MIX: 0 none, 1 72 v_pk_fma_f32, 2 144 v_fma_f32, 3 72 v_pk_fma + 18 v_permlane32_swap,
//      4 18 v_permlane32_swap, 5 36 v_pk_fma_f32, 6 72 v_fma_f32
template <int MIX, bool SYNC, bool MFMA>
__global__ __launch_bounds__(512, 1) void k(unsigned long long* cyc, float s) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wid < 4) {
    f4 acc[36];
#pragma unroll
    for (int x = 0; x < 36; ++x) acc[x] = f4{s, s, s, s};
    const float a = s * lane, b = s + lane;
    for (int g = 0; g < STEPS; ++g) {
      if constexpr (MFMA) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int x = 0; x < 36; ++x) acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[x], 0, 0, 0);
      }
      if constexpr (SYNC) __builtin_amdgcn_s_barrier();
    }
    float r = 0.f;
#pragma unroll
    for (int x = 0; x < 36; ++x) r += acc[x][0];
    if (r == 1234.5f) cyc[4096] = 1;
  } else {
    f2 v[12];
    float w[24];
#pragma unroll
    for (int j = 0; j < 12; ++j) v[j] = f2{s * (lane + j), s + j};
#pragma unroll
    for (int j = 0; j < 24; ++j) w[j] = s * (lane + 3 * j);
    const f2 m2 = {s, s}, c2 = {0.5f, 0.5f};
    for (int g = 0; g < STEPS; ++g) {
      if constexpr (MIX == 1 || MIX == 3 || MIX == 5) {
#pragma unroll
        for (int i = 0; i < (MIX == 5 ? 3 : 6); ++i)
#pragma unroll
          for (int j = 0; j < 12; ++j) v[j] = __builtin_elementwise_fma(v[j], m2, c2);
      }
      if constexpr (MIX == 2 || MIX == 6) {
#pragma unroll
        for (int i = 0; i < (MIX == 2 ? 6 : 3); ++i)
#pragma unroll
          for (int j = 0; j < 24; ++j) w[j] = __builtin_fmaf(w[j], s, 0.5f);
      }
      if constexpr (MIX == 3 || MIX == 4) {
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j].x), __float_as_uint(v[j].y), false, false);
          v[j] = f2{__uint_as_float(r[0]), __uint_as_float(r[1])};
        }
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j + 3].y), __float_as_uint(v[j + 3].x), false, false);
          v[j + 3] = f2{__uint_as_float(r[1]), __uint_as_float(r[0])};
        }
      }
      if constexpr (SYNC) __builtin_amdgcn_s_barrier();
    }
    float r = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) r += v[j].x + v[j].y;
#pragma unroll
    for (int j = 0; j < 24; ++j) r += w[j];
    if (r == 1234.5f) cyc[4097] = 1;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 8 + wid] = t1 - t0;
}

template <int MIX, bool SYNC, bool MFMA>
void run(const char* name, unsigned long long* d) {
  std::vector<unsigned long long> h(256 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<MIX, SYNC, MFMA>), dim3(256), dim3(512), 0, 0, d, 1.0001f);
  hipDeviceSynchronize();
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> m, v;
  for (int b = 0; b < 256; ++b)
    for (int w = 0; w < 8; ++w) (w < 4 ? m : v).push_back(h[b * 8 + w]);
  std::sort(m.begin(), m.end());
  std::sort(v.begin(), v.end());
  printf("%-34s %s  MFMA waves %7.0f cyc/step   VALU waves %7.0f cyc/step\n", name, SYNC ? "barrier" : "free   ",
         (double)m[m.size() / 2] / STEPS, (double)v[v.size() / 2] / STEPS);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 8192 * 8);
  run<0, true, true>("144 MFMA alone", d);
  run<1, true, false>("72 v_pk_fma alone", d);
  run<2, true, false>("144 v_fma alone", d);
  run<3, true, false>("72 pk_fma + 18 permlane alone", d);
  run<1, true, true>("144 MFMA + 72 v_pk_fma", d);
  run<2, true, true>("144 MFMA + 144 v_fma", d);
  run<3, true, true>("144 MFMA + 72 pk_fma + 18 permlane", d);
  run<4, true, true>("144 MFMA + 18 permlane", d);
  run<5, true, true>("144 MFMA + 36 v_pk_fma", d);
  run<6, true, true>("144 MFMA + 72 v_fma", d);
  run<1, false, true>("144 MFMA + 72 v_pk_fma", d);
  run<2, false, true>("144 MFMA + 144 v_fma", d);
  run<3, false, true>("144 MFMA + 72 pk_fma + 18 permlane", d);
  return 0;
}
