// L2 channel spread of the serving conv kernel's fragment loads (tools only, never shipped).
// Each wave issues 36 buffer_load_dwordx4 of 16 rows x 64 B (row stride S bytes), 12 loads in
// flight, like convs_kernel's weight and input
// fragments at IR-101 stage 3 (S = 9216: a weight row; S = 1024: an NHWC pixel of 256 channels):
// wave w's k-th load is chunk 4k + w, 64 B along the rows.
// 208 workgroups of 4 waves; workgroups g = x + 8 s share rows by (x, s / 13) as the kernel's
// cout blocks do.  Prints us per launch (back to back, 200 launches) per stride.
//   hipcc --offload-arch=gfx950 -O3 tools/l2_stride_bench.hip -o tools/wv/l2_stride_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void frag_loads(const float* base, long long bytes, int S, int contiguous, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = blockIdx.x;
  const int grp = (g & 7) + 8 * ((g >> 3) / 13);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, 0x00020000);
  // row-strided: lane (row l & 15, quad l >> 4); contiguous: lane l reads 16 B at 16 l of a 1-KiB block
  const int lbase = contiguous ? grp * 16 * S + lane * 16 : grp * 16 * S + (lane & 15) * S + (lane >> 4) * 16;
  const int step = contiguous ? 1024 : 64;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  u32x4 v[CH];
#pragma unroll
  for (int d = 0; d < CH; ++d) v[d] = __builtin_amdgcn_raw_buffer_load_b128(r, lbase + (4 * d + w) * step, 0, 0);
  for (int i0 = 0; i0 < 36; i0 += CH) {
#pragma unroll
    for (int d = 0; d < CH; ++d) {
      acc.x += __uint_as_float(v[d].x);
      acc.y += __uint_as_float(v[d].y);
      const int k = i0 + d + CH;
      v[d] = __builtin_amdgcn_raw_buffer_load_b128(r, k < 36 ? lbase + (4 * k + w) * step : 0x7F000000, 0, 0);
    }
  }
  if (acc.x == 1.2345f) out[threadIdx.x] = acc.y;
}

int main() {
  const long long bytes = 256ll << 20;
  float* buf;
  float* out;
  (void)hipMalloc(&buf, bytes);
  (void)hipMalloc(&out, 4096);
  (void)hipMemset(buf, 0, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int strides[] = {1024, 1024 + 64, 1024 + 128, 1024 + 256, 9216, 9216 + 64, 9216 + 128, 4608, 2048};
  for (int contiguous = 0; contiguous < 2; ++contiguous)
    for (int S : strides) {
      if (contiguous && S != 9216) continue;
      // contiguous: the same 144 KiB per row group as 1-KiB blocks (lane l: 16 B at 16 l)
      for (int rep = 0; rep < 2; ++rep) {
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(frag_loads<12>, dim3(208), dim3(256), 0, 0, buf, bytes, S, contiguous, out);
        (void)hipEventRecord(a, 0);
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(frag_loads<12>, dim3(208), dim3(256), 0, 0, buf, bytes, S, contiguous, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep) printf("%s S=%5d: %.2f us per launch\n", contiguous ? "contiguous 1-KiB blocks" : "16 rows x 64 B", S, ms * 1e3f / 200);
      }
    }
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(frag_loads<12>, dim3(208), dim3(256), 0, 0, buf, bytes, 9216, 0, out);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  return 0;
}
