// Per-layer microbenchmark of the Winograd conv kernel (tools/ only, not shipped).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I facerecognitionpipeline_amd/csrc \
//        -x hip tools/wino_bench.cpp -o tools/wino_bench
// Usage: wino_bench [B] [reps]  -> one line per shape: us/launch, direct-equivalent TF/s,
// executed (Winograd-domain) MFMA TF/s.
#include "../facerecognitionpipeline_amd/csrc/conv_winograd.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace frhip;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void fill(float* p, long long n, unsigned seed, float scale) {
  long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13;
  x *= 0x5bd1e995;
  x ^= x >> 15;
  p[i] = ((x & 0xffffff) / 16777216.f - 0.5f) * scale;
}

static float* dalloc(long long n, unsigned seed, float scale) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  fill<<<(n + 255) / 256, 256>>>(p, n, seed, scale);
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  struct Shape {
    int H, C;
  } shapes[] = {{112, 64}, {56, 64}, {28, 128}, {14, 256}, {7, 512}};
  for (auto sh : shapes) {
    const int H = sh.H, C = sh.C;
    const long long act = (long long)B * H * H * C;
    float* x = dalloc(act, 1, 2.f);
    float* res = dalloc(act, 2, 2.f);
    float* y;
    CK(hipMalloc(&y, act * 4));
    float* w = dalloc((long long)C * 9 * C, 3, 0.1f);
    float* u;
    CK(hipMalloc(&u, wino_weight_floats(C, C) * 4));
    CK(launch_wino_weights(w, u, C, C, 0));
    float* sc = dalloc(C, 4, 0.5f);
    float* shf = dalloc(C, 5, 0.5f);
    float* al = dalloc(C, 6, 0.5f);
    for (int epi = 0; epi < 2; ++epi) {
      WinoParams p{};
      p.x = x;
      p.u = u;
      p.y = y;
      p.pre_scale = epi == 0 ? sc : nullptr;
      p.pre_shift = epi == 0 ? shf : nullptr;
      p.post_scale = sc;
      p.post_shift = shf;
      p.prelu = al;
      p.res = res;
      p.B = B;
      p.H = H;
      p.W = H;
      p.Cin = C;
      p.Cout = C;
      const bool pre = epi == 0;
      const Epi e = epi == 0 ? EPI_AFFINE_PRELU : EPI_AFFINE_RES;
      for (int i = 0; i < 3; ++i) CK(launch_wino(p, pre, e, 0));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, 0));
      for (int i = 0; i < reps; ++i) CK(launch_wino(p, pre, e, 0));
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = 1e3 * ms / reps;
      const double alg = 2.0 * B * H * H * (double)C * C * 9;
      const int T = (H + 1) / 2;
      const double exe = 2.0 * B * T * T * 16.0 * C * C;
      printf("H=%3d C=%3d %s  %8.1f us  alg %6.1f TF/s  exec %6.1f TF/s (%4.1f%% of 157.3)\n", H, C,
             epi == 0 ? "pre+prelu" : "residual ", us, alg / us * 1e-6, exe / us * 1e-6, exe / us * 1e-6 / 1.573);
    }
    CK(hipFree(x));
    CK(hipFree(res));
    CK(hipFree(y));
    CK(hipFree(w));
    CK(hipFree(u));
    CK(hipFree(sc));
    CK(hipFree(shf));
    CK(hipFree(al));
  }
  return 0;
}
