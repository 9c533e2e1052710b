// Stand-alone timing of one F(4x4) Winograd conv layer (launches back to back), linked
// against a (possibly modified) copy of csrc/conv_winograd4.hip by tools/w4g_variants.py.
// usage: w4g_bench B H Cin Cout epi iters   (epi 1 = pre-BN + BN + PReLU, 2 = BN + residual)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <cmath>
#include <algorithm>
#include <vector>

#include "frhip_kernels.h"

using namespace frhip;

extern "C" void w4g_after_run() __attribute__((weak));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static float* dev_rand(size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = d(g);
  float* p = nullptr;
  CK(hipMalloc((void**)&p, n * sizeof(float)));
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s B H Cin Cout epi iters\n", argv[0]);
    return 2;
  }
  const int B = atoi(argv[1]), H = atoi(argv[2]), Cin = atoi(argv[3]), Cout = atoi(argv[4]);
  const int epi = atoi(argv[5]), iters = atoi(argv[6]);
  const size_t nx = (size_t)B * H * H * Cin, ny = (size_t)B * H * H * Cout;
  float* x = dev_rand(nx, -1.f, 1.f, 1);
  float* w = dev_rand((size_t)Cout * 9 * Cin, -0.05f, 0.05f, 2);
  float* res = dev_rand(ny, -1.f, 1.f, 3);
  float* psc = dev_rand(Cin, 0.5f, 1.5f, 4);
  float* psh = dev_rand(Cin, -0.1f, 0.1f, 5);
  float* qsc = dev_rand(Cout, 0.5f, 1.5f, 6);
  float* qsh = dev_rand(Cout, -0.1f, 0.1f, 7);
  float* al = dev_rand(Cout, 0.1f, 0.3f, 8);
  float *u = nullptr, *y = nullptr;
  CK(hipMalloc((void**)&u, wino4_weight_floats(Cout, Cin) * sizeof(float)));
  CK(hipMalloc((void**)&y, ny * sizeof(float)));
  const bool pre = epi == 1;
  CK(launch_wino4_weights(w, pre ? psc : nullptr, u, Cout, Cin, nullptr));
  Wino4Params p{};
  p.x = x;
  p.u = u;
  p.y = y;
  p.pre_t = pre ? psh : nullptr;  // any per-channel t: the timing does not depend on its values
  p.post_scale = qsc;
  p.post_shift = qsh;
  p.prelu = al;
  p.res = epi == 2 ? res : nullptr;
  // split-K partial slots (small grids)
  float* part = nullptr;
  const long long part_floats = 257ll * 2 * 16 * 16 * 64;
  CK(hipMalloc((void**)&part, part_floats * sizeof(float)));
  p.part = part;
  p.part_floats = part_floats;
  // argv[7]: round 4-5's stream-K tail mode; the library dropped it in round 6 (tools/w4_archive/),
  // the argument is read and ignored so older command lines still parse.  argv[7] = 2 instead sets
  // p.shapes = 2 (the wide / tall item shapes at every grid size, for layers that have one)
  p.shapes = argc > 7 && atoi(argv[7]) == 2 ? 2 : 1;
  p.no_split = argc > 8 ? atoi(argv[8]) : 0;  // 1: whole items only (no split-K)
  // argv[9] lanes: 1 one stream; 2 two streams of B/2 each, launches interleaved (fr_set_lanes)
  const int nl = argc > 9 ? atoi(argv[9]) : 1;
  // argv[10] layouts (W4_BLK_* bits: 1 x, 2 res, 4 y channel-blocked); timing only, the data is not
  // rearranged, and the check below compares with a launch of the same layouts
  p.blk = argc > 10 ? atoi(argv[10]) : 0;
  p.B = B;
  p.H = H;
  p.W = H;
  p.Cin = Cin;
  p.Cout = Cout;
  hipStream_t st[2] = {nullptr, nullptr};
  Wino4Params pl[2] = {p, p};
  if (nl == 2) {
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    const int hb = B / 2;
    for (int l = 0; l < 2; ++l) {
      pl[l].B = l ? B - hb : hb;
      pl[l].x = x + (size_t)l * hb * H * H * Cin;
      pl[l].y = y + (size_t)l * hb * H * H * Cout;
      pl[l].res = p.res ? res + (size_t)l * hb * H * H * Cout : nullptr;
      if (l) CK(hipMalloc((void**)&pl[l].part, part_floats * sizeof(float)));  // each lane its own partial slots
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int n) {
    for (int i = 0; i < n; ++i)
      for (int l = 0; l < nl; ++l) CK(launch_wino4(pl[l], pre, (Epi)epi, st[l]));
  };
  run(3);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, nullptr));
  if (nl == 2) {  // fork both streams from the null stream's event, join back
    CK(hipStreamWaitEvent(st[0], e0, 0));
    CK(hipStreamWaitEvent(st[1], e0, 0));
  }
  run(iters);
  if (nl == 2) {
    hipEvent_t j0, j1;
    CK(hipEventCreate(&j0));
    CK(hipEventCreate(&j1));
    CK(hipEventRecord(j0, st[0]));
    CK(hipEventRecord(j1, st[1]));
    CK(hipStreamWaitEvent(nullptr, j0, 0));
    CK(hipStreamWaitEvent(nullptr, j1, 0));
  }
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float t = 0;
  CK(hipEventElapsedTime(&t, e0, e1));
  Wino4Params c = p;
  wino4_canvas(c);
  const double exec = 2.0 * 36.0 * c.ntiles * (double)Cin * Cout;
  // check: the same layer on 64-cout whole items only (no split-K, no item shapes, one stream) into a
  // second buffer
  float* y2 = nullptr;
  CK(hipMalloc((void**)&y2, ny * sizeof(float)));
  Wino4Params q = p;
  q.y = y2;
  q.no_split = 1;
  q.shapes = 0;
  CK(launch_wino4(q, pre, (Epi)epi, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<float> h1(ny), h2(ny);
  CK(hipMemcpy(h1.data(), y, ny * sizeof(float), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), y2, ny * sizeof(float), hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  size_t ndiff = 0;
  for (size_t i = 0; i < ny; ++i) {
    const double d = std::fabs((double)h1[i] - h2[i]);
    md = std::max(md, d);
    mx = std::max(mx, (double)std::fabs(h2[i]));
    ndiff += h1[i] != h2[i];
  }
  printf("B=%d H=%d %d->%d epi=%d lanes=%d shapes=%d blk=%d: %.1f us (%.1f TF executed) | vs whole items: max|d| %.3g (max|y| %.3g), %zu differ\n",
         B, H, Cin, Cout, epi, nl, p.shapes, p.blk, 1e3 * t / iters, exec / (1e-3 * t / iters) / 1e12, md, mx, ndiff);
  if (w4g_after_run) w4g_after_run();  // instrumented variants (w4g_variants.py "stamps") report here
  return 0;
}
