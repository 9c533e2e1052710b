// Stand-alone check and timing of the symmetric-wave F(4x4) kernel
// (tools/w4_archive/conv_winograd4s.hip, in the library in round 5) against the F(4x4) one on the same
// layer (same U), and both against a float64 direct convolution of the first images.
// usage: w4s_bench B H Cin Cout epi iters [nimg_check] [lanes] [copies] [blk] [sk]   (epi 1 = pre-BN + BN + PReLU, 2 = BN + residual,
//        3 = BN + PReLU without pre-BN; W6_ZERO_SHIFT=1: pre-BN shift 0; lanes 2: timing as two
//        streams of B/2 each, launches interleaved, as the network's two lanes run; copies N: the
//        timed launches cycle through N copies of x, U and res, so that with N >= 8 the working set
//        exceeds the 256 MB MALL as the network's layer sequence does); blk: W4_BLK_* layout bits
//        for the timed launches of both kernels (the data is not rearranged: timing only); sk: the
//        shipping kernel's sk_mode (default 1; the network runs 0)
// build: SRC=w4s tools/w6_build.sh (hipcc, gfx950)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "conv_winograd4s.hip"  // the symmetric-wave kernel (tools/w4_archive/)

using namespace frhip;

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

static std::vector<float> host_rand(size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = d(g);
  return h;
}
static float* to_dev(const std::vector<float>& h) {
  float* p = nullptr;
  CK(hipMalloc((void**)&p, h.size() * sizeof(float)));
  CK(hipMemcpy(p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

// float64 direct 3x3 / pad 1 conv of images [0, nimg) with the same pre-BN / epilogue, NHWC
__global__ void direct_ref(const float* x, const float* w, const float* psc, const float* psh, const float* qsc,
                           const float* qsh, const float* al, const float* res, double* y, int nimg, int H, int W,
                           int Cin, int Cout, int epi) {
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (idx >= (long long)nimg * H * W * Cout) return;
  const int o = idx % Cout;
  const long long px = idx / Cout;
  const int xx = px % W, yy = (px / W) % H, b = px / ((long long)W * H);
  double acc = 0.0;
  for (int ky = 0; ky < 3; ++ky)
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = yy + ky - 1, ix = xx + kx - 1;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
      const float* xp = x + (((long long)b * H + iy) * W + ix) * Cin;
      const float* wp = w + ((long long)(o * 3 + ky) * 3 + kx) * Cin;
      for (int c = 0; c < Cin; ++c) {
        const double v = epi == 1 ? (double)xp[c] * psc[c] + psh[c] : (double)xp[c];  // pre-BN
        acc += v * wp[c];
      }
    }
  double v = acc * qsc[o] + qsh[o];
  if (epi == 1 || epi == 3) v = v > 0 ? v : v * al[o];
  if (epi == 2) v += res[idx];
  y[idx] = v;
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s B H Cin Cout epi iters [nimg_check]\n", argv[0]);
    return 2;
  }
  const int B = atoi(argv[1]), H = atoi(argv[2]), Cin = atoi(argv[3]), Cout = atoi(argv[4]);
  const int epi = atoi(argv[5]), iters = atoi(argv[6]);
  const int nchk = std::min(B, argc > 7 ? atoi(argv[7]) : 2);
  const bool pre = epi == 1;
  const int kepi = epi == 3 ? 1 : epi;  // the Epi the kernels run
  const size_t nx = (size_t)B * H * H * Cin, ny = (size_t)B * H * H * Cout;
  if (Cin % 16 || Cout % 64) {
    fprintf(stderr, "shape not supported by wino4s\n");
    return 2;
  }
  const auto hx = host_rand(nx, -1.f, 1.f, 1), hw = host_rand((size_t)Cout * 9 * Cin, -0.05f, 0.05f, 2);
  const auto hres = host_rand(ny, -1.f, 1.f, 3), hpsc = host_rand(Cin, 0.5f, 1.5f, 4),
             hpsh0 = host_rand(Cin, -0.1f, 0.1f, 5);
  std::vector<float> hpsh = hpsh0;
  if (getenv("W6_ZERO_SHIFT") && atoi(getenv("W6_ZERO_SHIFT"))) std::fill(hpsh.begin(), hpsh.end(), 0.f);
  const auto hqsc = host_rand(Cout, 0.5f, 1.5f, 6), hqsh = host_rand(Cout, -0.1f, 0.1f, 7),
             hal = host_rand(Cout, 0.1f, 0.3f, 8);
  std::vector<float> ht(Cin);
  for (int c = 0; c < Cin; ++c) ht[c] = hpsh[c] / hpsc[c];
  float *x = to_dev(hx), *w = to_dev(hw), *res = to_dev(hres), *psc = to_dev(hpsc), *psh = to_dev(hpsh);
  float *qsc = to_dev(hqsc), *qsh = to_dev(hqsh), *al = to_dev(hal), *pt = to_dev(ht);
  float *u4 = nullptr, *y4 = nullptr, *y6 = nullptr;
  CK(hipMalloc((void**)&u4, wino4_weight_floats(Cout, Cin) * sizeof(float)));
  CK(hipMalloc((void**)&y4, ny * sizeof(float)));
  CK(hipMalloc((void**)&y6, ny * sizeof(float)));
  CK(hipMemset(y4, 0, ny * sizeof(float)));
  CK(hipMemset(y6, 0, ny * sizeof(float)));
  CK(launch_wino4_weights(w, pre ? psc : nullptr, u4, Cout, Cin, nullptr));

  Wino4Params p4{};
  p4.x = x;
  p4.u = u4;
  p4.y = y4;
  p4.pre_t = pre ? pt : nullptr;
  p4.post_scale = qsc;
  p4.post_shift = qsh;
  p4.prelu = al;
  p4.res = epi == 2 ? res : nullptr;
  const long long part_floats = 257ll * 2 * 16 * 16 * 64;
  CK(hipMalloc((void**)&p4.part, part_floats * sizeof(float)));
  p4.part_floats = part_floats;
  const int cnt_cap = 1 << 16;
  CK(hipMalloc((void**)&p4.cnt, cnt_cap * sizeof(int)));
  CK(hipMemset(p4.cnt, 0, cnt_cap * sizeof(int)));
  p4.cnt_cap = cnt_cap;
  p4.sk_mode = 1;
  p4.B = B;
  p4.H = H;
  p4.W = H;
  p4.Cin = Cin;
  p4.Cout = Cout;

  Wino4Params p6 = p4;  // the same layer for the symmetric-wave kernel (it reads the fields it needs)
  p6.y = y6;

  // correctness first (one launch each), against float64 direct conv of the first nchk images
  CK(launch_wino4(p4, pre, (Epi)kepi, nullptr));
  CK(launch_wino4s(p6, pre, (Epi)kepi, nullptr));
  CK(hipDeviceSynchronize());
  const size_t nref = (size_t)nchk * H * H * Cout;
  double* yr = nullptr;
  CK(hipMalloc((void**)&yr, nref * sizeof(double)));
  hipLaunchKernelGGL(direct_ref, dim3((nref + 255) / 256), dim3(256), 0, nullptr, x, w, psc, psh, qsc, qsh, al, res, yr,
                     nchk, H, H, Cin, Cout, epi);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<double> hr(nref);
  std::vector<float> h4(ny), h6(ny);
  CK(hipMemcpy(hr.data(), yr, nref * sizeof(double), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h4.data(), y4, ny * sizeof(float), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h6.data(), y6, ny * sizeof(float), hipMemcpyDeviceToHost));
  double e4 = 0, e6 = 0, mx = 0, d46 = 0, m4 = 0;
  for (size_t i = 0; i < nref; ++i) {
    e4 = std::max(e4, std::fabs(h4[i] - hr[i]));
    e6 = std::max(e6, std::fabs(h6[i] - hr[i]));
    mx = std::max(mx, std::fabs(hr[i]));
  }
  size_t bad = 0;
  for (size_t i = 0; i < ny; ++i) {
    const double d = std::fabs((double)h6[i] - h4[i]);
    d46 = std::max(d46, d);
    m4 = std::max(m4, (double)std::fabs(h4[i]));
    bad += !(d <= 1e-3 * std::max(1.0, (double)std::fabs(h4[i])));
  }

  if (bad) {  // where the outliers sit: by output channel mod 64, by pixel of the image, by image
    std::vector<size_t> bc(64, 0), bp((size_t)H * H, 0), bi(std::min(B, 16), 0);
    for (size_t i = 0; i < ny; ++i) {
      const double d = std::fabs((double)h6[i] - h4[i]);
      if (d <= 1e-3 * std::max(1.0, (double)std::fabs(h4[i]))) continue;
      const size_t px = i / Cout, img = px / ((size_t)H * H);
      ++bc[(i % Cout) % 64];
      ++bp[px % ((size_t)H * H)];
      if (img < bi.size()) ++bi[img];
    }
    printf("  bad by cout%%64:");
    for (auto v : bc) printf(" %zu", v);
    printf("\n  bad by pixel (rows):\n");
    for (int y = 0; y < H; ++y) {
      printf("   ");
      for (int x = 0; x < H; ++x) printf(" %5zu", bp[(size_t)y * H + x]);
      printf("\n");
    }
    printf("  bad by image:");
    for (auto v : bi) printf(" %zu", v);
    printf("\n");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    for (int i = 0; i < 3; ++i) CK(launch());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < iters; ++i) CK(launch());
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float t = 0;
    CK(hipEventElapsedTime(&t, e0, e1));
    return 1e3 * t / iters;
  };
  const int nl = argc > 8 ? atoi(argv[8]) : 1;
  p4.blk = p6.blk = argc > 10 ? atoi(argv[10]) : 0;
  p4.sk_mode = argc > 11 ? atoi(argv[11]) : 1;
  hipStream_t st[2] = {nullptr, nullptr};
  Wino4Params p4l[2] = {p4, p4};
  Wino4Params p6l[2] = {p6, p6};
  if (nl == 2) {
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    const int hb = B / 2;
    for (int l = 0; l < 2; ++l) {
      const size_t xo = (size_t)l * hb * H * H * Cin, yo = (size_t)l * hb * H * H * Cout;
      p4l[l].B = p6l[l].B = l ? B - hb : hb;
      p4l[l].x = p6l[l].x = x + xo;
      p4l[l].y = y4 + yo;
      p6l[l].y = y6 + yo;
      p4l[l].res = p6l[l].res = epi == 2 ? res + yo : nullptr;
      if (l) {  // the second lane's own partial slots and tickets
        CK(hipMalloc((void**)&p4l[l].part, part_floats * sizeof(float)));
        CK(hipMalloc((void**)&p4l[l].cnt, cnt_cap * sizeof(int)));
        CK(hipMemset(p4l[l].cnt, 0, cnt_cap * sizeof(int)));
      }
    }
  }
  // one "launch" = both lanes' launches (nl == 2, forked from and joined to the null stream)
  hipEvent_t f0, j0, j1;
  CK(hipEventCreate(&f0));
  CK(hipEventCreate(&j0));
  CK(hipEventCreate(&j1));
  auto lanes = [&](auto one) -> hipError_t {
    if (nl != 2) return one(0, (hipStream_t) nullptr);
    CK(hipEventRecord(f0, nullptr));
    CK(hipStreamWaitEvent(st[0], f0, 0));
    CK(hipStreamWaitEvent(st[1], f0, 0));
    for (int l = 0; l < 2; ++l) CK(one(l, st[l]));
    CK(hipEventRecord(j0, st[0]));
    CK(hipEventRecord(j1, st[1]));
    CK(hipStreamWaitEvent(nullptr, j0, 0));
    CK(hipStreamWaitEvent(nullptr, j1, 0));
    return hipSuccess;
  };
  const int ncopy = argc > 9 ? std::max(1, atoi(argv[9])) : 1;
  std::vector<float*> xs{x}, us{u4}, rs{res};
  for (int c = 1; c < ncopy; ++c) {
    float *xc = nullptr, *uc = nullptr, *rc = nullptr;
    const size_t nu = wino4_weight_floats(Cout, Cin);
    CK(hipMalloc((void**)&xc, nx * sizeof(float)));
    CK(hipMalloc((void**)&uc, nu * sizeof(float)));
    CK(hipMalloc((void**)&rc, ny * sizeof(float)));
    CK(hipMemcpy(xc, x, nx * sizeof(float), hipMemcpyDeviceToDevice));
    CK(hipMemcpy(uc, u4, nu * sizeof(float), hipMemcpyDeviceToDevice));
    CK(hipMemcpy(rc, res, ny * sizeof(float), hipMemcpyDeviceToDevice));
    xs.push_back(xc);
    us.push_back(uc);
    rs.push_back(rc);
  }
  int it4 = 0, it6 = 0;
  auto pick = [&](auto q, int l, int c) {  // lane l's params on copy c
    const size_t xo = (size_t)(l ? B / 2 : 0) * H * H * Cin, yo = (size_t)(l ? B / 2 : 0) * H * H * Cout;
    q.x = xs[c] + xo;
    q.u = us[c];
    if (epi == 2) q.res = rs[c] + yo;
    return q;
  };
  auto run4 = [&] {
    const int c = it4++ % ncopy;
    return lanes([&](int l, hipStream_t s) { return launch_wino4(pick(p4l[l], l, c), pre, (Epi)kepi, s); });
  };
  auto run6 = [&] {
    const int c = it6++ % ncopy;
    return lanes([&](int l, hipStream_t s) { return launch_wino4s(pick(p6l[l], l, c), pre, (Epi)kepi, s); });
  };
  const double t4 = timeit(run4);
  const double t6 = timeit(run6);
  const double t4b = timeit(run4);
  const double t6b = timeit(run6);
  Wino4Params c4 = p4;
  wino4_canvas(c4);
  const double alg = 2.0 * 9.0 * (double)B * H * H * Cin * Cout;  // direct-conv FLOPs
  printf("B=%d lanes=%d copies=%d blk=%d H=%d %d->%d epi=%d | vs f64 direct (%d img, max|y| %.3g): wino4 %.3g, wino4s %.3g | wino4s vs wino4 "
         "all: max|d| %.3g (max|y| %.3g), %zu beyond 1e-3 rel | wino4 %.1f/%.1f us, wino4s %.1f/%.1f us "
         "(%.3f of wino4; %d tiles, %.1f direct-TF/s)\n",
         B, nl, ncopy, p4.blk, H, Cin, Cout, epi, nchk, mx, e4, e6, d46, m4, bad, t4, t4b, t6, t6b, std::min(t6, t6b) / std::min(t4, t4b),
         c4.ntiles, alg / (1e-6 * std::min(t6, t6b)) / 1e12);
  return bad ? 1 : 0;
}
