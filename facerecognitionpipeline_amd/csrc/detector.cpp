// SCRFD-10G face detector behind the C ABI (arch "scrfd_10g", model_type "scrfd").
//
// Replaces FaceDetector.detect (face_recognition.py:31-48) -> insightface FaceAnalysis
// ('buffalo_l').get -> SCRFD det_10g (onnxruntime) at det_size 640x640.  The network
// restatement, its state-dict keys and the post-processing are those of oracle/scrfd.py
// (parity unpinned: no insightface / ONNX files offline).
//
// Layout: every activation is NHWC f32 with channels padded to a multiple of 32 (the
// conv kernel's K-step is 32 channels of one tap); padded channels carry zero weights,
// zero BN scale/shift and therefore stay exactly 0 through ReLU and residual adds.
//   letterbox (u8)  -> det_stem (3->28, s2) -> conv 28->28 -> conv 28->56 -> maxpool
//   -> BasicBlock stages (3,4,2,3) x (56,88,88,224), strides 1,2,2,2 (avg-pool
//      downsample = one 2x2 stride-2 conv with w/4)
//   -> PAFPN (lateral 1x1, top-down nearest add, 3x3, bottom-up 3x3 s2 add, 3x3) to 56
//   -> per level: 3 x (conv3x3 80 + BN + ReLU) -> one conv3x3 80->30 (cls 2 | bbox 8 | kps 20)
//   -> decode (sigmoid, anchors, / det_scale) -> sort + NMS
#include <cmath>
#include <cstring>

#include "runtime.h"

using namespace frhip;

namespace frhip_rt {

namespace {

constexpr int STAGE_BLOCKS[4] = {3, 4, 2, 3};
constexpr int STAGE_PLANES[4] = {56, 88, 88, 224};
constexpr int STEM = 56, NECK = 56, HEADC = 80;
constexpr int STRIDES[3] = {8, 16, 32};

int pad32(int c) { return (c + 31) / 32 * 32; }
int pad16(int c) { return (c + 15) / 16 * 16; }

struct DetBlock {
  ConvW conv1, conv2, down;
  bool has_down = false;
};

std::string blk(int s, int u) { return "backbone.layer" + std::to_string(s + 1) + "." + std::to_string(u) + "."; }

}  // namespace

struct Detector {
  int max_frames = 0, det_w = 640, det_h = 640;
  float* arena = nullptr;
  float *stem_w = nullptr, *stem_scale = nullptr, *stem_shift = nullptr;
  float* zeros = nullptr;  // zero PReLU slopes (= ReLU), 256 channels
  ConvW stem1, stem2;
  std::vector<DetBlock> blocks[4];
  ConvW lateral[3], fpn[3], down[2], pafpn[2], tower[3][3], head[3];
  // workspace
  void* ws = nullptr;
  size_t ws_bytes = 0;
  uint8_t* canvas = nullptr;
  float *big0 = nullptr, *big1 = nullptr, *mid[3] = {nullptr, nullptr, nullptr}, *dbuf = nullptr;
  float *c_out[3] = {nullptr, nullptr, nullptr}, *lat[3] = {nullptr, nullptr, nullptr};
  float *inter[3] = {nullptr, nullptr, nullptr}, *outs[3] = {nullptr, nullptr, nullptr};
  float *tA = nullptr, *tB = nullptr, *hd[3] = {nullptr, nullptr, nullptr};
  float* pool = nullptr;  // AvgPool2d(2, 2) of a stage's input (the downsample shortcut's 1x1 conv input)
  float* cand = nullptr;
  int* count = nullptr;
  float* dets = nullptr;
  int* dets_count = nullptr;
  int* tabs = nullptr;  // [det_w + det_h][4]
  int dets_cap = 0;
  bool row_reduce = true;  // row_plan (frt_set_detector_row_reduction switches it off for A/B)
  std::vector<int> htabs;
  ~Detector() {
    (void)hipFree(arena);
    (void)hipFree(ws);
  }
};

void detector_destroy(Detector* d) { delete d; }

void detector_set_row_reduction(Detector* d, bool on) {
  if (d) d->row_reduce = on;
}

void detector_convs(Detector* d, std::vector<ConvW*>& out) {
  if (!d) return;
  out.push_back(&d->stem1);
  out.push_back(&d->stem2);
  for (auto& st : d->blocks)
    for (auto& b : st) {
      out.push_back(&b.conv1);
      out.push_back(&b.conv2);
      out.push_back(&b.down);
    }
  for (int i = 0; i < 3; ++i) {
    out.push_back(&d->lateral[i]);
    out.push_back(&d->fpn[i]);
    out.push_back(&d->head[i]);
    for (auto& t : d->tower[i]) out.push_back(&t);
  }
  for (int i = 0; i < 2; ++i) {
    out.push_back(&d->down[i]);
    out.push_back(&d->pafpn[i]);
  }
}

std::map<std::string, size_t> detector_schema() {
  std::map<std::string, size_t> m;
  auto conv = [&](const std::string& k, int o, int i, int kh) { m[k] = (size_t)o * i * kh * kh; };
  conv("backbone.stem.0.conv.weight", STEM / 2, 3, 3);
  add_bn(m, "backbone.stem.0.bn", STEM / 2);
  conv("backbone.stem.1.conv.weight", STEM / 2, STEM / 2, 3);
  add_bn(m, "backbone.stem.1.bn", STEM / 2);
  conv("backbone.stem.2.conv.weight", STEM, STEM / 2, 3);
  add_bn(m, "backbone.stem.2.bn", STEM);
  int cin = STEM;
  for (int s = 0; s < 4; ++s) {
    for (int u = 0; u < STAGE_BLOCKS[s]; ++u) {
      const int ci = u == 0 ? cin : STAGE_PLANES[s], co = STAGE_PLANES[s];
      const std::string p = blk(s, u);
      conv(p + "conv1.weight", co, ci, 3);
      add_bn(m, p + "bn1", co);
      conv(p + "conv2.weight", co, co, 3);
      add_bn(m, p + "bn2", co);
      if (u == 0 && (s > 0 || ci != co)) {
        conv(p + "downsample.1.weight", co, ci, 1);
        add_bn(m, p + "downsample.2", co);
      }
    }
    cin = STAGE_PLANES[s];
  }
  for (int i = 0; i < 3; ++i) {
    const std::string l = std::to_string(i);
    conv("neck.lateral_convs." + l + ".conv.weight", NECK, STAGE_PLANES[i + 1], 1);
    m["neck.lateral_convs." + l + ".conv.bias"] = NECK;
    conv("neck.fpn_convs." + l + ".conv.weight", NECK, NECK, 3);
    m["neck.fpn_convs." + l + ".conv.bias"] = NECK;
    if (i < 2) {
      conv("neck.downsample_convs." + l + ".conv.weight", NECK, NECK, 3);
      m["neck.downsample_convs." + l + ".conv.bias"] = NECK;
      conv("neck.pafpn_convs." + l + ".conv.weight", NECK, NECK, 3);
      m["neck.pafpn_convs." + l + ".conv.bias"] = NECK;
    }
    for (int j = 0; j < 3; ++j) {
      const std::string t = "bbox_head.towers." + l + "." + std::to_string(j);
      conv(t + ".conv.weight", HEADC, j == 0 ? NECK : HEADC, 3);
      add_bn(m, t + ".bn", HEADC);
    }
    conv("bbox_head.cls." + l + ".weight", 2, HEADC, 3);
    m["bbox_head.cls." + l + ".bias"] = 2;
    conv("bbox_head.reg." + l + ".weight", 8, HEADC, 3);
    m["bbox_head.reg." + l + ".bias"] = 8;
    conv("bbox_head.kps." + l + ".weight", 20, HEADC, 3);
    m["bbox_head.kps." + l + ".bias"] = 20;
  }
  return m;
}

namespace {

// [O][I][k][k] -> [Op][k][k][Ip] zero-padded (times `mul`, exact for powers of two).
std::vector<float> pack_w(const std::vector<float>& w, int O, int I, int k, int Op, int Ip, int taps_rep = 1,
                          float mul = 1.f) {
  const int kk = k * taps_rep;  // taps_rep = 2 turns a 1x1 conv into a 2x2 (avg-pool fold)
  std::vector<float> r((size_t)Op * kk * kk * Ip, 0.f);
  for (int o = 0; o < O; ++o)
    for (int i = 0; i < I; ++i)
      for (int y = 0; y < kk; ++y)
        for (int x = 0; x < kk; ++x)
          r[(((size_t)o * kk + y) * kk + x) * Ip + i] = w[(((size_t)o * I + i) * k + y / taps_rep) * k + x / taps_rep] * mul;
  return r;
}

std::vector<float> padv(const std::vector<float>& v, int n) {
  std::vector<float> r(n, 0.f);
  std::copy(v.begin(), v.end(), r.begin());
  return r;
}

// Channels are padded to 32 (the direct kernel's K-step); the head towers, whose convs all run on
// F(4x4) (16-channel K-steps), to 16: 80 channels, not 96 (head_pad16)
void set_geom(ConvW& c, int cin, int cout, int k, int stride, int pad, bool p16 = false) {
  c.cin = p16 ? pad16(cin) : pad32(cin);
  c.cout = p16 ? pad16(cout) : pad32(cout);
  c.kh = c.kw = k;
  c.stride = stride;
  c.pad = pad;
}

}  // namespace

int detector_finalize(fr_handle* h) {
  auto P = [&](const std::string& k) -> const std::vector<float>& { return *getp(h, k); };
  auto* d = h->det ? h->det : new Detector();
  h->det = d;
  Packer pk;
  std::vector<float> sc, sh;
  // conv + BN(+ReLU): weights packed, BN folded into post scale/shift, ReLU = zero slopes
  auto conv_bn = [&](ConvW& c, const std::string& wk, const std::string& bnk, int cin, int cout, int k, int stride,
                     int pad, bool relu, int taps_rep = 1, float mul = 1.f, bool p16 = false) {
    set_geom(c, cin, cout, k * taps_rep, stride, pad, p16);
    pk.put(&c.w, pack_w(P(wk), cout, cin, k, c.cout, c.cin, taps_rep, mul));
    bn_fold(&P(bnk + ".weight"), &P(bnk + ".bias"), P(bnk + ".running_mean"), P(bnk + ".running_var"), sc, sh);
    pk.put(&c.post_scale, padv(sc, c.cout));
    pk.put(&c.post_shift, padv(sh, c.cout));
    c.prelu = relu ? reinterpret_cast<float*>(1) : nullptr;  // patched to d->zeros after upload
  };
  // conv + bias
  auto conv_bias = [&](ConvW& c, const std::string& wk, const std::string& bk, int cin, int cout, int k, int stride,
                       int pad) {
    set_geom(c, cin, cout, k, stride, pad);
    pk.put(&c.w, pack_w(P(wk), cout, cin, k, c.cout, c.cin));
    pk.put(&c.post_scale, padv(std::vector<float>(cout, 1.f), c.cout));
    pk.put(&c.post_shift, padv(P(bk), c.cout));
  };
  // stem conv 0 (3 -> 28, direct kernel): [28][3][3][3] -> [ky][kx][ci][Cp]
  {
    const auto& w = P("backbone.stem.0.conv.weight");
    const int C = pad32(STEM / 2);
    std::vector<float> r(27 * C, 0.f);
    for (int o = 0; o < STEM / 2; ++o)
      for (int c = 0; c < 3; ++c)
        for (int y = 0; y < 3; ++y)
          for (int x = 0; x < 3; ++x) r[((y * 3 + x) * 3 + c) * C + o] = w[((o * 3 + c) * 3 + y) * 3 + x];
    pk.put(&d->stem_w, r);
    bn_fold(&P("backbone.stem.0.bn.weight"), &P("backbone.stem.0.bn.bias"), P("backbone.stem.0.bn.running_mean"),
            P("backbone.stem.0.bn.running_var"), sc, sh);
    pk.put(&d->stem_scale, padv(sc, C));
    pk.put(&d->stem_shift, padv(sh, C));
  }
  pk.put(&d->zeros, std::vector<float>(256, 0.f));
  conv_bn(d->stem1, "backbone.stem.1.conv.weight", "backbone.stem.1.bn", STEM / 2, STEM / 2, 3, 1, 1, true);
  conv_bn(d->stem2, "backbone.stem.2.conv.weight", "backbone.stem.2.bn", STEM / 2, STEM, 3, 1, 1, true);
  int cin = STEM;
  for (int s = 0; s < 4; ++s) {
    d->blocks[s].assign(STAGE_BLOCKS[s], DetBlock{});
    for (int u = 0; u < STAGE_BLOCKS[s]; ++u) {
      const int ci = u == 0 ? cin : STAGE_PLANES[s], co = STAGE_PLANES[s];
      const int stride = (u == 0 && s > 0) ? 2 : 1;
      DetBlock& b = d->blocks[s][u];
      const std::string p = blk(s, u);
      conv_bn(b.conv1, p + "conv1.weight", p + "bn1", ci, co, 3, stride, 1, true);
      conv_bn(b.conv2, p + "conv2.weight", p + "bn2", co, co, 3, 1, 1, true);
      if (u == 0 && (s > 0 || ci != co)) {
        b.has_down = true;
        // AvgPool2d(2, 2) (launch_avgpool2) then this conv1x1 + BN; stage 1 (stride 1): conv1x1 alone
        conv_bn(b.down, p + "downsample.1.weight", p + "downsample.2", ci, co, 1, 1, 0, false);
      }
    }
    cin = STAGE_PLANES[s];
  }
  for (int i = 0; i < 3; ++i) {
    const std::string l = std::to_string(i);
    conv_bias(d->lateral[i], "neck.lateral_convs." + l + ".conv.weight", "neck.lateral_convs." + l + ".conv.bias",
              STAGE_PLANES[i + 1], NECK, 1, 1, 0);
    conv_bias(d->fpn[i], "neck.fpn_convs." + l + ".conv.weight", "neck.fpn_convs." + l + ".conv.bias", NECK, NECK, 3,
              1, 1);
    if (i < 2) {
      conv_bias(d->down[i], "neck.downsample_convs." + l + ".conv.weight", "neck.downsample_convs." + l + ".conv.bias",
                NECK, NECK, 3, 2, 1);
      conv_bias(d->pafpn[i], "neck.pafpn_convs." + l + ".conv.weight", "neck.pafpn_convs." + l + ".conv.bias", NECK,
                NECK, 3, 1, 1);
    }
    for (int j = 0; j < 3; ++j) {
      const std::string t = "bbox_head.towers." + l + "." + std::to_string(j);
      conv_bn(d->tower[i][j], t + ".conv.weight", t + ".bn", j == 0 ? NECK : HEADC, HEADC, 3, 1, 1, true, 1, 1.f,
              true);
    }
    // cls | reg | kps as one conv 80 -> 30 (channel order = the ONNX outputs' per-anchor layout)
    {
      ConvW& c = d->head[i];
      set_geom(c, HEADC, 30, 3, 1, 1, true);
      std::vector<float> w((size_t)30 * HEADC * 9), b(30);
      const auto& wc = P("bbox_head.cls." + l + ".weight");
      const auto& wr = P("bbox_head.reg." + l + ".weight");
      const auto& wk = P("bbox_head.kps." + l + ".weight");
      std::copy(wc.begin(), wc.end(), w.begin());
      std::copy(wr.begin(), wr.end(), w.begin() + (size_t)2 * HEADC * 9);
      std::copy(wk.begin(), wk.end(), w.begin() + (size_t)10 * HEADC * 9);
      const auto& bc = P("bbox_head.cls." + l + ".bias");
      const auto& br = P("bbox_head.reg." + l + ".bias");
      const auto& bk = P("bbox_head.kps." + l + ".bias");
      std::copy(bc.begin(), bc.end(), b.begin());
      std::copy(br.begin(), br.end(), b.begin() + 2);
      std::copy(bk.begin(), bk.end(), b.begin() + 10);
      pk.put(&c.w, pack_w(w, 30, HEADC, 3, c.cout, c.cin));
      pk.put(&c.post_scale, padv(std::vector<float>(30, 1.f), c.cout));
      pk.put(&c.post_shift, padv(b, c.cout));
    }
  }
  if (d->arena) FR_HIP(h, hipFree(d->arena));
  d->arena = nullptr;
  FR_HIP(h, hipMalloc((void**)&d->arena, pk.buf.size() * sizeof(float)));
  FR_HIP(h, hipMemcpy(d->arena, pk.buf.data(), pk.buf.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& f : pk.fix) *f.first = d->arena + f.second;
  // ReLU convs share the zero-slope vector
  auto relu = [&](ConvW& c) {
    if (c.prelu) c.prelu = d->zeros;
  };
  relu(d->stem1);
  relu(d->stem2);
  for (auto& st : d->blocks)
    for (auto& b : st) {
      relu(b.conv1);
      relu(b.conv2);
    }
  for (auto& lv : d->tower)
    for (auto& c : lv) relu(c);

  // workspace for max_frames letterboxed 640x640 images
  const size_t B = (size_t)h->max_batch;
  d->max_frames = h->max_batch;
  const size_t W0 = d->det_w / 2, H0 = d->det_h / 2;  // stem resolution
  const size_t p1 = pad32(STAGE_PLANES[1]), p2 = pad32(STAGE_PLANES[2]), p3 = pad32(STAGE_PLANES[3]);
  const size_t nk = pad32(NECK), hc = pad32(HEADC);
  size_t off = 0;
  std::vector<std::pair<void**, size_t>> plan;
  auto take = [&](void** dst, size_t bytes) {
    plan.push_back({dst, off});
    off += (bytes + 255) & ~size_t(255);
  };
  const size_t f4 = sizeof(float);
  const size_t hw[3] = {(size_t)(d->det_h / 8) * (d->det_w / 8), (size_t)(d->det_h / 16) * (d->det_w / 16),
                        (size_t)(d->det_h / 32) * (d->det_w / 32)};
  take((void**)&d->canvas, B * d->det_h * d->det_w * 3);
  take((void**)&d->big0, B * H0 * W0 * pad32(STEM) * f4);
  take((void**)&d->big1, B * H0 * W0 * pad32(STEM / 2) * f4);  // stem1 output (28 -> 32 channels)
  for (auto& m : d->mid) take((void**)&m, B * (H0 / 2) * (W0 / 2) * pad32(STEM) * f4);
  take((void**)&d->dbuf, B * hw[0] * p1 * f4);
  take((void**)&d->c_out[0], B * hw[0] * p1 * f4);
  take((void**)&d->c_out[1], B * hw[1] * p2 * f4);
  take((void**)&d->c_out[2], B * hw[2] * p3 * f4);
  for (int i = 0; i < 3; ++i) {
    take((void**)&d->lat[i], B * hw[i] * nk * f4);
    take((void**)&d->inter[i], B * hw[i] * nk * f4);
    take((void**)&d->outs[i], B * hw[i] * nk * f4);
    take((void**)&d->hd[i], B * hw[i] * 32 * f4);
  }
  take((void**)&d->pool, B * hw[0] * pad32(STEM) * f4);  // the largest: stage 2's input pooled to 80x80
  take((void**)&d->tA, B * hw[0] * hc * f4);
  take((void**)&d->tB, B * hw[0] * hc * f4);
  d->dets_cap = 1024;
  take((void**)&d->cand, B * DET_MAX_CANDIDATES * 16 * f4);
  take((void**)&d->count, B * sizeof(int));
  take((void**)&d->dets, B * d->dets_cap * 15 * f4);
  take((void**)&d->dets_count, B * sizeof(int));
  take((void**)&d->tabs, (size_t)(d->det_w + d->det_h) * 4 * sizeof(int));
  if (d->ws) FR_HIP(h, hipFree(d->ws));
  d->ws = nullptr;
  FR_HIP(h, hipMalloc(&d->ws, off));
  d->ws_bytes = off;
  for (auto& p : plan) *p.first = (char*)d->ws + p.second;
  if (ensure_stream_k(h->device, &h->cus, &h->sk_ws, &h->sk_ws_floats, &h->sk_cnt, &h->sk_cnt_cap) != FR_OK)
    return fail(h, FR_ERR_HIP, "stream-K workspace allocation failed");
  return FR_OK;
}

// cv::resize INTER_LINEAR coefficient table for one axis: (src0, src1, w0, w1) per output
// (also the resize branch of FaceEmbedder.preprocess, frhip_runtime.cpp).
#pragma clang fp contract(off)
void resize_axis_table(int dsize, int ssize, int* t) {
  const double scale = 1.0 / ((double)dsize / ssize);
  for (int d = 0; d < dsize; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f -= (float)s;
    if (s < 0) {
      f = 0.f;
      s = 0;
    }
    if (s >= ssize - 1) {
      f = 0.f;
      s = ssize - 1;
    }
    t[4 * d] = s;
    t[4 * d + 1] = std::min(s + 1, ssize - 1);
    t[4 * d + 2] = (int)std::lrint((1.f - f) * 2048.f);
    t[4 * d + 3] = (int)std::lrint(f * 2048.f);
  }
}
#pragma clang fp contract(on)

int resize_simd_end(int row) {
  // SSE2 vertical pass: 16-element chunks while x <= row-16, then 8-element chunks while x < row-8
  int x = 0;
  while (x <= row - 16) x += 16;
  while (x < row - 8) x += 8;
  return x;
}

namespace {

int dconv(fr_handle* h, const ConvW& c, const float* x, float* y, int B, int H, int W, Epi epi, const float* res,
          hipStream_t s) {
  return run_conv(h, c, x, y, B, H, W, epi, res, 0, 0, 1, 0, s);
}

}  // namespace

namespace {

struct Geometry {
  int new_w = 0, new_h = 0, simd_end = 0;
  double det_scale = 1.0;
  int skip1 = 0, skip2 = 0;  // canvas rows the stem + stage 1 / stage 2 do not compute (row_plan)
  int at1 = 0, at2 = 0;      // stage-1 / stage-2 output rows whose copies stand in for skipped rows
};

// Rows of a landscape letterbox the stem and stages 1-2 need not compute.  The canvas below the
// resized frame (rows new_h..det_h-1) is all zeros, so every layer maps it to rows that are all
// equal: a "run" [a, b) of identical rows between the rows the frame reaches (< a) and the rows
// the conv zero padding below the canvas reaches (>= b).  A 3x3 pad-1 conv of stride s maps a
// run [a, b) to [ceil((a + 1) / s), floor((b - 2) / s) + 1) (a 2x2 stride-2 pad-0 conv to
// [ceil(a / 2), floor((b - 2) / 2) + 1)): each output row whose window lies in the run is a run
// row, rows above and below it are computed from the same values at the same distance from the
// frame / from the canvas bottom.  So the network on a canvas with D fewer run rows (D a
// multiple of 32: every stride divides it, the bottom rows keep their parity) computes the same
// values above and below the run, as long as the run keeps >= 3 rows at every layer.  For a
// 1080p frame (new_h = 360) the stem and stage 1 run with D1 = 192 of 640 rows skipped, stage 2
// with D2 = 64; stage 1's output is expanded from D1 to D2 skipped rows and stage 2's to the full
// height by copying one run row into the missing rows (launch_row_expand).  The values are the
// full canvas's up to fp32 rounding: Winograd tiles round each row by its position in the tile,
// so run rows equal each other mathematically, not bitwise (tests/test_gpu_detector_rows.py).
void row_plan(int new_h, int DH, Geometry& g) {
  g.skip1 = g.skip2 = g.at1 = g.at2 = 0;
  if (new_h >= DH || new_h < 1) return;
  int a = new_h, b = DH, s = 1, dmax = DH;
  auto room = [&]() {
    const int r = (b - a - 3) * s;  // canvas rows the run can lose at this layer
    dmax = std::min(dmax, r < 0 ? -1 : r / 32 * 32);
  };
  auto conv3 = [&](int stride) {
    a = (a + 1 + stride - 1) / stride;
    b = (b - 2) / stride + 1;
    s *= stride;
    room();
  };
  conv3(2);  // stem 0 (3x3 s2)
  conv3(1);  // stem 1
  conv3(1);  // stem 2
  conv3(2);  // MaxPool2d(3, 2, 1)
  for (int u = 0; u < STAGE_BLOCKS[0]; ++u) {  // stage 1 (stride 1, identity shortcuts)
    conv3(1);
    conv3(1);
  }
  if (dmax <= 0) return;
  g.skip1 = dmax;
  g.at1 = a;
  for (int u = 0; u < STAGE_BLOCKS[1]; ++u) {  // stage 2
    if (u == 0) {  // conv1 3x3 s2 and the 2x2 s2 downsample both read the block input
      const int da = (a + 1) / 2, db = (b - 2) / 2 + 1;
      conv3(2);
      conv3(1);
      a = std::max(a, da);  // conv2 + downsample: rows equal in both are run rows
      b = std::min(b, db);
      room();
    } else {
      conv3(1);
      conv3(1);
    }
  }
  if (dmax <= 0) return;
  g.skip2 = dmax;
  g.at2 = a;
}

// Letterbox geometry (scrfd.py detect; Python floats are doubles) and the resize tables.
int setup_geometry(fr_handle* h, int height, int width, Geometry& g, hipStream_t s) {
  Detector* d = h->det;
  const int DW = d->det_w, DH = d->det_h;
  const double imr = (double)height / width, mr = (double)DH / DW;
  if (imr > mr) {
    g.new_h = DH;
    g.new_w = (int)(g.new_h / imr);
  } else {
    g.new_w = DW;
    g.new_h = (int)(g.new_w * imr);
  }
  if (g.new_w < 1 || g.new_h < 1) return fail(h, FR_ERR_INVALID_ARGUMENT, "frame too small to letterbox");
  g.det_scale = (double)g.new_h / height;
  d->htabs.assign((size_t)(g.new_w + g.new_h) * 4, 0);
  resize_axis_table(g.new_w, width, d->htabs.data());
  resize_axis_table(g.new_h, height, d->htabs.data() + 4 * g.new_w);
  g.simd_end = resize_simd_end(g.new_w * 3);
  if (d->row_reduce) row_plan(g.new_h, DH, g);
  FR_HIP(h, hipMemcpyAsync(d->tabs, d->htabs.data(), d->htabs.size() * sizeof(int), hipMemcpyHostToDevice, s));
  return FR_OK;
}

// Letterbox + network for B <= max_frames frames; head maps land in d->hd[0..2].
int forward_chunk(fr_handle* h, const uint8_t* fr, int B, int height, int width, const Geometry& g, hipStream_t s) {
  Detector* d = h->det;
  const int DW = d->det_w, DH = d->det_h;
  const int* xtab = d->tabs;
  const int* ytab = d->tabs + 4 * g.new_w;
  const int c0 = pad32(STEM / 2);
  // the stem and stage 1 run on a canvas of DH - skip1 rows, stage 2 on DH - skip2 (row_plan)
  const int Hc = DH - g.skip1;
  const int H0 = Hc / 2, W0 = DW / 2, H1 = H0 / 2, W1 = W0 / 2;
  const int new_w = g.new_w, new_h = g.new_h, simd_end = g.simd_end;
  hipError_t e = launch_letterbox(fr, B, height, width, xtab, ytab, new_w, new_h, simd_end, DW, Hc, d->canvas, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("letterbox: ") + hipGetErrorString(e));
  e = launch_det_stem(d->canvas, B, Hc, DW, c0, d->stem_w, d->stem_scale, d->stem_shift, d->big0, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("det stem: ") + hipGetErrorString(e));
  int rc = dconv(h, d->stem1, d->big0, d->big1, B, H0, W0, EPI_AFFINE_PRELU, nullptr, s);
  if (rc) return rc;
  rc = dconv(h, d->stem2, d->big1, d->big0, B, H0, W0, EPI_AFFINE_PRELU, nullptr, s);
  if (rc) return rc;
  e = launch_maxpool3(d->big0, B, H0, W0, pad32(STEM), d->mid[0], s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("maxpool: ") + hipGetErrorString(e));
  // backbone stages
  float* x = d->mid[0];
  auto pick = [&](const float* a, const float* b) -> float* {
    for (float* m : d->mid)
      if (m != a && m != b) return m;
    return nullptr;
  };
  int Hh = H1, Ww = W1;
  for (int st = 0; st < 4; ++st) {
    if (st == 1 && g.skip1) {  // stage 1's output to stage 2's height
      float* full = pick(x, nullptr);
      e = launch_row_expand(x, B, Hh, Ww, pad32(STAGE_PLANES[0]), g.at1, (DH - g.skip2) / 4, full, s);
      if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("row expand: ") + hipGetErrorString(e));
      x = full;
      Hh = (DH - g.skip2) / 4;
    }
    if (st == 2 && g.skip2) {  // stage 2's output (the FPN's level-0 input) to full height
      e = launch_row_expand(x, B, Hh, Ww, pad32(STAGE_PLANES[1]), g.at2, DH / 8, d->c_out[0], s);
      if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("row expand: ") + hipGetErrorString(e));
      x = d->c_out[0];
      Hh = DH / 8;
    }
    for (size_t u = 0; u < d->blocks[st].size(); ++u) {
      const DetBlock& b = d->blocks[st][u];
      const int Ho = (Hh + 2 - 3) / b.conv1.stride + 1, Wo = (Ww + 2 - 3) / b.conv1.stride + 1;
      float* t = pick(x, nullptr);
      // the stages' outputs go to c_out[] (the FPN's inputs); stage 2's through the expansion
      const bool last = st > 0 && u + 1 == d->blocks[st].size() && !(st == 1 && g.skip2);
      float* y = last ? d->c_out[st - 1] : pick(x, t);
      rc = dconv(h, b.conv1, x, t, B, Hh, Ww, EPI_AFFINE_PRELU, nullptr, s);
      if (rc) return rc;
      const float* res = x;
      if (b.has_down) {
        const float* xd = x;
        if (b.conv1.stride == 2) {
          e = launch_avgpool2(x, B, Hh, Ww, b.down.cin, d->pool, s);
          if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("avgpool: ") + hipGetErrorString(e));
          xd = d->pool;
        }
        rc = dconv(h, b.down, xd, d->dbuf, B, Ho, Wo, EPI_AFFINE, nullptr, s);
        if (rc) return rc;
        res = d->dbuf;
      }
      rc = dconv(h, b.conv2, t, y, B, Ho, Wo, EPI_AFFINE_RES_PRELU, res, s);
      if (rc) return rc;
      x = y;
      Hh = Ho;
      Ww = Wo;
    }
  }
  // PAFPN
  const int lh[3] = {DH / 8, DH / 16, DH / 32}, lw[3] = {DW / 8, DW / 16, DW / 32};
  for (int i = 0; i < 3; ++i) {
    rc = dconv(h, d->lateral[i], d->c_out[i], d->lat[i], B, lh[i], lw[i], EPI_AFFINE, nullptr, s);
    if (rc) return rc;
  }
  for (int i = 2; i > 0; --i) {
    e = launch_upsample_add(d->lat[i - 1], d->lat[i], B, lh[i], lw[i], pad32(NECK), s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("upsample: ") + hipGetErrorString(e));
  }
  for (int i = 0; i < 3; ++i) {
    rc = dconv(h, d->fpn[i], d->lat[i], d->inter[i], B, lh[i], lw[i], EPI_AFFINE, nullptr, s);
    if (rc) return rc;
  }
  for (int i = 0; i < 2; ++i) {  // inter[i+1] += down_i(inter[i]) (in place: residual read, then write)
    rc = dconv(h, d->down[i], d->inter[i], d->inter[i + 1], B, lh[i], lw[i], EPI_AFFINE_RES, d->inter[i + 1], s);
    if (rc) return rc;
  }
  for (int i = 1; i < 3; ++i) {
    rc = dconv(h, d->pafpn[i - 1], d->inter[i], d->outs[i], B, lh[i], lw[i], EPI_AFFINE, nullptr, s);
    if (rc) return rc;
  }
  // heads
  for (int i = 0; i < 3; ++i) {
    const float* f = i == 0 ? d->inter[0] : d->outs[i];
    rc = dconv(h, d->tower[i][0], f, d->tA, B, lh[i], lw[i], EPI_AFFINE_PRELU, nullptr, s);
    if (rc) return rc;
    rc = dconv(h, d->tower[i][1], d->tA, d->tB, B, lh[i], lw[i], EPI_AFFINE_PRELU, nullptr, s);
    if (rc) return rc;
    rc = dconv(h, d->tower[i][2], d->tB, d->tA, B, lh[i], lw[i], EPI_AFFINE_PRELU, nullptr, s);
    if (rc) return rc;
    rc = dconv(h, d->head[i], d->tA, d->hd[i], B, lh[i], lw[i], EPI_AFFINE, nullptr, s);
    if (rc) return rc;
  }
  return FR_OK;
}

}  // namespace

int detector_run(fr_handle* h, const uint8_t* frames, int n, int height, int width, float det_thresh, int max_faces,
                 float* dets, int32_t* counts, hipStream_t s) {
  Detector* d = h->det;
  const int DW = d->det_w, DH = d->det_h;
  Geometry g;
  int rc = setup_geometry(h, height, width, g, s);
  if (rc) return rc;
  const double det_scale = g.det_scale;
  const int lh[3] = {DH / 8, DH / 16, DH / 32}, lw[3] = {DW / 8, DW / 16, DW / 32};
  const int fmax = std::min(max_faces, d->dets_cap);
  std::vector<float> hbuf;
  std::vector<int> hcnt, hraw;
  for (int off = 0; off < n; off += d->max_frames) {
    const int B = std::min(d->max_frames, n - off);
    rc = forward_chunk(h, frames + (size_t)off * height * width * 3, B, height, width, g, s);
    if (rc) return rc;
    hipError_t e;
    // decode + NMS
    FR_HIP(h, hipMemsetAsync(d->count, 0, B * sizeof(int), s));
    DetDecodeParams dp{};
    int base = 0;
    for (int i = 0; i < 3; ++i) {
      dp.head[i] = d->hd[i];
      dp.hw[i] = lh[i] * lw[i];
      dp.w[i] = lw[i];
      dp.stride[i] = STRIDES[i];
      dp.anchor_base[i] = base;
      base += dp.hw[i] * 2;
    }
    dp.thresh = det_thresh;
    dp.det_scale = (float)det_scale;
    dp.cap = DET_MAX_CANDIDATES;
    dp.count = d->count;
    dp.cand = d->cand;
    e = launch_decode(dp, B, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("decode: ") + hipGetErrorString(e));
    e = launch_nms(d->cand, d->count, B, DET_MAX_CANDIDATES, 0.4f, d->dets_cap, d->dets, d->dets_count, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("nms: ") + hipGetErrorString(e));
    hbuf.resize((size_t)B * d->dets_cap * 15);
    hcnt.resize(B);
    hraw.resize(B);
    FR_HIP(h, hipMemcpyAsync(hbuf.data(), d->dets, hbuf.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    FR_HIP(h, hipMemcpyAsync(hcnt.data(), d->dets_count, B * sizeof(int), hipMemcpyDeviceToHost, s));
    FR_HIP(h, hipMemcpyAsync(hraw.data(), d->count, B * sizeof(int), hipMemcpyDeviceToHost, s));
    FR_HIP(h, hipStreamSynchronize(s));
    for (int b = 0; b < B; ++b) {
      if (hraw[b] > DET_MAX_CANDIDATES)
        return fail(h, FR_ERR_UNSUPPORTED,
                    "frame " + std::to_string(off + b) + " has " + std::to_string(hraw[b]) +
                        " anchors above det_thresh (limit " + std::to_string(DET_MAX_CANDIDATES) + ")");
      counts[off + b] = hcnt[b];
      const int k = std::min(hcnt[b], fmax);
      std::memcpy(dets + ((size_t)(off + b) * max_faces) * 15, hbuf.data() + (size_t)b * d->dets_cap * 15,
                  (size_t)k * 15 * sizeof(float));
    }
  }
  return FR_OK;
}

int detector_forward(fr_handle* h, const uint8_t* frames, int n, int height, int width, float* heads,
                     uint8_t* canvas, hipStream_t s) {
  Detector* d = h->det;
  if (n > d->max_frames) return fail(h, FR_ERR_INVALID_ARGUMENT, "n exceeds the handle's max_batch");
  Geometry g;
  int rc = setup_geometry(h, height, width, g, s);
  if (rc) return rc;
  rc = forward_chunk(h, frames, n, height, width, g, s);
  if (rc) return rc;
  size_t off = 0;
  for (int i = 0; i < 3; ++i) {
    const size_t bytes = (size_t)n * (d->det_h >> (3 + i)) * (d->det_w >> (3 + i)) * 32 * sizeof(float);
    FR_HIP(h, hipMemcpyAsync((char*)heads + off, d->hd[i], bytes, hipMemcpyDeviceToDevice, s));
    off += bytes;
  }
  if (canvas) {  // the full det_h-row canvases (the rows row_plan skipped are zeros)
    const size_t row = (size_t)d->det_w * 3, Hc = (size_t)(d->det_h - g.skip1);
    FR_HIP(h, hipMemcpy2DAsync(canvas, d->det_h * row, d->canvas, Hc * row, Hc * row, n, hipMemcpyDeviceToDevice, s));
    if (g.skip1)
      FR_HIP(h, hipMemset2DAsync(canvas + Hc * row, d->det_h * row, 0, (size_t)g.skip1 * row, n, s));
  }
  FR_HIP(h, hipStreamSynchronize(s));
  return FR_OK;
}

}  // namespace frhip_rt
