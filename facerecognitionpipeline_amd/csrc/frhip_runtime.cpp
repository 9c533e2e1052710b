// libfrhip runtime: handle, state-dict ingestion + BatchNorm folding, the IR
// forward executor and the gallery matcher behind the C ABI of include/frhip.h.
//
// Host-side C++ (compiled by hipcc for the HIP runtime API only).  What it
// replaces in the reference:
//   FaceEmbedder.__init__/load_state_dict   face_embedder.py:27-62
//   FaceEmbedder.extract_embeddings_batch   face_embedder.py:137-182 (A3)
//   GalleryManager.get_gallery_embeddings   gallery_manager.py:177-187 (A10)
//   GalleryManager.search                   gallery_manager.py:189-205 (A11)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/frhip.h"
#include "../../include/frhip_testing.h"
#include "frhip_kernels.h"
#include "runtime.h"

using namespace frhip;
using namespace frhip_rt;

namespace frhip_rt {

thread_local std::string g_create_error;

std::vector<BlockSpec> block_specs(const std::string& arch, bool* ok) {
  int units[4];
  *ok = true;
  if (arch == "ir_50") {
    int u[4] = {3, 4, 14, 3};
    memcpy(units, u, sizeof(u));
  } else if (arch == "ir_101") {
    int u[4] = {3, 13, 30, 3};
    memcpy(units, u, sizeof(u));
  } else if (arch == "ir_34") {
    int u[4] = {3, 4, 6, 3};
    memcpy(units, u, sizeof(u));
  } else if (arch == "ir_18") {
    int u[4] = {2, 2, 2, 2};
    memcpy(units, u, sizeof(u));
  } else {
    *ok = false;
    return {};
  }
  const int widths[4] = {64, 128, 256, 512};
  std::vector<BlockSpec> v;
  int in = 64;
  for (int s = 0; s < 4; ++s) {
    v.push_back({in, widths[s], 2});
    for (int u = 1; u < units[s]; ++u) v.push_back({widths[s], widths[s], 1});
    in = widths[s];
  }
  return v;
}

}  // namespace frhip_rt

namespace frhip_rt {

int fail(fr_handle* h, int code, const std::string& msg) {
  if (h)
    h->err = msg;
  else
    g_create_error = msg;
  return code;
}

int ensure_dev_err(fr_handle* h) {
  if (h->dev_err) return FR_OK;
  FR_HIP(h, hipHostMalloc((void**)&h->dev_err, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
  *(volatile int*)h->dev_err = 0;
  return FR_OK;
}

int check_dev_err(fr_handle* h) {
  if (!h->dev_err) return FR_OK;
  const int v = *(volatile int*)h->dev_err;
  if (!v) return FR_OK;
  *(volatile int*)h->dev_err = 0;
  return fail(h, FR_ERR_HIP,
              (v & FR_DEVERR_W4_HANDOFF)
                  ? "F(4x4) ring hand-off timed out in wino4_kernel: the results of the work queued on this handle "
                    "before this call are invalid"
                  : "device error word set (" + std::to_string(v) + ")");
}



void add_bn(std::map<std::string, size_t>& m, const std::string& p, int c, bool affine) {
  if (affine) {
    m[p + ".weight"] = c;
    m[p + ".bias"] = c;
  }
  m[p + ".running_mean"] = c;
  m[p + ".running_var"] = c;
  m[p + ".num_batches_tracked"] = 1;
}

std::map<std::string, size_t> schema(const std::vector<BlockSpec>& specs) {
  std::map<std::string, size_t> m;
  m["input_layer.0.weight"] = 64 * 3 * 9;
  add_bn(m, "input_layer.1", 64);
  m["input_layer.2.weight"] = 64;
  add_bn(m, "output_layer.0", 512);
  m["output_layer.3.weight"] = (size_t)512 * 512 * 49;
  m["output_layer.3.bias"] = 512;
  add_bn(m, "output_layer.4", 512, false);
  for (size_t i = 0; i < specs.size(); ++i) {
    const auto& s = specs[i];
    const std::string p = "body." + std::to_string(i) + ".";
    if (s.cin != s.depth) {
      m[p + "shortcut_layer.0.weight"] = (size_t)s.depth * s.cin;
      add_bn(m, p + "shortcut_layer.1", s.depth);
    }
    add_bn(m, p + "res_layer.0", s.cin);
    m[p + "res_layer.1.weight"] = (size_t)s.depth * s.cin * 9;
    add_bn(m, p + "res_layer.2", s.depth);
    m[p + "res_layer.3.weight"] = s.depth;
    m[p + "res_layer.4.weight"] = (size_t)s.depth * s.depth * 9;
    add_bn(m, p + "res_layer.5", s.depth);
  }
  return m;
}

// insightface arcface_torch IResNet keys (the network behind the reference's ArcFace ONNX
// files, face_embedder.py:64-88): every stage's first unit has a conv1x1+BN downsample,
// BN1d `features` is affine, and the model output is not L2-normalised.
std::map<std::string, size_t> schema_arcface(const std::vector<BlockSpec>& specs) {
  std::map<std::string, size_t> m;
  m["conv1.weight"] = 64 * 3 * 9;
  add_bn(m, "bn1", 64);
  m["prelu.weight"] = 64;
  add_bn(m, "bn2", 512);
  m["fc.weight"] = (size_t)512 * 512 * 49;
  m["fc.bias"] = 512;
  add_bn(m, "features", 512);
  int stage = 0, unit = 0;
  for (size_t i = 0; i < specs.size(); ++i) {
    const auto& s = specs[i];
    if (s.stride == 2 && i > 0) {
      ++stage;
      unit = 0;
    }
    const std::string p = "layer" + std::to_string(stage + 1) + "." + std::to_string(unit) + ".";
    add_bn(m, p + "bn1", s.cin);
    m[p + "conv1.weight"] = (size_t)s.depth * s.cin * 9;
    add_bn(m, p + "bn2", s.depth);
    m[p + "prelu.weight"] = s.depth;
    m[p + "conv2.weight"] = (size_t)s.depth * s.depth * 9;
    add_bn(m, p + "bn3", s.depth);
    if (s.stride == 2) {
      m[p + "downsample.0.weight"] = (size_t)s.depth * s.cin;
      add_bn(m, p + "downsample.1", s.depth);
    }
    ++unit;
  }
  return m;
}

// State-dict key names of one residual unit / the stem / the head, per model family.
struct UnitKeys {
  std::string pre_bn, conv1, mid_bn, prelu, conv2, out_bn, sc_conv, sc_bn;
};

UnitKeys unit_keys(bool arcface, const std::vector<BlockSpec>& specs, size_t i) {
  if (!arcface) {
    const std::string p = "body." + std::to_string(i) + ".";
    return {p + "res_layer.0", p + "res_layer.1.weight", p + "res_layer.2", p + "res_layer.3.weight",
            p + "res_layer.4.weight", p + "res_layer.5", p + "shortcut_layer.0.weight", p + "shortcut_layer.1"};
  }
  int stage = 0, unit = 0;
  for (size_t j = 1; j <= i; ++j) {
    if (specs[j].stride == 2) {
      ++stage;
      unit = 0;
    } else {
      ++unit;
    }
  }
  const std::string p = "layer" + std::to_string(stage + 1) + "." + std::to_string(unit) + ".";
  return {p + "bn1", p + "conv1.weight", p + "bn2", p + "prelu.weight", p + "conv2.weight", p + "bn3",
          p + "downsample.0.weight", p + "downsample.1"};
}


// PyTorch CPU eval BatchNorm computes alpha = gamma/sqrt(var+eps), beta = bias - mean*alpha
// in the input dtype and applies x*alpha + beta (ATen batch_norm_cpu_collect_linear_and_constant_terms).
void bn_fold(const std::vector<float>* gamma, const std::vector<float>* beta, const std::vector<float>& mean,
             const std::vector<float>& var, std::vector<float>& scale, std::vector<float>& shift) {
  const size_t c = mean.size();
  scale.resize(c);
  shift.resize(c);
  for (size_t i = 0; i < c; ++i) {
    const float invstd = 1.0f / std::sqrt(var[i] + 1e-5f);
    const float g = gamma ? (*gamma)[i] : 1.0f;
    const float b = beta ? (*beta)[i] : 0.0f;
    scale[i] = invstd * g;
    shift[i] = b - mean[i] * scale[i];
  }
}

// [O][I][kh][kw] -> [O][kh][kw][I]
std::vector<float> repack_oihw(const std::vector<float>& w, int O, int I, int kh, int kw) {
  std::vector<float> r((size_t)O * I * kh * kw);
  for (int o = 0; o < O; ++o)
    for (int i = 0; i < I; ++i)
      for (int y = 0; y < kh; ++y)
        for (int x = 0; x < kw; ++x)
          r[(((size_t)o * kh + y) * kw + x) * I + i] = w[(((size_t)o * I + i) * kh + y) * kw + x];
  return r;
}

int ensure_buf(fr_handle* h, void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return FR_OK;
  if (*p) FR_HIP(h, hipFree(*p));
  *p = nullptr;
  *cap = 0;
  FR_HIP(h, hipMalloc(p, bytes));
  *cap = bytes;
  return FR_OK;
}

// Stream-K slabs for P = CUs x (<=2 blocks/CU) blocks x 2 slots x the largest tile (256x128).
int ensure_stream_k(int device, int* cus, float** ws, long long* ws_floats, int** cnt, int* cnt_cap) {
  if (*ws) return FR_OK;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
  const long long floats = (long long)n * 4 * 2 * 256 * 128;
  const int cap = 8 * n;
  if (hipMalloc((void**)ws, floats * sizeof(float)) != hipSuccess) return FR_ERR_HIP;
  if (hipMalloc((void**)cnt, cap * sizeof(int)) != hipSuccess) return FR_ERR_HIP;
  if (hipMemset(*cnt, 0, cap * sizeof(int)) != hipSuccess) return FR_ERR_HIP;
  *cus = n;
  *ws_floats = floats;
  *cnt_cap = cap;
  return FR_OK;
}

hipEvent_t take_event(fr_handle* h) {
  if (!h->pool.empty()) {
    hipEvent_t e = h->pool.back();
    h->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct ProfScope {
  fr_handle* h;
  hipStream_t s;
  ProfEvent ev{};
  bool on;
  ProfScope(fr_handle* h_, hipStream_t s_, double flop, int kind, double exec_flop = -1.0)
      : h(h_), s(s_), on(h_->prof) {
    if (!on) return;
    ev.a = take_event(h);
    ev.b = take_event(h);
    ev.flop = flop;
    ev.exec_flop = exec_flop < 0 ? flop : exec_flop;
    ev.kind = kind;
    if (!ev.a || !ev.b) {
      on = false;
      return;
    }
    (void)hipEventRecord(ev.a, s);
  }
  ~ProfScope() {
    if (!on) return;
    (void)hipEventRecord(ev.b, s);
    h->events.push_back(ev);
  }
};

// A/B (frt_set_conv2sc_tile): the tile of the fused stride-2 conv2 + conv-shortcut launches, -1 = the rule
static int g_conv2sc_tile = -1;
// A/B (frt_set_wino4_nbg): tile blocks per XCD item group of the F(4x4) launches, 0 = the rule
static int g_wino4_nbg = 0;
// cap on the F(4x4) split-K parts of small grids (frt_set_wino4_max_split: serving sweeps); 0 = none
static int g_wino4_max_split = 0;
// the stage-1 stride-2 conv2 on its band kernel (frt_set_s2_band: tests compare it with the
// implicit-GEMM kernel)
static int g_s2band = 1;
// poll bound of wino4_kernel's ring hand-off waits (frt_set_wino4_poll_limit: tests force expiry)
static int g_wino4_poll = WINO4_POLL_DEFAULT;
// F(4x4) item shapes for layers of 65..96 and of <= 32 couts (frt_set_wino4_shapes: A/B and tests)
static int g_wino4_shapes = 1;


// serving conv kernel: layers of at most this many output pixels (n * Ho * Wo).  Batch 1 also
// takes stage 1's 56x56 layers: 1.0626 vs 1.0740 ms per embed + match, medians of 8 runs each
// interleaved in one process, spreads 0.0003 / 0.0007 ms (profiles/r05/serving_pixel_limit_ab.txt,
// tools/serve_small_ab.py --pixels); at batch 2 their 6,272 pixels, and stage 2's 1,568, are
// faster on F(4x4) split-K (1.50 vs 1.52-1.54 ms with 4,096; profiles/r04/serving/pixel_threshold_ab.txt)
static inline long long convs_max_m(const fr_handle* h, int n) { return n == 1 ? h->convs_max_m1 : 1024; }

// The geometry fields of conv cw over a B x H x W input: what the kernel-selection rules read.
static ConvParams conv_shape(const ConvW& cw, int B, int H, int W) {
  ConvParams p{};
  p.B = B;
  p.H = H;
  p.W = W;
  p.Cin = cw.cin;
  p.Cout = cw.cout;
  p.KH = cw.kh;
  p.KW = cw.kw;
  p.stride = cw.stride;
  p.pad = cw.pad;
  p.Ho = (H + 2 * cw.pad - cw.kh) / cw.stride + 1;
  p.Wo = (W + 2 * cw.pad - cw.kw) / cw.stride + 1;
  p.M = B * p.Ho * p.Wo;
  p.Cin2 = std::max(cw.cin2, 0);
  return p;
}

// Whether run_conv puts this launch on the serving conv kernel (conv_small.hip).  One rule for
// run_conv's branch and for forward_lanes' plan of which activations are channel-blocked (the
// kernel is the only consumer / producer of that layout), so the two cannot disagree.
// has_x2: the fused shortcut's input will be passed (cw.cin2 > 0).
static bool convs_takes(const fr_handle* h, const ConvW& cw, ConvParams p, Epi epi, int nsplit, bool has_x2) {
  static const float sentinel = 0.f;
  if (has_x2 && !p.x2) p.x2 = &sentinel;  // convs_supported only checks that it is given
  return p.B <= h->convs_max_n && p.M <= convs_max_m(h, p.B) && !h->detector && h->prec == PREC_F32 && nsplit == 1 &&
         cw.w_frag && convs_supported(p, cw.pre_scale != nullptr, epi);
}

// Whether run_conv puts this conv on the F(4x4) kernel (the branch below; the plan of channel-
// blocked activations in forward_lanes reads the same rule).  Ho / Wo: the conv's output size.
static bool w4_takes(const fr_handle* h, const ConvW& cw, Epi epi, int res_H, int res_W, int Ho, int Wo) {
  const bool wino_epi = (epi == EPI_AFFINE_PRELU && cw.pre_scale) || (epi == EPI_AFFINE_RES && !cw.pre_scale && res_H == Ho);
  // F(4x4) also takes the detector's epilogues (no pre-BN; residual of the output's shape)
  const bool wino4_epi = wino_epi || (!cw.pre_scale && (epi == EPI_AFFINE_PRELU || epi == EPI_AFFINE ||
                                                        ((epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_PRELU) &&
                                                         (res_H == 0 || res_H == Ho) && (res_W == 0 || res_W == Wo))));
  return h->winograd && h->wino_m == 4 && h->prec == PREC_F32 && cw.wino4 && wino4_epi &&
         wino4_supported(cw.cin, cw.cout, cw.kh, cw.kw, cw.stride, cw.pad);
}

int run_conv(fr_handle* h, const ConvW& cw, const float* x, float* y, int B, int H, int W, Epi epi,
             const float* res, int res_H, int res_W, int nsplit, long long split_stride, hipStream_t s,
             const LaneWs* L, const float* x2) {
  float* const sk_ws = L ? L->sk_ws : h->sk_ws;
  int* const sk_cnt = L ? L->sk_cnt : h->sk_cnt;
  float* const w4part = L ? L->w4part : h->w4part;
  ConvParams p{};
  p.x = x;
  p.w = cw.w;
  p.y = y;
  p.pre_scale = cw.pre_scale;
  p.pre_shift = cw.pre_shift;
  p.post_scale = cw.post_scale;
  p.post_shift = cw.post_shift;
  p.prelu = cw.prelu;
  p.res = res;
  p.B = B;
  p.H = H;
  p.W = W;
  p.Cin = cw.cin;
  p.Cout = cw.cout;
  p.KH = cw.kh;
  p.KW = cw.kw;
  p.stride = cw.stride;
  p.pad = cw.pad;
  p.Ho = (H + 2 * cw.pad - cw.kh) / cw.stride + 1;
  p.Wo = (W + 2 * cw.pad - cw.kw) / cw.stride + 1;
  p.res_H = res_H;
  p.res_W = res_W;
  p.M = B * p.Ho * p.Wo;
  p.steps_total = cw.kh * cw.kw * cw.cin / 32;
  if (cw.cin2 > 0) {
    p.x2 = x2;
    p.Cin2 = cw.cin2;
    p.steps1 = p.steps_total;
    p.steps_total += cw.cin2 / 32;
  }
  p.steps_per_split = (p.steps_total + nsplit - 1) / nsplit;
  p.split_stride = split_stride;
  if (h->stream_k && nsplit == 1 && sk_ws) {
    p.sk_cus = h->cus;
    p.sk_ws = sk_ws;
    p.sk_ws_floats = L ? L->sk_ws_floats : h->sk_ws_floats;
    p.sk_cnt = sk_cnt;
    p.sk_cnt_cap = L ? L->sk_cnt_cap : h->sk_cnt_cap;
  }
  const double flop = 2.0 * p.M * (double)p.Cout * (cw.kh * cw.kw * cw.cin + cw.cin2);
  // serving batches (n <= convs_max_n): every body 3x3 conv as one launch with the whole K per
  // 16x16 tile (conv_small.hip); f32 parity path only
  // (layers of at most convs_max_m(B) output pixels: stage 1's 112x112 conv1, 784 pixel blocks
  // x 4 cout blocks, stays on F(4x4) split-K, which is faster there: 54 vs ~20 us)
  if (convs_takes(h, cw, p, epi, nsplit, x2 != nullptr)) {
    if (h->w4_blk)  // forward_lanes plans F(4x4) layouts only when no lane reaches this branch
      return fail(h, FR_ERR_HIP, "internal: F(4x4) channel-blocked activations in the serving conv kernel");
    p.w = cw.w_frag;
    p.blk = h->convs_blk;
    if (h->convs_y2 && epi != EPI_AFFINE_PRELU) {
      p.y2 = h->convs_y2;
      p.y2_scale = h->convs_y2_scale;
      p.y2_shift = h->convs_y2_shift;
    }
    ProfScope ps(h, s, flop, FR_PROF_CONV_DIRECT);
    const hipError_t e = launch_convs(p, cw.pre_scale != nullptr, epi, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("serving conv launch: ") + hipGetErrorString(e));
    if (p.y2) h->convs_y2_done = true;
    return FR_OK;
  }
  if (h->convs_blk)  // forward_lanes only sets it for layers the branch above takes
    return fail(h, FR_ERR_HIP, "internal: channel-blocked activations outside the serving conv kernel");
  // Tile per layer shape, from tools/conv_sweep.py on MI355X at B=256 with the stream-K
  // schedule (profiles/r01/sweep.txt): 8-wave 128x64 for the 64-channel
  // stage and the 128-channel residual convs, 8-wave 128x128 for the 1x1 shortcuts,
  // 8-wave 256x128 for every other 3x3 conv and the FC.
  // Winograd F(4x4,3x3) for the stride-1 3x3 convs (f32 parity path only)
  if (w4_takes(h, cw, epi, res_H, res_W, p.Ho, p.Wo)) {
    Wino4Params wp{};
    wp.x = x;
    wp.u = cw.wino4;
    wp.y = y;
    wp.pre_t = cw.wino4_t;
    wp.post_scale = cw.post_scale;
    wp.post_shift = cw.post_shift;
    wp.prelu = cw.prelu;
    wp.res = res;
    wp.B = B;
    wp.H = H;
    wp.W = W;
    wp.Cin = cw.cin;
    wp.Cout = cw.cout;
    wp.part = w4part;
    wp.part_floats = w4part ? fr_handle::W4PART_FLOATS : 0;
    wp.max_split = g_wino4_max_split;
    wp.err = h->dev_err;
    wp.poll_max = g_wino4_poll > 0 ? g_wino4_poll : -1;
    wp.blk = h->w4_blk;  // forward_lanes' plan of channel-blocked activations
    wp.nbg_override = g_wino4_nbg;
    wp.shapes = g_wino4_shapes;
    Wino4Params cv = wp;
    cv.blk = 0;
    wino4_canvas(cv);
    // executed: 36 products per (canvas) 4x4 tile and (cin, cout) pair (the same canvas either kernel)
    const double exec = 2.0 * 36.0 * cv.ntiles * (double)cw.cin * cw.cout;
    ProfScope ps(h, s, flop, FR_PROF_CONV_WINOGRAD, exec);
    const bool pre = cw.pre_scale != nullptr;
    hipError_t e = launch_wino4(wp, pre, epi, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("winograd4 launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  if (h->w4_blk)  // forward_lanes only sets it for layers the F(4x4) branch above takes
    return fail(h, FR_ERR_HIP, "internal: channel-blocked activations outside the F(4x4) kernel");
  // Winograd F(2x2,3x3) for the stride-1 3x3 convs (f32 parity path only)
  if (h->winograd && h->prec == PREC_F32 && cw.wino &&
      ((epi == EPI_AFFINE_PRELU && cw.pre_scale) || (epi == EPI_AFFINE_RES && !cw.pre_scale && res_H == p.Ho))) {
    WinoParams wp{};
    wp.x = x;
    wp.u = cw.wino;
    wp.y = y;
    wp.pre_scale = cw.pre_scale;
    wp.pre_shift = cw.pre_shift;
    wp.post_scale = cw.post_scale;
    wp.post_shift = cw.post_shift;
    wp.prelu = cw.prelu;
    wp.res = res;
    wp.B = B;
    wp.H = H;
    wp.W = W;
    wp.Cin = cw.cin;
    wp.Cout = cw.cout;
    // executed: 16 products per 2x2 output tile (padded tiles included) and (cin, cout) pair
    const double exec = 2.0 * 16.0 * B * ((H + 1) / 2) * ((W + 1) / 2) * (double)cw.cin * cw.cout;
    ProfScope ps(h, s, flop, FR_PROF_CONV_WINOGRAD, exec);
    hipError_t e = launch_wino(wp, cw.pre_scale != nullptr, epi, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("winograd launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  // the stage-1 stride-2 conv2 + MaxPool shortcut (64 -> 64 channels) of a batch of >= 16 crops on
  // its band kernel (conv_s2.hip: input rows staged once in LDS for all 9 taps); serving batches
  // keep the split-K direct path below, which spreads a few images' work over every CU
  if (g_s2band && !h->detector && h->prec == PREC_F32 && epi == EPI_AFFINE_RES_SUB && !cw.pre_scale && cw.cin2 == 0 &&
      nsplit == 1 && B >= 16 && res_H == H && res_W == W &&
      s2c64_supported(cw.cin, cw.cout, cw.kh, cw.kw, cw.stride, cw.pad, H, W)) {
    S2Params sp{};
    sp.x = x;
    sp.w = cw.w;
    sp.post_scale = cw.post_scale;
    sp.post_shift = cw.post_shift;
    sp.res = res;
    sp.y = y;
    sp.B = B;
    sp.H = H;
    sp.W = W;
    ProfScope ps(h, s, flop, FR_PROF_CONV_DIRECT);
    const hipError_t e = launch_s2c64(sp, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("stride-2 band conv launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  // Round-2 sweep with loads two K-steps ahead on the <= 32-accumulator tiles
  // (profiles/r02/sweep_s2.txt): 128x64/W8 also for the 256-channel stride-2 conv2 (111.9 ->
  // 115.6 TF/s) and 256x128/W8 for the 512-channel shortcut (49.4 -> 63.2).
  ConvTile tile = TILE_256x128_W8;
  if (cw.cout <= 64 || (cw.cout == 128 && epi == EPI_AFFINE_RES && cw.kh == 3) ||
      (cw.cout == 256 && epi == EPI_AFFINE_RES && cw.kh == 3 && cw.stride == 2))
    tile = TILE_128x64_W8;
  else if (cw.kh == 1 && cw.kw == 1 && p.H > 1)
    tile = cw.cout >= 512 ? TILE_256x128_W8 : TILE_128x128_W8;
  else if (p.H == 1)
    tile = TILE_64x128;  // gallery scores (1x1 GEMM)
  // embedding serving batches (M = B*Ho*Wo <= 4096: the stride-2 / 1x1 convs at batch <= ~20):
  // the 64x128 tile gives stream-K more, smaller tiles (batch 1: 2.28 -> 2.15 ms per forward).
  // The detector's tile set (conv_det.hip) has no 64x128 instance.
  // the detector's implicit-GEMM convs (tools/det_conv_sweep.py at the C4 shapes, 32 frames, every
  // tile of the instance sets): the stride-2 3x3 convs of 96 / 224 couts on 128x128/W8 (stage 2 / 3 /
  // 4 conv1: 299 -> 295, 123 -> 117, 77 -> 72 us), the stride-8 lateral 1x1 (M = 204,800, N = 64) on
  // 256x64 (72 -> 64 us); the rest keep the rule's tile (within 5 us of their best)
  if (h->detector && nsplit == 1) {
    if (cw.kh == 3 && cw.cout > 64)
      tile = TILE_128x128_W8;
    else if (cw.kh == 1 && cw.cout <= 64 && p.M >= 131072)
      tile = TILE_256x64;
  }
  if (cw.cin2 > 0 && g_conv2sc_tile >= 0 && nsplit == 1) tile = (ConvTile)g_conv2sc_tile;
  if (!h->detector && p.M <= 4096 && nsplit == 1) tile = TILE_64x128;
  // the head FC (split-K) of a serving batch (M = n <= 64 rows) or of <= 256 crops (tools/fc_sweep.py,
  // 32 splits: --batch 128 43.0 us on 128x64/W8 vs 106 on 256x128/W8; --batch 256 69.3 vs 111.8).
  // 129..256 rows on 64x128 (round 3, inside a one-lane IR-101 forward: 75.6 -> 63.9 us,
  // tools/gpu_fc_ab.sh)
  if (!h->detector && nsplit > 1 && cw.kh == 7 && p.M <= 256)
    tile = (p.M <= 64 || p.M > 128) ? TILE_64x128 : TILE_128x64_W8;
  // serving batches: a stride-2 conv2 (+ fused shortcut) as a split-K launch of >= 4 K-steps per
  // split in one round of workgroups, then a parallel fixup, instead of stream-K, whose last
  // arriver per tile summed ~20 slabs of 32 KB alone (batch 1: 26-31 us per launch)
  if (!h->detector && nsplit == 1 && p.M <= 4096 && cw.kh == 3 && h->prec == PREC_F32 && !cw.pre_scale &&
      (epi == EPI_AFFINE || epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_SUB) && sk_ws && h->cus > 0) {
    const long long ntile = (long long)((p.M + 63) / 64) * ((p.Cout + 127) / 128);
    const long long cap = (L ? L->sk_ws_floats : h->sk_ws_floats) / ((long long)p.M * p.Cout);
    int S = (int)std::min<long long>(std::min<long long>(32, p.steps_total / 4), std::min<long long>(h->cus / ntile, cap));
    if (S > 1) {
      ConvParams q = p;
      q.sk_cus = 0;
      q.steps_per_split = (p.steps_total + S - 1) / S;
      S = (p.steps_total + q.steps_per_split - 1) / q.steps_per_split;
      q.split_stride = (long long)p.M * p.Cout;
      q.y = sk_ws;
      q.res = nullptr;
      ProfScope ps(h, s, flop, FR_PROF_CONV_DIRECT);
      hipError_t e = launch_conv(q, TILE_64x128, false, EPI_RAW, S, s, h->prec);
      if (e == hipSuccess) e = launch_conv_split_fixup(p, epi, sk_ws, S, q.split_stride, s);
      if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("conv split-K launch: ") + hipGetErrorString(e));
      return FR_OK;
    }
  }
  ProfScope ps(h, s, flop, FR_PROF_CONV_DIRECT);
  hipError_t e = launch_conv(p, tile, cw.pre_scale != nullptr, epi, nsplit, s, h->prec);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("conv launch: ") + hipGetErrorString(e));
  return FR_OK;
}

// The handle's own workspace as lane 0.
LaneWs lane0_ws(fr_handle* h) {
  LaneWs L;
  for (int i = 0; i < 3; ++i) L.act[i] = h->act[i];
  L.sc_buf = h->sc_buf;
  L.partial = h->partial;
  L.w4part = h->w4part;
  L.sk_ws = h->sk_ws;
  L.sk_ws_floats = h->sk_ws_floats;
  L.sk_cnt = h->sk_cnt;
  L.sk_cnt_cap = h->sk_cnt_cap;
  return L;
}

// Frees lane l's (>= 1) activation workspace (after a failed ensure_lane).  Only work queued on
// the lane's own stream can still read it (earlier calls joined that stream back into theirs),
// so a sync of that stream -- not of the device, which would stall other handles -- suffices.
void release_lane(fr_handle* h, int l) {
  LaneWs& L = h->lane_ws[l];
  if (h->lane_stream[l]) (void)hipStreamSynchronize(h->lane_stream[l]);
  for (auto& a : L.act) {
    if (a) (void)hipFree(a);
    a = nullptr;
  }
  if (L.sc_buf) (void)hipFree(L.sc_buf);
  if (L.partial) (void)hipFree(L.partial);
  L.sc_buf = L.partial = nullptr;
  h->lane_batch[l] = 0;
}

// Lane l's (>= 1) workspace for up to `batch` crops, its stream and its join event.
int ensure_lane(fr_handle* h, int l, int batch) {
  LaneWs& L = h->lane_ws[l];
  if (h->lane_batch[l] < batch) {
    for (auto& a : L.act) {
      if (a) FR_HIP(h, hipFree(a));
      a = nullptr;
    }
    if (L.sc_buf) FR_HIP(h, hipFree(L.sc_buf));
    if (L.partial) FR_HIP(h, hipFree(L.partial));
    L.sc_buf = L.partial = nullptr;
    h->lane_batch[l] = 0;
    const size_t mb = batch;
    for (auto& a : L.act) FR_HIP(h, hipMalloc((void**)&a, mb * 112 * 112 * 64 * sizeof(float)));
    FR_HIP(h, hipMalloc((void**)&L.sc_buf, mb * 56 * 56 * 64 * sizeof(float)));
    // head partials: also a serving batch's 4x split (forward_lanes), whatever the lane's size
    FR_HIP(h, hipMalloc((void**)&L.partial, (size_t)fr_handle::HEAD_PARTS * std::max<size_t>(mb, h->max_batch) * 512 *
                                                sizeof(float)));
    h->lane_batch[l] = batch;
  }
  if (!L.w4part) {
    FR_HIP(h, hipMalloc((void**)&L.w4part, fr_handle::W4PART_FLOATS * sizeof(float)));
  }
  if (ensure_stream_k(h->device, &h->cus, &L.sk_ws, &L.sk_ws_floats, &L.sk_cnt, &L.sk_cnt_cap) != FR_OK)
    return fail(h, FR_ERR_HIP, "stream-K workspace allocation failed");
  if (!h->lane_stream[l]) FR_HIP(h, hipStreamCreateWithFlags(&h->lane_stream[l], hipStreamNonBlocking));
  if (!h->lane_fork) FR_HIP(h, hipEventCreateWithFlags(&h->lane_fork, hipEventDisableTiming));
  if (!h->lane_join[l]) FR_HIP(h, hipEventCreateWithFlags(&h->lane_join[l], hipEventDisableTiming));
  return FR_OK;
}

// One forward of up to max_batch crops: rgb (device) -> out (device) [n][512], as nl lanes
// (lane l: crops [off[l], off[l] + cnt[l]) on stream st[l] with workspace L[l]).  Every launch is
// issued for each lane in turn, so while one lane's layer runs its last, part-empty round the
// other lane's launch of the same layer is already queued.
int forward_lanes(fr_handle* h, const uint8_t* rgb, const int* off, const int* cnt, int nl, float* out,
                  int normalize, const hipStream_t* st, const LaneWs* L) {
  for (int l = 0; l < nl; ++l) {
    const int n = cnt[l];
    ProfScope ps(h, st[l], 2.0 * n * 112.0 * 112.0 * 64 * 27, 0);
    hipError_t e = launch_stem(rgb + (size_t)off[l] * 112 * 112 * 3, n, h->lut, h->stem_w, h->stem_scale,
                               h->stem_shift, h->stem_prelu, L[l].act[0], st[l]);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("stem launch: ") + hipGetErrorString(e));
  }
  int cur = 0, HW = 112;
  struct Y2Scope {
    fr_handle* h;
    ~Y2Scope() {
      h->convs_y2 = nullptr;
      h->convs_blk = 0;
    }
  } y2_scope{h};
  bool pre_done = false;  // the previous conv2 wrote this block's pre-BN input into L[0].sc_buf
  // Which activations are channel-blocked: in a one-lane serving forward, those passed between
  // two layers that run_conv puts on the serving conv kernel (same rule as its branch).
  const size_t nb = h->blocks.size();
  std::vector<char> all_convs(nb, 0), out_blk(nb, 0);
  {
    const bool serving = nl == 1 && h->convs_blocked;
    // the launches forward_lanes makes below: conv1 (pre-BN, BN, PReLU) at the block's input size;
    // conv2 with the fused conv shortcut (EPI_AFFINE + x2), the identity residual or the
    // MaxPool(1,2) one (an unfused conv shortcut keeps NHWC: its own launch reads the input)
    auto on_convs = [&](const ConvW& c, int hw, Epi epi, bool x2) {
      return serving && convs_takes(h, c, conv_shape(c, cnt[0], hw, hw), epi, 1, x2);
    };
    std::vector<char> conv2_convs(nb, 0);
    int hw = 112;
    for (size_t bi = 0; bi < nb; ++bi) {
      const BlockW& b = h->blocks[bi];
      const bool fused = b.has_sc_conv && h->fuse_shortcut && b.conv2_sc.w;
      const int ho = hw / b.spec.stride;
      conv2_convs[bi] = fused ? on_convs(b.conv2_sc, hw, EPI_AFFINE, true)
                              : !b.has_sc_conv && on_convs(b.conv2, hw, b.spec.stride == 1 ? EPI_AFFINE_RES
                                                                                          : EPI_AFFINE_RES_SUB, false);
      all_convs[bi] = conv2_convs[bi] && on_convs(b.conv1, hw, EPI_AFFINE_PRELU, false);
      hw = ho;
    }
    for (size_t bi = 0; bi + 1 < nb; ++bi) out_blk[bi] = conv2_convs[bi] && all_convs[bi + 1];
  }
  // Channel-blocked activations between F(4x4) layers (batches the serving kernel does not take):
  // a block's conv1 output when both convs of the block run on F(4x4); a block's output when its
  // conv2 and the next block's conv1 and conv2 (identity residual) do.  Every other tensor -- the
  // stem's, the stride-2 / shortcut / FC kernels' inputs and outputs -- stays NHWC.  The layouts
  // change nothing in the arithmetic: embeddings are bitwise the NHWC forward's (tested).
  std::vector<char> w4r_blk(nb, 0), w4y_blk(nb, 0);
  // (every lane must be past the serving kernel's batch limit: with an uneven split a smaller lane
  // could take the serving branch, which does not read the F(4x4) layout bits)
  int cnt_min = cnt[0];
  for (int l = 1; l < nl; ++l) cnt_min = std::min(cnt_min, cnt[l]);
  if (h->w4_blocked && cnt_min > h->convs_max_n && !h->detector) {
    std::vector<char> c1(nb, 0), c2(nb, 0);
    int hw = 112;
    for (size_t bi = 0; bi < nb; ++bi) {
      const BlockW& b = h->blocks[bi];
      const int ho = hw / b.spec.stride;
      c1[bi] = w4_takes(h, b.conv1, EPI_AFFINE_PRELU, 0, 0, hw, hw);
      // (a conv shortcut or a stride-2 conv2 runs on another kernel)
      c2[bi] = !b.has_sc_conv && b.spec.stride == 1 && w4_takes(h, b.conv2, EPI_AFFINE_RES, hw, hw, hw, hw);
      hw = ho;
    }
    for (size_t bi = 0; bi < nb; ++bi) {
      w4r_blk[bi] = c1[bi] && c2[bi];
      w4y_blk[bi] = c2[bi] && bi + 1 < nb && c1[bi + 1] && c2[bi + 1];
    }
    // a lone blocked block output makes both conv2s around it seams (residual and output in
    // different layouts: the RMIX instances, ~1% slower than NHWC, profiles/r05/w4ab_layouts_table.txt)
    // and no conv2 of the run gains: IR stages 1 and 4 (two F(4x4) blocks each) stay NHWC
    std::vector<char> keep(nb, 0);
    for (size_t bi = 0; bi < nb; ++bi)
      keep[bi] = w4y_blk[bi] && ((bi > 0 && w4y_blk[bi - 1]) || (bi + 1 < nb && w4y_blk[bi + 1]));
    w4y_blk = keep;
  }
  struct W4Scope {
    fr_handle* h;
    ~W4Scope() { h->w4_blk = 0; }
  } w4_scope{h};
  for (size_t bi = 0; bi < h->blocks.size(); ++bi) {
    const BlockW& b = h->blocks[bi];
    const int nxt = cur == 0 ? 1 : 0;
    const int Ho = HW / b.spec.stride;
    const bool in_blk = bi > 0 && out_blk[bi - 1], r_blk = all_convs[bi];
    h->convs_blk = (in_blk ? CONVS_BLK_X : 0) | (r_blk ? CONVS_BLK_Y : 0);
    const bool w4_in = bi > 0 && w4y_blk[bi - 1];
    h->w4_blk = (w4_in ? W4_BLK_X : 0) | (w4r_blk[bi] ? W4_BLK_Y : 0);
    for (int l = 0; l < nl; ++l) {
      int rc;
      if (pre_done) {
        // BN(x) is already in sc_buf: conv1 without pre-BN (and not on the F(4x4) / F(2x2)
        // filters, which have the pre-BN scale folded in)
        ConvW c1 = b.conv1;
        c1.pre_scale = c1.pre_shift = nullptr;
        c1.wino = c1.wino4 = c1.wino4_t = nullptr;
        rc = run_conv(h, c1, L[l].sc_buf, L[l].act[2], cnt[l], HW, HW, EPI_AFFINE_PRELU, nullptr, 0, 0, 1, 0, st[l],
                      &L[l]);
      } else {
        rc = run_conv(h, b.conv1, L[l].act[cur], L[l].act[2], cnt[l], HW, HW, EPI_AFFINE_PRELU, nullptr, 0, 0, 1,
                      0, st[l], &L[l]);
      }
      if (rc) return rc;
    }
    // a one-lane forward's conv2 on the serving conv kernel also writes the next block's pre-BN
    // input (sc_buf is free then unless this block's unfused shortcut uses it)
    const bool fused = b.has_sc_conv && h->fuse_shortcut && b.conv2_sc.w;
    h->convs_y2 = nullptr;
    h->convs_y2_done = false;
    h->convs_blk = (r_blk ? CONVS_BLK_X : 0) | (in_blk ? CONVS_BLK_X2 | CONVS_BLK_RES : 0) | (out_blk[bi] ? CONVS_BLK_Y : 0);
    h->w4_blk = (w4r_blk[bi] ? W4_BLK_X : 0) | (w4_in ? W4_BLK_RES : 0) | (w4y_blk[bi] ? W4_BLK_Y : 0);
    if (nl == 1 && h->convs_pre_epilogue && bi + 1 < h->blocks.size() && (fused || !b.has_sc_conv) &&
        h->blocks[bi + 1].conv1.pre_scale && (size_t)Ho * Ho * b.spec.depth <= (size_t)56 * 56 * 64) {
      h->convs_y2 = L[0].sc_buf;
      h->convs_y2_scale = h->blocks[bi + 1].conv1.pre_scale;
      h->convs_y2_shift = h->blocks[bi + 1].conv1.pre_shift;
    }
    for (int l = 0; l < nl; ++l) {
      float* x = L[l].act[cur];
      float* r = L[l].act[2];
      float* y = L[l].act[nxt];
      const int n = cnt[l];
      int rc;
      if (b.has_sc_conv && h->fuse_shortcut && b.conv2_sc.w) {
        rc = run_conv(h, b.conv2_sc, r, y, n, HW, HW, EPI_AFFINE, nullptr, 0, 0, 1, 0, st[l], &L[l], x);
      } else if (b.has_sc_conv) {
        rc = run_conv(h, b.sc, x, L[l].sc_buf, n, HW, HW, EPI_AFFINE, nullptr, 0, 0, 1, 0, st[l], &L[l]);
        if (rc) return rc;
        rc = run_conv(h, b.conv2, r, y, n, HW, HW, EPI_AFFINE_RES, L[l].sc_buf, Ho, Ho, 1, 0, st[l], &L[l]);
      } else if (b.spec.stride == 1) {
        rc = run_conv(h, b.conv2, r, y, n, HW, HW, EPI_AFFINE_RES, x, HW, HW, 1, 0, st[l], &L[l]);
      } else {
        rc = run_conv(h, b.conv2, r, y, n, HW, HW, EPI_AFFINE_RES_SUB, x, HW, HW, 1, 0, st[l], &L[l]);
      }
      if (rc) return rc;
    }
    pre_done = h->convs_y2_done;
    h->convs_y2 = nullptr;
    h->convs_y2_done = false;
    h->convs_blk = 0;
    h->w4_blk = 0;
    cur = nxt;
    HW = Ho;
  }
  for (int l = 0; l < nl; ++l) {
    const int n = cnt[l];
    const long long split_stride = (long long)n * 512;
    // serving batches (4 n <= max_batch): the FC's 784 K-steps in 98 splits of 8, so its 51 MB
    // of weights stream through many workgroups (batch 1: 78 us with 49 splits on 256x128, 27.7
    // with 196 on 64x128, 24.8 with 98: tools/fc_sweep.py --batch 1); larger batches in 32
    // splits of 25 (tools/fc_sweep.py: B = 256 79.2 -> 69.3 us, a 128-crop lane 47.3 -> 43.0,
    // vs 49 splits).  Decided by n alone (every lane's partials hold HEAD_PARTS x max_batch
    // rows), so a lane's part computes exactly as a one-lane forward of the same crops.
    const int hs = 4 * n <= h->max_batch ? fr_handle::HEAD_SPLIT_SMALL : fr_handle::HEAD_SPLIT;
    int rc = run_conv(h, h->head, L[l].act[cur], L[l].partial, n, 7, 7, EPI_RAW, nullptr, 0, 0, hs,
                      split_stride, st[l], &L[l]);
    if (rc) return rc;
    ProfScope ps(h, st[l], 0.0, 0);
    hipError_t e = launch_head_reduce(L[l].partial, hs, split_stride, h->fc_bias, h->bn1d_scale,
                                      h->bn1d_shift, out + (size_t)off[l] * 512, n, normalize, !h->arcface, st[l]);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("head launch: ") + hipGetErrorString(e));
  }
  return FR_OK;
}

// One forward of up to max_batch crops: rgb (device) -> out (device) [n][512].  With lanes on
// (fr_set_lanes), the batch runs as nl = min(lane_max, n / lane_min) near-equal parts: lanes
// 1 .. nl - 1 fork from s and join back into it, so the call is stream-ordered on s like a single
// forward.  Profiled and graph-captured forwards stay one lane (per-launch events would overlap;
// a captured graph replays on one stream).
int forward_chunk(fr_handle* h, const uint8_t* rgb, int n, float* out, int normalize, hipStream_t s) {
  const LaneWs L0 = lane0_ws(h);
  const int nl = (h->lane_min <= 0 || h->prof || h->capturing) ? 1 : std::max(1, std::min(h->lane_max, n / h->lane_min));
  if (nl == 1) {
    const int off = 0;
    return forward_lanes(h, rgb, &off, &n, 1, out, normalize, &s, &L0);
  }
  int off[MAX_LANES], cnt[MAX_LANES];
  hipStream_t st[MAX_LANES];
  LaneWs L[MAX_LANES];
  // lane buffers sized for the largest part of a max_batch forward, so they are made once
  const int cap = (h->max_batch + nl - 1) / nl;
  for (int l = 0, o = 0; l < nl; ++l) {
    cnt[l] = n / nl + (l < n % nl ? 1 : 0);
    off[l] = o;
    o += cnt[l];
    if (l > 0 && ensure_lane(h, l, std::max(cnt[l], cap)) != FR_OK) {
      // no memory for the second lane's workspace: run this and later forwards as one lane
      // (what worked before lanes existed) instead of failing the call; fr_set_lanes re-enables
      (void)hipGetLastError();  // clear the failed allocation's sticky error
      release_lane(h, l);
      h->lane_min = 0;  // visible through fr_get_lanes
      h->lanes_fallback = true;
      h->err.clear();  // the call succeeds: no stale allocation message for the next failure
      const int off0 = 0;
      return forward_lanes(h, rgb, &off0, &n, 1, out, normalize, &s, &L0);
    }
    st[l] = l ? h->lane_stream[l] : s;
    L[l] = l ? h->lane_ws[l] : L0;
  }
  FR_HIP(h, hipEventRecord(h->lane_fork, s));
  for (int l = 1; l < nl; ++l) FR_HIP(h, hipStreamWaitEvent(st[l], h->lane_fork, 0));
  const int rc = forward_lanes(h, rgb, off, cnt, nl, out, normalize, st, L);
  // join even after a failed launch, so that nothing of this call is left unordered behind s
  hipError_t e = hipSuccess;
  for (int l = 1; l < nl; ++l) {
    hipError_t e1 = hipEventRecord(h->lane_join[l], st[l]);
    if (e1 == hipSuccess) e1 = hipStreamWaitEvent(s, h->lane_join[l], 0);
    if (e == hipSuccess) e = e1;
  }
  if (rc) return rc;
  FR_HIP(h, e);
  return FR_OK;
}

void clear_graphs(fr_handle* h) {
  if (h->graphs.empty()) return;
  (void)hipDeviceSynchronize();  // no replay of these graphs may still be in flight
  for (auto& g : h->graphs) (void)hipGraphExecDestroy(g.exec);
  h->graphs.clear();
}

// Capture forward_chunk(in_stage -> emb_stage) for n crops as a hipGraph.  Every pointer and
// size a launch takes is fixed for (n, normalize) once the handle is finalised, and the
// stream-K tickets re-arm themselves, so the graph replays without updates.
int capture_graph(fr_handle* h, int n, int normalize) {
  if (!h->cap_stream) FR_HIP(h, hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
  FR_HIP(h, hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
  h->capturing = true;
  const int rc = forward_chunk(h, h->in_stage, n, h->emb_stage, normalize, h->cap_stream);
  h->capturing = false;
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(h->cap_stream, &g);
  if (rc != FR_OK || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    return rc != FR_OK ? rc : fail(h, FR_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ei != hipSuccess) return fail(h, FR_ERR_HIP, std::string("graph instantiate: ") + hipGetErrorString(ei));
  h->graphs.push_back({n, normalize, ex});
  return FR_OK;
}

// One forward of n <= max_batch crops from in_stage to emb_stage.  Small n (the serving
// pattern: a frame's faces, or batch 1) is launch-bound, so with fr_set_graph_batch those
// forwards replay a captured graph: the first call for an n runs eagerly (loading every
// kernel), then captures; later calls are one hipGraphLaunch.
int forward_staged(fr_handle* h, int n, int normalize, hipStream_t s) {
  if (n > h->graph_max_n || h->prof) return forward_chunk(h, h->in_stage, n, h->emb_stage, normalize, s);
  for (const auto& g : h->graphs)
    if (g.n == n && g.normalize == normalize) {
      FR_HIP(h, hipGraphLaunch(g.exec, s));
      return FR_OK;
    }
  const int rc = forward_chunk(h, h->in_stage, n, h->emb_stage, normalize, s);
  if (rc != FR_OK) return rc;
  return capture_graph(h, n, normalize);
}

int embed_device(fr_handle* h, const uint8_t* rgb, int n, float* out, int normalize, hipStream_t s) {
  if (n > 0 && n <= h->graph_max_n && !h->prof) {
    FR_HIP(h, hipMemcpyAsync(h->in_stage, rgb, (size_t)n * 112 * 112 * 3, hipMemcpyDeviceToDevice, s));
    const int rc = forward_staged(h, n, normalize, s);
    if (rc != FR_OK) return rc;
    FR_HIP(h, hipMemcpyAsync(out, h->emb_stage, (size_t)n * 512 * sizeof(float), hipMemcpyDeviceToDevice, s));
    return FR_OK;
  }
  for (int off = 0; off < n; off += h->max_batch) {
    const int bn = std::min(h->max_batch, n - off);
    int rc = forward_chunk(h, rgb + (size_t)off * 112 * 112 * 3, bn, out + (size_t)off * 512, normalize, s);
    if (rc) return rc;
  }
  return FR_OK;
}

// cv2.resize(crop, (112, 112), INTER_LINEAR) of n H x W crops (face_embedder.py:94-96), device to
// device, in OpenCV's fixed point (the letterbox kernel of the detector with a 112 x 112 canvas).
// The coefficient tables are built once per source size and kept on the device, at most
// RS_TABS_MAX of them (least recently used one replaced: a server resizing crops of arbitrary
// sizes keeps a bounded cache).
int resize_device(fr_handle* h, const uint8_t* src, int n, int H, int W, uint8_t* dst, hipStream_t s) {
  fr_handle::ResizeTab* t = nullptr;
  for (auto& r : h->rs_tabs)
    if (r.H == H && r.W == W) t = &r;
  if (!t) {
    std::vector<int> host(4 * (112 + 112));
    resize_axis_table(112, W, host.data());
    resize_axis_table(112, H, host.data() + 4 * 112);
    if (h->rs_tabs.size() >= fr_handle::RS_TABS_MAX) {
      t = &*std::min_element(h->rs_tabs.begin(), h->rs_tabs.end(),
                             [](const fr_handle::ResizeTab& a, const fr_handle::ResizeTab& b) { return a.used < b.used; });
      // the replaced table may still be read by a resize queued earlier, on s or on another
      // stream: the copy waits for that launch (its event), then goes in stream order on s
      if (t->last) FR_HIP(h, hipStreamWaitEvent(s, t->last, 0));
      FR_HIP(h, hipMemcpyAsync(t->tab, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice, s));
      FR_HIP(h, hipStreamSynchronize(s));  // the pageable host table must outlive the copy
      t->H = H;
      t->W = W;
      t->simd_end = resize_simd_end(112 * 3);
    } else {
      int* d = nullptr;
      FR_HIP(h, hipMalloc((void**)&d, host.size() * sizeof(int)));
      FR_HIP(h, hipMemcpy(d, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice));
      h->rs_tabs.push_back({H, W, resize_simd_end(112 * 3), d, 0, nullptr});
      t = &h->rs_tabs.back();
    }
  }
  t->used = ++h->rs_clock;
  ProfScope ps(h, s, 0.0, 0);
  hipError_t e = launch_letterbox(src, n, H, W, t->tab, t->tab + 4 * 112, 112, 112, t->simd_end, 112, 112, dst, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("resize launch: ") + hipGetErrorString(e));
  // (never inside a graph capture: captured forwards start at in_stage, after the resize)
  if (!t->last) FR_HIP(h, hipEventCreateWithFlags(&t->last, hipEventDisableTiming));
  FR_HIP(h, hipEventRecord(t->last, s));
  return FR_OK;
}

int check_crop_size(fr_handle* h, int height, int width) {
  if (height < 1 || width < 1 || height > 8192 || width > 8192)
    return fail(h, FR_ERR_INVALID_ARGUMENT, "crop height/width must be in [1, 8192]");
  return FR_OK;
}

// Embed n crops of any size: 112 x 112 go straight to the forward, others through resize_device
// one max_batch chunk at a time.
int embed_any(fr_handle* h, const uint8_t* rgb, int n, int height, int width, float* out, int normalize,
              hipStream_t s) {
  if (height == 112 && width == 112) return embed_device(h, rgb, n, out, normalize, s);
  for (int off = 0; off < n; off += h->max_batch) {
    const int bn = std::min(h->max_batch, n - off);
    int rc = resize_device(h, rgb + (size_t)off * height * width * 3, bn, height, width, h->rs_stage, s);
    if (rc) return rc;
    rc = embed_device(h, h->rs_stage, bn, out + (size_t)off * 512, normalize, s);
    if (rc) return rc;
  }
  return FR_OK;
}

int match_device(fr_handle* h, const float* Q, int n, int k, int32_t* idx, float* score, hipStream_t s) {
  if (h->G <= 0) return fail(h, FR_ERR_STATE, "gallery is empty (fr_gallery_set first)");
  if (k < 1 || k > h->G) return fail(h, FR_ERR_INVALID_ARGUMENT, "k must be in [1, G]");
  if (n <= 0) return FR_OK;
  int rc;
  if (n <= 16 && (long long)n * h->G * 4 < (1ll << 31)) {
    // serving-sized: normalisation fused into one scores launch (embed_misc.hip), then top-k
    rc = ensure_buf(h, (void**)&h->scores, &h->scores_cap, (size_t)n * h->G * sizeof(float));
    if (rc) return rc;
    ProfScope ps(h, s, 0.0, 0);
    hipError_t e = launch_scores_small(Q, h->gallery, h->G, h->scores, n, s);
    if (e == hipSuccess) e = launch_topk(h->scores, n, h->G, k, idx, score, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("match launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  rc = ensure_buf(h, (void**)&h->qn, &h->qn_cap, (size_t)n * 512 * sizeof(float));
  if (rc) return rc;
  if (ensure_stream_k(h->device, &h->cus, &h->sk_ws, &h->sk_ws_floats, &h->sk_cnt, &h->sk_cnt_cap) != FR_OK)
    return fail(h, FR_ERR_HIP, "stream-K workspace allocation failed");
  {
    ProfScope ps(h, s, 0.0, 0);
    hipError_t e = launch_l2norm_rows(Q, h->qn, n, 512, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("l2norm launch: ") + hipGetErrorString(e));
  }
  ConvW g;
  g.w = h->gallery;
  g.cin = 512;
  g.cout = h->G;
  g.kh = g.kw = 1;
  g.stride = 1;
  g.pad = 0;
  // score matrices below 2 GiB (the conv epilogue's 32-bit offsets): queries in chunks
  const int nc = (int)std::max<long long>(1, std::min<long long>(n, ((1ll << 31) - 1) / ((long long)h->G * 4)));
  rc = ensure_buf(h, (void**)&h->scores, &h->scores_cap, (size_t)nc * h->G * sizeof(float));
  if (rc) return rc;
  for (int q0 = 0; q0 < n; q0 += nc) {
    const int qn = std::min(nc, n - q0);
    rc = run_conv(h, g, h->qn + (size_t)q0 * 512, h->scores, qn, 1, 1, EPI_RAW, nullptr, 0, 0, 1, 0, s);
    if (rc) return rc;
    ProfScope ps(h, s, 0.0, 0);
    hipError_t e = launch_topk(h->scores, qn, h->G, k, idx + (size_t)q0 * k, score + (size_t)q0 * k, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("topk launch: ") + hipGetErrorString(e));
  }
  return FR_OK;
}

// ---- FaceAligner (face_recognition.py:50-75) host side: cv2.estimateAffinePartial2D with its
// defaults (RANSAC 3 px / 2000 iterations / 0.99, 10 LM refine iterations), restating OpenCV's
// ptsetreg.cpp + levmarq.cpp, and warpAffine's inverse.  Same IEEE operation order as
// oracle/align_ref.py (fit_similarity and helpers), so both produce identical doubles.
#pragma clang fp contract(off)
namespace {
constexpr double kDblMin = 2.2250738585072014e-308, kDblEps = 2.220446049250313e-16;
constexpr double kFltEps = 1.1920928955078125e-07;

// cv::RNG (core/rand.cpp): 64-bit multiply-with-carry
struct CvRng {
  uint64_t state;
  explicit CvRng(uint64_t s) : state(s ? s : 0xffffffffull) {}
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + (unsigned)a); }
};

// AffinePartial2DEstimatorCallback::runKernel: the similarity through 2 point pairs
void kernel2(const double f[4], const double t[4], double H[6]) {
  const double x1 = f[0], y1 = f[1], x2 = f[2], y2 = f[3];
  const double X1 = t[0], Y1 = t[1], X2 = t[2], Y2 = t[3];
  const double den = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2);
  const double d = den != 0 ? 1. / den : INFINITY;
  const double S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2));
  const double S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2));
  const double S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2));
  const double S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2));
  H[0] = H[4] = S0;
  H[1] = -S1;
  H[2] = S2;
  H[3] = S1;
  H[5] = S3;
}

// computeError (float32 model and arithmetic) + findInliers
int find_inliers(const double M[6], const float* src, const float* dst, int n, double thr, bool* mask) {
  const float F0 = (float)M[0], F1 = (float)M[1], F2 = (float)M[2], F3 = (float)M[3], F4 = (float)M[4], F5 = (float)M[5];
  const float t = (float)(thr * thr);
  int nz = 0;
  for (int i = 0; i < n; ++i) {
    const float a = F0 * src[2 * i] + F1 * src[2 * i + 1] + F2 - dst[2 * i];
    const float b = F3 * src[2 * i] + F4 * src[2 * i + 1] + F5 - dst[2 * i + 1];
    mask[i] = a * a + b * b <= t;
    nz += mask[i];
  }
  return nz;
}

// RANSACUpdateNumIters, (1 - ep)^2 as one product
int update_num_iters(double p, double ep, int max_iters) {
  p = std::min(std::max(p, 0.), 1.);
  ep = std::min(std::max(ep, 0.), 1.);
  double num = std::max(1. - p, kDblMin);
  const double q = 1. - ep;
  double denom = 1. - q * q;
  if (denom < kDblMin) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)std::nearbyint(num / denom);
}

// Gaussian elimination with partial pivoting (n = 4); a zero pivot leaves its unknown 0
void solve4(const double A[4][4], const double b[4], double x[4]) {
  double M[4][5];
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) M[i][j] = A[i][j];
    M[i][4] = b[i];
  }
  for (int c = 0; c < 4; ++c) {
    int p = c;
    for (int r = c + 1; r < 4; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
    if (p != c)
      for (int k = 0; k < 5; ++k) std::swap(M[c][k], M[p][k]);
    if (M[c][c] == 0.0) continue;
    for (int r = c + 1; r < 4; ++r) {
      const double f = M[r][c] / M[c][c];
      for (int k = c; k < 5; ++k) M[r][k] = M[r][k] - f * M[c][k];
    }
  }
  for (int c = 3; c >= 0; --c) {
    x[c] = 0.0;
    if (M[c][c] == 0.0) continue;
    double s = M[c][4];
    for (int k = c + 1; k < 4; ++k) s = s - M[c][k] * x[k];
    x[c] = s / M[c][c];
  }
}

// AffinePartial2DRefineCallback::compute, h = (a, b, tx, ty): residuals r[2n] and, if J, the
// normal equations A = J^T J, v = J^T r (sums in index order)
void refine_compute(const double h[4], const double* src, const double* dst, int n, double* r, double A[4][4],
                    double v[4]) {
  for (int i = 0; i < n; ++i) {
    const double Mx = src[2 * i], My = src[2 * i + 1];
    const double xi = h[0] * Mx - h[1] * My + h[2];
    const double yi = h[1] * Mx + h[0] * My + h[3];
    r[2 * i] = xi - dst[2 * i];
    r[2 * i + 1] = yi - dst[2 * i + 1];
  }
  if (!A) return;
  double J[16][4];
  for (int i = 0; i < n; ++i) {
    const double Mx = src[2 * i], My = src[2 * i + 1];
    const double j0[4] = {Mx, -My, 1., 0.}, j1[4] = {My, Mx, 0., 1.};
    for (int c = 0; c < 4; ++c) {
      J[2 * i][c] = j0[c];
      J[2 * i + 1][c] = j1[c];
    }
  }
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int k = 0; k < 2 * n; ++k) s += J[k][i] * J[k][j];
      A[i][j] = s;
    }
    double s = 0.0;
    for (int k = 0; k < 2 * n; ++k) s += J[k][i] * r[k];
    v[i] = s;
  }
}

double sumsq(const double* r, int m) {
  double s = 0.0;
  for (int i = 0; i < m; ++i) s += r[i] * r[i];
  return s;
}

double dot4(const double* a, const double* b) {
  double s = 0.0;
  for (int i = 0; i < 4; ++i) s += a[i] * b[i];
  return s;
}

double maxabs(const double* a, int m) {
  double s = 0.0;
  for (int i = 0; i < m; ++i) s = std::max(s, std::fabs(a[i]));
  return s;
}

// LMSolverImpl::run (levmarq.cpp, OpenCV 3.x-4.5)
void lm_refine(double x[4], const double* src, const double* dst, int n, int max_iters) {
  double r[16], rd[16], A[4][4], v[4], D[4];
  refine_compute(x, src, dst, n, r, A, v);
  double S = sumsq(r, 2 * n);
  for (int i = 0; i < 4; ++i) D[i] = A[i][i];
  const double Rlo = 0.25, Rhi = 0.75;
  double lambda = 1, lc = 0.75;
  for (int iter = 0;;) {
    double Ap[4][4], d[4], xd[4], temp[4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) Ap[i][j] = A[i][j] + (i == j ? lambda * D[i] : 0.0);
    solve4(Ap, v, d);
    for (int i = 0; i < 4; ++i) xd[i] = x[i] - d[i];
    refine_compute(xd, src, dst, n, rd, nullptr, nullptr);
    const double Sd = sumsq(rd, 2 * n);
    for (int i = 0; i < 4; ++i) temp[i] = -dot4(A[i], d) + 2.0 * v[i];  // gemm(A, d, -1, v, 2)
    const double dS = dot4(d, temp);
    const double R = (S - Sd) / (std::fabs(dS) > kDblEps ? dS : 1.0);
    if (R > Rhi) {
      lambda *= 0.5;
      if (lambda < lc) lambda = 0;
    } else if (R < Rlo) {
      const double t = dot4(d, v);
      double nu = (Sd - S) / (std::fabs(t) > kDblEps ? t : 1.0) + 2.0;
      nu = std::min(std::max(nu, 2.0), 10.0);
      if (lambda == 0) {
        double maxval = kDblEps;
        for (int i = 0; i < 4; ++i) {
          double e[4] = {0, 0, 0, 0}, col[4];
          e[i] = 1.0;
          solve4(A, e, col);
          maxval = std::max(maxval, std::fabs(col[i]));
        }
        lambda = lc = 1.0 / maxval;
        nu *= 0.5;
      }
      lambda *= nu;
    }
    if (Sd < S) {
      S = Sd;
      memcpy(x, xd, sizeof(xd));
      refine_compute(x, src, dst, n, r, A, v);
    }
    ++iter;
    if (!(iter < max_iters && maxabs(d, 4) >= kFltEps && maxabs(r, 2 * n) >= kFltEps)) break;
  }
}
}  // namespace

// estimateAffinePartial2D(src, dst)[0]: returns false (M NaN) where cv2 returns None
bool fit_similarity(const float* src_f, const float* dst_f, int n, double M[6]) {
  for (int i = 0; i < 6; ++i) M[i] = NAN;
  if (n < 2 || n > 8) return false;
  double src[16], dst[16];
  for (int i = 0; i < 2 * n; ++i) {
    src[i] = src_f[i];
    dst[i] = dst_f[i];
  }
  if (n == 2) {
    kernel2(src, dst, M);
    return true;
  }
  CvRng rng(~0ull);
  bool mask[8], best_mask[8];
  double best[6];
  int niters = 2000, good = 0;
  for (int it = 0; it < niters; ++it) {
    const int i0 = rng.uniform(0, n);
    int i1 = rng.uniform(0, n);
    while (i1 == i0) i1 = rng.uniform(0, n);
    const double f[4] = {src[2 * i0], src[2 * i0 + 1], src[2 * i1], src[2 * i1 + 1]};
    const double t[4] = {dst[2 * i0], dst[2 * i0 + 1], dst[2 * i1], dst[2 * i1 + 1]};
    double Mi[6];
    kernel2(f, t, Mi);
    const int g = find_inliers(Mi, src_f, dst_f, n, 3.0, mask);
    if (g > std::max(good, 1)) {
      memcpy(best, Mi, sizeof(best));
      memcpy(best_mask, mask, sizeof(mask));
      good = g;
      niters = update_num_iters(0.99, (double)(n - g) / n, niters);
    }
  }
  if (good <= 0) return false;
  double si[16], di[16];
  int m = 0;
  for (int i = 0; i < n; ++i)
    if (best_mask[i]) {
      si[2 * m] = src[2 * i];
      si[2 * m + 1] = src[2 * i + 1];
      di[2 * m] = dst[2 * i];
      di[2 * m + 1] = dst[2 * i + 1];
      ++m;
    }
  double h[4] = {best[0], best[3], best[2], best[5]};
  lm_refine(h, si, di, m, 10);
  M[0] = M[4] = h[0];
  M[1] = -h[1];
  M[2] = h[2];
  M[3] = h[1];
  M[5] = h[3];
  return true;
}

void invert_affine(const double Mf[6], double Mi[6]) {
  double m[6];
  memcpy(m, Mf, sizeof(m));
  double D = m[0] * m[4] - m[1] * m[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = m[4] * D, A22 = m[0] * D;
  m[0] = A11;
  m[1] *= -D;
  m[3] *= -D;
  m[4] = A22;
  const double b1 = -m[0] * m[2] - m[1] * m[5];
  const double b2 = -m[3] * m[2] - m[4] * m[5];
  m[2] = b1;
  m[5] = b2;
  memcpy(Mi, m, sizeof(m));
}
#pragma clang fp contract(on)

void reference_template(int S, float t[10]) {
  const double r[10] = {0.34, 0.46, 0.66, 0.46, 0.50, 0.61, 0.37, 0.74, 0.63, 0.74};
  for (int i = 0; i < 10; ++i) t[i] = (float)(r[i] * S);
}

const std::vector<float>* getp(fr_handle* h, const std::string& k) {
  auto it = h->params.find(k);
  return it == h->params.end() ? nullptr : &it->second;
}

}  // namespace

extern "C" {

int fr_create(const char* architecture, const char* model_type, int device, int max_batch, fr_handle** out) {
  if (!out) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  const std::string arch = architecture ? architecture : "";
  const std::string mt = model_type ? model_type : "";
  const bool detector = arch == "scrfd_10g";
  bool ok = detector;
  auto specs = detector ? std::vector<BlockSpec>{} : block_specs(arch, &ok);
  if (!ok)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT,
                "Unknown architecture: " + arch + ". Available: ['ir_50', 'ir_101', 'scrfd_10g']");
  if (detector ? mt != "scrfd" : (mt != "adaface" && mt != "arcface"))
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT,
                "Unknown model_type: " + mt + (detector ? ". scrfd_10g takes 'scrfd'" : ". Must be 'adaface' or 'arcface'"));
  if (max_batch < 1 || max_batch > 512)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "max_batch must be in [1, 512]");
  if (detector && max_batch > 64)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "scrfd_10g: max_batch (frames per forward) must be in [1, 64]");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(nullptr, FR_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "device index out of range");
  auto h = std::make_unique<fr_handle>();
  h->arch = arch;
  h->model_type = mt;
  h->arcface = mt == "arcface";
  h->device = device;
  h->max_batch = max_batch;
  h->lane_min = detector ? 0 : FR_LANES_MIN_DEFAULT;
  h->lane_max = FR_LANES_MAX_DEFAULT;
  h->specs = specs;
  h->detector = detector;
  h->expected = detector ? detector_schema() : h->arcface ? schema_arcface(specs) : schema(specs);
  *out = h.release();
  return FR_OK;
}

int fr_destroy(fr_handle* h) {
  if (!h) return FR_OK;
  {
    DeviceGuard g(h->device);
    (void)hipDeviceSynchronize();
    delete h;
  }
  return FR_OK;
}

int fr_set_param(fr_handle* h, const char* name, const float* host_data, int64_t numel) {
  if (!h || !name) return fail(h, FR_ERR_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  const std::string k = name;
  auto it = h->expected.find(k);
  if (it == h->expected.end()) return fail(h, FR_ERR_INVALID_ARGUMENT, "Unexpected key(s) in state_dict: \"" + k + "\"");
  if (k.size() > 20 && k.compare(k.size() - 20, 20, ".num_batches_tracked") == 0) return FR_OK;
  if (numel != (int64_t)it->second || (!host_data && numel > 0))
    return fail(h, FR_ERR_INVALID_ARGUMENT,
                "size mismatch for " + k + ": expected " + std::to_string(it->second) + " elements, got " +
                    std::to_string(numel));
  h->params[k].assign(host_data, host_data + numel);
  h->finalized = false;
  return FR_OK;
}

// F(2x2,3x3) filters G g G^T of every eligible conv, built on the device from the arena the
// first time the algorithm is selected after fr_finalize (16/9 of the 3x3 weights).
static int ensure_wino2(fr_handle* h) {
  if (h->wino_arena) return FR_OK;
  std::vector<ConvW*> wconvs;
  size_t wfloats = 0;
  for (auto& b : h->blocks)
    for (ConvW* c : {&b.conv1, &b.conv2}) {
      c->wino = nullptr;
      if (c->w && wino_supported(c->cin, c->cout, c->kh, c->kw, c->stride, c->pad)) {
        wconvs.push_back(c);
        wfloats += wino_weight_floats(c->cout, c->cin);
      }
    }
  if (!wfloats) return FR_OK;
  FR_HIP(h, hipMalloc((void**)&h->wino_arena, wfloats * sizeof(float)));
  size_t off = 0;
  for (ConvW* c : wconvs) {
    c->wino = h->wino_arena + off;
    FR_HIP(h, launch_wino_weights(c->w, c->wino, c->cout, c->cin, nullptr));
    off += wino_weight_floats(c->cout, c->cin);
  }
  FR_HIP(h, hipDeviceSynchronize());
  return FR_OK;
}

// F(4x4,3x3) filters of every eligible conv, built on the device from the arena the first
// time the algorithm is selected after fr_finalize (36/9 = 4x the 3x3 weights).
// The pre-activation BN of a conv1 is folded: U = G (g * scale) G^T and t = shift / scale is
// added to the in-image input pixels, so BN(x) = scale (x + t).  A conv whose BN scale has a
// zero (t not finite) keeps the direct kernel.
static bool wino4_pre_fold(const ConvW* c, std::vector<float>& t) {
  t.assign(c->cin, 0.f);
  if (!c->pre_scale) return true;
  std::vector<float> sc(c->cin), sh(c->cin);
  if (hipMemcpy(sc.data(), c->pre_scale, c->cin * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(sh.data(), c->pre_shift, c->cin * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    return false;
  for (int i = 0; i < c->cin; ++i) {
    t[i] = sh[i] / sc[i];
    if (sc[i] == 0.f || !std::isfinite(t[i])) return false;
  }
  return true;
}

static int ensure_wino4(fr_handle* h) {
  if (h->wino4_arena) return FR_OK;
  std::vector<ConvW*> wconvs;
  std::vector<std::vector<float>> ts;
  size_t wfloats = 0;
  std::vector<ConvW*> all;
  for (auto& b : h->blocks)
    for (ConvW* c : {&b.conv1, &b.conv2}) all.push_back(c);
  detector_convs(h->det, all);
  for (ConvW* c : all) {
    c->wino4 = nullptr;
    c->wino4_t = nullptr;
    std::vector<float> t;
    if (c->w && wino4_supported(c->cin, c->cout, c->kh, c->kw, c->stride, c->pad) && wino4_pre_fold(c, t)) {
      wconvs.push_back(c);
      ts.push_back(std::move(t));
      wfloats += wino4_weight_floats(c->cout, c->cin) + (c->pre_scale ? c->cin : 0);
    }
  }
  if (!wfloats) return FR_OK;
  FR_HIP(h, hipMalloc((void**)&h->wino4_arena, wfloats * sizeof(float)));
  size_t off = 0;
  for (size_t k = 0; k < wconvs.size(); ++k) {
    ConvW* c = wconvs[k];
    c->wino4 = h->wino4_arena + off;
    off += wino4_weight_floats(c->cout, c->cin);
    FR_HIP(h, launch_wino4_weights(c->w, c->pre_scale, c->wino4, c->cout, c->cin, nullptr));
    if (c->pre_scale) {
      c->wino4_t = h->wino4_arena + off;
      off += c->cin;
      FR_HIP(h, hipMemcpy(c->wino4_t, ts[k].data(), c->cin * sizeof(float), hipMemcpyHostToDevice));
    }
  }
  FR_HIP(h, hipDeviceSynchronize());
  return FR_OK;
}

static void drop_wino4(fr_handle* h) {
  (void)hipFree(h->wino4_arena);
  h->wino4_arena = nullptr;
  std::vector<ConvW*> all;
  for (auto& b : h->blocks)
    for (ConvW* c : {&b.conv1, &b.conv2}) all.push_back(c);
  detector_convs(h->det, all);
  for (ConvW* c : all) {
    c->wino4 = nullptr;
    c->wino4_t = nullptr;
  }
}

// The serving conv kernel's filters (fragment order) for every body 3x3 conv it can run: conv1,
// conv2 and the fused conv2 + shortcut of each block (embedding models only).
static int ensure_convs_weights(fr_handle* h) {
  if (h->convs_arena || h->detector) return FR_OK;
  std::vector<ConvW*> cs;
  size_t floats = 0;
  for (auto& b : h->blocks)
    for (ConvW* c : {&b.conv1, &b.conv2, &b.conv2_sc}) {
      c->w_frag = nullptr;
      if (c->w && c->kh == 3 && c->kw == 3 && c->cin % 16 == 0 && c->cout % 16 == 0 && c->cin2 % 16 == 0) {
        cs.push_back(c);
        floats += (size_t)c->cout * (9 * c->cin + c->cin2);
      }
    }
  if (!floats) return FR_OK;
  FR_HIP(h, hipMalloc((void**)&h->convs_arena, floats * sizeof(float)));
  size_t off = 0;
  for (ConvW* c : cs) {
    c->w_frag = h->convs_arena + off;
    off += (size_t)c->cout * (9 * c->cin + c->cin2);
    FR_HIP(h, launch_convs_weights(c->w, c->w_frag, c->cout, 9 * c->cin + c->cin2, nullptr));
  }
  FR_HIP(h, hipDeviceSynchronize());
  return FR_OK;
}

static int ensure_winograd(fr_handle* h) {
  if (!h->winograd) return FR_OK;
  if (h->wino_m == 2) return ensure_wino2(h);
  // bf16x3 runs the direct split-bf16 kernel; the F(4x4) path is f32 only
  return ensure_wino4(h);
}

int fr_finalize(fr_handle* h) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  std::string missing;
  for (const auto& kv : h->expected) {
    if (kv.first.size() > 20 && kv.first.compare(kv.first.size() - 20, 20, ".num_batches_tracked") == 0) continue;
    if (!h->params.count(kv.first)) missing += (missing.empty() ? "\"" : ", \"") + kv.first + "\"";
  }
  if (!missing.empty()) return fail(h, FR_ERR_MISSING_PARAM, "Missing key(s) in state_dict: " + missing);
  DeviceGuard dg(h->device);
  if (int rc = ensure_dev_err(h)) return rc;
  clear_graphs(h);
  if (h->detector) {
    int rc = detector_finalize(h);
    if (rc) return rc;
    // the detector's stride-1 3x3 convs run on the F(4x4) kernel as well (run_conv)
    drop_wino4(h);
    if (h->wino_m == 4 && (rc = ensure_winograd(h)) != FR_OK) return rc;
    h->finalized = true;
    return FR_OK;
  }

  Packer pk;
  std::vector<float> sc, sh;
  auto P = [&](const std::string& k) -> const std::vector<float>& { return *getp(h, k); };
  auto bn = [&](const std::string& p, float** dsc, float** dsh, bool affine = true) {
    bn_fold(affine ? &P(p + ".weight") : nullptr, affine ? &P(p + ".bias") : nullptr, P(p + ".running_mean"),
            P(p + ".running_var"), sc, sh);
    pk.put(dsc, sc);
    pk.put(dsh, sh);
  };

  // preprocessing LUT in float64 then float32: AdaFace (v/255.0 - 0.5)/0.5 (face_embedder.py:99-101),
  // ArcFace (v - 127.5)/127.5 (face_embedder.py:105-110)
  std::vector<float> lut(256);
  for (int v = 0; v < 256; ++v) lut[v] = h->arcface ? (float)((v - 127.5) / 127.5) : (float)((v / 255.0 - 0.5) / 0.5);
  pk.put(&h->lut, lut);
  const bool af = h->arcface;
  // stem: [64][3][3][3] (BGR channel order) -> [ky][kx][c_rgb][64]
  {
    const auto& w = P(af ? "conv1.weight" : "input_layer.0.weight");
    std::vector<float> r(27 * 64);
    for (int o = 0; o < 64; ++o)
      for (int c = 0; c < 3; ++c)
        for (int y = 0; y < 3; ++y)
          for (int x = 0; x < 3; ++x) r[((y * 3 + x) * 3 + (2 - c)) * 64 + o] = w[((o * 3 + c) * 3 + y) * 3 + x];
    pk.put(&h->stem_w, r);
    bn(af ? "bn1" : "input_layer.1", &h->stem_scale, &h->stem_shift);
    pk.put(&h->stem_prelu, P(af ? "prelu.weight" : "input_layer.2.weight"));
  }
  h->blocks.assign(h->specs.size(), BlockW{});
  for (size_t i = 0; i < h->specs.size(); ++i) {
    const auto& s = h->specs[i];
    BlockW& b = h->blocks[i];
    b.spec = s;
    const UnitKeys k = unit_keys(af, h->specs, i);
    b.conv1.cin = s.cin;
    b.conv1.cout = s.depth;
    b.conv1.kh = b.conv1.kw = 3;
    b.conv1.stride = 1;
    b.conv1.pad = 1;
    pk.put(&b.conv1.w, repack_oihw(P(k.conv1), s.depth, s.cin, 3, 3));
    bn(k.pre_bn, &b.conv1.pre_scale, &b.conv1.pre_shift);
    bn(k.mid_bn, &b.conv1.post_scale, &b.conv1.post_shift);
    pk.put(&b.conv1.prelu, P(k.prelu));
    b.conv2.cin = s.depth;
    b.conv2.cout = s.depth;
    b.conv2.kh = b.conv2.kw = 3;
    b.conv2.stride = s.stride;
    b.conv2.pad = 1;
    const std::vector<float> w2 = repack_oihw(P(k.conv2), s.depth, s.depth, 3, 3);
    pk.put(&b.conv2.w, w2);
    bn(k.out_bn, &b.conv2.post_scale, &b.conv2.post_shift);
    const std::vector<float> sc2 = sc, sh2 = sh;
    // AdaFace: conv shortcut only where the width changes (MaxPool2d(1,2) in stage 1);
    // ArcFace: a conv1x1 downsample on every strided unit
    if (af ? s.stride == 2 : s.cin != s.depth) {
      b.has_sc_conv = true;
      b.sc.cin = s.cin;
      b.sc.cout = s.depth;
      b.sc.kh = b.sc.kw = 1;
      b.sc.stride = s.stride;
      b.sc.pad = 0;
      pk.put(&b.sc.w, P(k.sc_conv));  // [O][I][1][1] == [O][1][1][I]
      bn(k.sc_bn, &b.sc.post_scale, &b.sc.post_shift);
      if (s.stride == 2 && s.depth % 32 == 0 && s.cin % 32 == 0) {
        // fused conv2 + shortcut: y = sum (w2 * s2) r + sum (wsc * s_sc) x + (b2 + b_sc)
        const auto& wsc = P(k.sc_conv);
        const int K2 = 9 * s.depth, Kf = K2 + s.cin;
        std::vector<float> wf((size_t)s.depth * Kf), one(s.depth, 1.f), shf(s.depth);
        for (int o = 0; o < s.depth; ++o) {
          for (int q = 0; q < K2; ++q) wf[(size_t)o * Kf + q] = w2[(size_t)o * K2 + q] * sc2[o];
          for (int c = 0; c < s.cin; ++c) wf[(size_t)o * Kf + K2 + c] = wsc[(size_t)o * s.cin + c] * sc[o];
          shf[o] = sh2[o] + sh[o];
        }
        b.conv2_sc = b.conv2;
        b.conv2_sc.cin2 = s.cin;
        pk.put(&b.conv2_sc.w, wf);
        pk.put(&b.conv2_sc.post_scale, one);
        pk.put(&b.conv2_sc.post_shift, shf);
      }
    }
  }
  // head: BN2d(512) as pre-affine; Linear(25088,512) with NCHW-flatten columns
  // (c*49 + y*7 + x) permuted to NHWC taps ((y*7 + x)*512 + c); BN1d (affine for ArcFace).
  {
    h->head.cin = 512;
    h->head.cout = 512;
    h->head.kh = h->head.kw = 7;
    h->head.stride = 1;
    h->head.pad = 0;
    const auto& w = P(af ? "fc.weight" : "output_layer.3.weight");
    std::vector<float> r((size_t)512 * 25088);
    for (int o = 0; o < 512; ++o)
      for (int c = 0; c < 512; ++c)
        for (int t = 0; t < 49; ++t) r[(size_t)o * 25088 + (size_t)t * 512 + c] = w[(size_t)o * 25088 + (size_t)c * 49 + t];
    pk.put(&h->head.w, r);
    bn(af ? "bn2" : "output_layer.0", &h->head.pre_scale, &h->head.pre_shift);
    pk.put(&h->fc_bias, P(af ? "fc.bias" : "output_layer.3.bias"));
    bn(af ? "features" : "output_layer.4", &h->bn1d_scale, &h->bn1d_shift, af);
  }

  if (h->arena) FR_HIP(h, hipFree(h->arena));
  h->arena = nullptr;
  FR_HIP(h, hipMalloc((void**)&h->arena, pk.buf.size() * sizeof(float)));
  FR_HIP(h, hipMemcpy(h->arena, pk.buf.data(), pk.buf.size() * sizeof(float), hipMemcpyHostToDevice));
  h->arena_floats = pk.buf.size();
  for (auto& f : pk.fix) *f.first = h->arena + f.second;

  // Winograd filters are built from the arena on the device for the selected algorithm only
  // (ensure_wino2 / ensure_wino4); a later fr_set_conv_algorithm builds the other set
  if (h->wino_arena) FR_HIP(h, hipFree(h->wino_arena));
  h->wino_arena = nullptr;
  drop_wino4(h);
  if (h->convs_arena) FR_HIP(h, hipFree(h->convs_arena));
  h->convs_arena = nullptr;
  for (auto& b : h->blocks) {
    b.conv1.wino = nullptr;
    b.conv2.wino = nullptr;
  }

  // workspace for max_batch crops
  const size_t mb = h->max_batch;
  if (!h->act[0]) {
    for (auto& a : h->act) FR_HIP(h, hipMalloc((void**)&a, mb * 112 * 112 * 64 * sizeof(float)));
    // shortcut output: 28x28x128 per image (AdaFace; stage 1 has no conv shortcut), 56x56x64 (ArcFace)
    FR_HIP(h, hipMalloc((void**)&h->sc_buf, mb * 56 * 56 * 64 * sizeof(float)));
    FR_HIP(h, hipMalloc((void**)&h->partial, (size_t)fr_handle::HEAD_PARTS * mb * 512 * sizeof(float)));
    FR_HIP(h, hipMalloc((void**)&h->in_stage, mb * 112 * 112 * 3));
    FR_HIP(h, hipMalloc((void**)&h->rs_stage, mb * 112 * 112 * 3));
    FR_HIP(h, hipMalloc((void**)&h->emb_stage, mb * 512 * sizeof(float)));
    FR_HIP(h, hipMalloc((void**)&h->w4part, fr_handle::W4PART_FLOATS * sizeof(float)));
  }
  if (ensure_stream_k(h->device, &h->cus, &h->sk_ws, &h->sk_ws_floats, &h->sk_cnt, &h->sk_cnt_cap) != FR_OK)
    return fail(h, FR_ERR_HIP, "stream-K workspace allocation failed");
  h->finalized = true;
  if (h->winograd) {
    const int rc = ensure_winograd(h);
    if (rc != FR_OK) {
      h->finalized = false;
      return rc;
    }
  }
  if (const int rc = ensure_convs_weights(h)) {
    h->finalized = false;
    return rc;
  }
  return FR_OK;
}

int fr_embed(fr_handle* h, const uint8_t* rgb, int n, int height, int width, float* out, int normalize,
             void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->detector) return fail(h, FR_ERR_STATE, "this handle is a detector (scrfd_10g); use fr_detect");
  if (!h->finalized) return fail(h, FR_ERR_STATE, "model not finalised (fr_finalize)");
  if (int rc = check_crop_size(h, height, width)) return rc;
  if (n < 0 || (n > 0 && (!rgb || !out))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  if (int rc = check_dev_err(h)) return rc;  // reported by earlier asynchronous work
  DeviceGuard dg(h->device);
  return embed_any(h, rgb, n, height, width, out, normalize, (hipStream_t)stream);
}

int fr_resize_crops(fr_handle* h, const uint8_t* src, int n, int height, int width, uint8_t* dst, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (int rc = check_crop_size(h, height, width)) return rc;
  if (n < 0 || (n > 0 && (!src || !dst))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  return resize_device(h, src, n, height, width, dst, (hipStream_t)stream);
}

int fr_embed_host(fr_handle* h, const uint8_t* rgb, int n, int height, int width, float* out, int normalize) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->detector) return fail(h, FR_ERR_STATE, "this handle is a detector (scrfd_10g); use fr_detect");
  if (!h->finalized) return fail(h, FR_ERR_STATE, "model not finalised (fr_finalize)");
  if (int rc = check_crop_size(h, height, width)) return rc;
  if (n < 0 || (n > 0 && (!rgb || !out))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  DeviceGuard dg(h->device);
  hipStream_t s = nullptr;
  const size_t crop = (size_t)height * width * 3;
  for (int off = 0; off < n; off += h->max_batch) {
    const int bn = std::min(h->max_batch, n - off);
    if (height == 112 && width == 112) {
      FR_HIP(h, hipMemcpyAsync(h->in_stage, rgb + (size_t)off * crop, (size_t)bn * crop, hipMemcpyHostToDevice, s));
    } else {  // raw crops to the device, then cv2.resize to 112 x 112 into the forward's input
      int rc = ensure_buf(h, &h->rs_src, &h->rs_src_cap, (size_t)bn * crop);
      if (rc) return rc;
      FR_HIP(h, hipMemcpyAsync(h->rs_src, rgb + (size_t)off * crop, (size_t)bn * crop, hipMemcpyHostToDevice, s));
      rc = resize_device(h, static_cast<const uint8_t*>(h->rs_src), bn, height, width, h->in_stage, s);
      if (rc) return rc;
    }
    int rc = forward_staged(h, bn, normalize, s);
    if (rc) return rc;
    FR_HIP(h, hipMemcpyAsync(out + (size_t)off * 512, h->emb_stage, (size_t)bn * 512 * sizeof(float),
                             hipMemcpyDeviceToHost, s));
  }
  FR_HIP(h, hipStreamSynchronize(s));
  return check_dev_err(h);
}

int fr_gallery_set(fr_handle* h, const float* E, int G, int D, int src_is_device, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (G < 0 || (G > 0 && !E)) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad gallery");
  if (G > 0 && D != 512) return fail(h, FR_ERR_INVALID_ARGUMENT, "gallery rows must be 512-d");
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  if (G == 0) {
    h->G = 0;
    return FR_OK;
  }
  void* p = h->gallery;
  int rc = ensure_buf(h, &p, &h->gallery_cap, (size_t)G * 512 * sizeof(float));
  h->gallery = (float*)p;
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(h->gallery, E, (size_t)G * 512 * sizeof(float),
                           src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  if (!src_is_device) FR_HIP(h, hipStreamSynchronize(s));
  h->G = G;
  return FR_OK;
}

// Grow the gallery allocation to hold `rows` rows, keeping the first G rows (stream-ordered).
int gallery_reserve(fr_handle* h, int rows, hipStream_t s) {
  const size_t need = (size_t)rows * 512 * sizeof(float);
  if (h->gallery_cap >= need) return FR_OK;
  const size_t want = std::max(need, std::min((size_t)h->gallery_cap * 2, need + ((size_t)256 << 20)));
  float* p = nullptr;
  FR_HIP(h, hipMalloc((void**)&p, want));
  if (h->G > 0) FR_HIP(h, hipMemcpyAsync(p, h->gallery, (size_t)h->G * 512 * sizeof(float), hipMemcpyDeviceToDevice, s));
  FR_HIP(h, hipStreamSynchronize(s));
  FR_HIP(h, hipFree(h->gallery));
  h->gallery = p;
  h->gallery_cap = want;
  return FR_OK;
}

int fr_gallery_write_rows(fr_handle* h, int row0, int n, const float* E, int src_is_device, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || row0 < 0 || row0 > h->G || (n > 0 && !E))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "rows must satisfy 0 <= row0 <= G, n >= 0");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  const int G2 = std::max(h->G, row0 + n);
  int rc = gallery_reserve(h, G2, s);
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(h->gallery + (size_t)row0 * 512, E, (size_t)n * 512 * sizeof(float),
                           src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  if (!src_is_device) FR_HIP(h, hipStreamSynchronize(s));
  h->G = G2;
  return FR_OK;
}

int fr_gallery_delete_rows(fr_handle* h, int row0, int n, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || row0 < 0 || row0 + n > h->G) return fail(h, FR_ERR_INVALID_ARGUMENT, "rows out of range");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t tail = (size_t)(h->G - row0 - n) * 512 * sizeof(float);
  if (tail > 0) {
    int rc = ensure_buf(h, &h->gallery_tmp, &h->gallery_tmp_cap, tail);
    if (rc) return rc;
    float* src = h->gallery + (size_t)(row0 + n) * 512;
    FR_HIP(h, hipMemcpyAsync(h->gallery_tmp, src, tail, hipMemcpyDeviceToDevice, s));
    FR_HIP(h, hipMemcpyAsync(h->gallery + (size_t)row0 * 512, h->gallery_tmp, tail, hipMemcpyDeviceToDevice, s));
  }
  h->G -= n;
  return FR_OK;
}

int fr_gallery_read(fr_handle* h, int row0, int n, float* out, int dst_is_device, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || row0 < 0 || row0 + n > h->G || (n > 0 && !out))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "rows out of range");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  FR_HIP(h, hipMemcpyAsync(out, h->gallery + (size_t)row0 * 512, (size_t)n * 512 * sizeof(float),
                           dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
  if (!dst_is_device) FR_HIP(h, hipStreamSynchronize(s));
  return FR_OK;
}

int fr_build_templates(fr_handle* h, const float* emb, const int32_t* offsets, int n_students, int method,
                       float min_similarity, float* templates, int32_t* kept, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n_students < 0 || (n_students > 0 && (!emb || !offsets || !templates)))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n_students or NULL buffer");
  if (method < FR_TEMPLATE_MEAN || method > FR_TEMPLATE_WEIGHTED_MEAN)
    return fail(h, FR_ERR_INVALID_ARGUMENT, "method must be FR_TEMPLATE_MEAN, _MEDIAN or _WEIGHTED_MEAN");
  if (n_students == 0) return FR_OK;
  if (offsets[0] != 0) return fail(h, FR_ERR_INVALID_ARGUMENT, "offsets[0] must be 0");
  for (int i = 0; i < n_students; ++i) {
    const int n = offsets[i + 1] - offsets[i];
    if (n < 1 || n > TEMPLATE_MAX_SAMPLES)
      return fail(h, FR_ERR_INVALID_ARGUMENT,
                  "every student needs 1.." + std::to_string(TEMPLATE_MAX_SAMPLES) + " samples (student " +
                      std::to_string(i) + " has " + std::to_string(n) + ")");
  }
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t ob = (size_t)(n_students + 1) * sizeof(int32_t);
  int rc = ensure_buf(h, &h->tpl_offsets, &h->tpl_offsets_cap, ob);
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(h->tpl_offsets, offsets, ob, hipMemcpyHostToDevice, s));
  hipError_t e = launch_templates(emb, (const int*)h->tpl_offsets, n_students, method, min_similarity, templates,
                                  kept, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("template launch: ") + hipGetErrorString(e));
  FR_HIP(h, hipStreamSynchronize(s));  // the offsets were staged from pageable host memory
  return FR_OK;
}

int fr_gallery_size(fr_handle* h, int* G) {
  if (!h || !G) return fail(h, FR_ERR_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  *G = h->G;
  return FR_OK;
}

int fr_match_topk(fr_handle* h, const float* Q, int n, int k, int32_t* idx, float* score, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || (n > 0 && (!Q || !idx || !score))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  if (int rc = check_dev_err(h)) return rc;
  DeviceGuard dg(h->device);
  return match_device(h, Q, n, k, idx, score, (hipStream_t)stream);
}

int fr_match_topk_host(fr_handle* h, const float* Q, int n, int k, int32_t* idx, float* score) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || (n > 0 && (!Q || !idx || !score))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  if (n == 0) return FR_OK;
  if (k < 1 || k > h->G) return fail(h, FR_ERR_INVALID_ARGUMENT, "k must be in [1, G]");
  DeviceGuard dg(h->device);
  hipStream_t s = nullptr;
  const size_t qb = (size_t)n * 512 * sizeof(float), rb = (size_t)n * k * 4;
  int rc = ensure_buf(h, &h->match_io, &h->match_io_cap, qb + 2 * rb);
  if (rc) return rc;
  char* base = (char*)h->match_io;
  float* dq = (float*)base;
  int32_t* di = (int32_t*)(base + qb);
  float* ds = (float*)(base + qb + rb);
  FR_HIP(h, hipMemcpyAsync(dq, Q, qb, hipMemcpyHostToDevice, s));
  rc = match_device(h, dq, n, k, di, ds, s);
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(idx, di, rb, hipMemcpyDeviceToHost, s));
  FR_HIP(h, hipMemcpyAsync(score, ds, rb, hipMemcpyDeviceToHost, s));
  FR_HIP(h, hipStreamSynchronize(s));
  return check_dev_err(h);
}

int fr_embed_match(fr_handle* h, const uint8_t* rgb, int n, int k, int32_t* idx, float* score, float* emb_out,
                   void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->detector) return fail(h, FR_ERR_STATE, "this handle is a detector (scrfd_10g); use fr_detect");
  if (!h->finalized) return fail(h, FR_ERR_STATE, "model not finalised (fr_finalize)");
  if (n < 0 || (n > 0 && (!rgb || !idx || !score))) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad n or NULL buffer");
  if (h->G <= 0) return fail(h, FR_ERR_STATE, "gallery is empty (fr_gallery_set first)");
  if (int rc = check_dev_err(h)) return rc;  // reported by earlier asynchronous work
  DeviceGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  float* emb = emb_out;
  if (!emb) {
    int rc = ensure_buf(h, &h->match_io, &h->match_io_cap, (size_t)n * 512 * sizeof(float));
    if (rc) return rc;
    emb = (float*)h->match_io;
  }
  int rc = embed_device(h, rgb, n, emb, 1, s);
  if (rc) return rc;
  return match_device(h, emb, n, k, idx, score, s);
}

int fr_align_faces(fr_handle* h, const uint8_t* frame, int height, int width, const float* landmarks, int n,
                   int out_size, uint8_t* out, double* tforms, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || height <= 0 || width <= 0 || out_size <= 0 || out_size > 1024 ||
      (n > 0 && (!frame || !landmarks || !out)))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "bad alignment arguments");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  float tmpl[10];
  reference_template(out_size, tmpl);
  std::vector<double> minv((size_t)n * 6);
  for (int f = 0; f < n; ++f) {
    double Mf[6];
    if (!fit_similarity(landmarks + (size_t)f * 10, tmpl, 5, Mf))
      // cv2.estimateAffinePartial2D returns None here and the reference's warpAffine raises
      return fail(h, FR_ERR_INVALID_ARGUMENT, "similarity fit failed for face " + std::to_string(f));
    if (tforms) memcpy(tforms + (size_t)f * 6, Mf, sizeof(Mf));
    invert_affine(Mf, &minv[(size_t)f * 6]);
  }
  hipStream_t s = (hipStream_t)stream;
  if (n <= WARP_MAPS_BY_VALUE) {  // maps in the kernel arguments: no copy, no sync
    const hipError_t e = launch_warp_affine_by_value(frame, height, width, minv.data(), n, out_size, out, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("warp launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  int rc = ensure_buf(h, &h->align_m, &h->align_m_cap, minv.size() * sizeof(double));
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(h->align_m, minv.data(), minv.size() * sizeof(double), hipMemcpyHostToDevice, s));
  hipError_t e = launch_warp_affine(frame, height, width, (const double*)h->align_m, n, out_size, out, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("warp launch: ") + hipGetErrorString(e));
  // the host copy of the maps must outlive the async H2D copy
  FR_HIP(h, hipStreamSynchronize(s));
  return FR_OK;
}

int fr_warp_affine(fr_handle* h, const uint8_t* frame, int height, int width, const double* tforms, int n,
                   int out_size, uint8_t* out, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || height <= 0 || width <= 0 || out_size <= 0 || out_size > 1024 ||
      (n > 0 && (!frame || !tforms || !out)))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "bad warp arguments");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  std::vector<double> minv((size_t)n * 6);
  for (int f = 0; f < n; ++f) invert_affine(tforms + (size_t)f * 6, &minv[(size_t)f * 6]);
  hipStream_t s = (hipStream_t)stream;
  if (n <= WARP_MAPS_BY_VALUE) {  // maps in the kernel arguments: no copy, no sync
    const hipError_t e = launch_warp_affine_by_value(frame, height, width, minv.data(), n, out_size, out, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("warp launch: ") + hipGetErrorString(e));
    return FR_OK;
  }
  int rc = ensure_buf(h, &h->align_m, &h->align_m_cap, minv.size() * sizeof(double));
  if (rc) return rc;
  FR_HIP(h, hipMemcpyAsync(h->align_m, minv.data(), minv.size() * sizeof(double), hipMemcpyHostToDevice, s));
  hipError_t e = launch_warp_affine(frame, height, width, (const double*)h->align_m, n, out_size, out, s);
  if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("warp launch: ") + hipGetErrorString(e));
  FR_HIP(h, hipStreamSynchronize(s));
  return FR_OK;
}

int fr_blur_scores(fr_handle* h, const uint8_t* crops, int n, int height, int width, int channels, double* scores,
                   void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (n < 0 || height < 1 || width < 1 || (long long)height * width >= (1ll << 31) ||
      (channels != 1 && channels != 3 && channels != 4) || (n > 0 && (!crops || !scores)))
    return fail(h, FR_ERR_INVALID_ARGUMENT, "bad blur arguments (height, width >= 1; channels 1, 3 or 4)");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  int rc = ensure_buf(h, &h->blur_out, &h->blur_out_cap, (size_t)n * sizeof(double));
  if (rc) return rc;
  const size_t img = (size_t)height * width * channels;
  const int per = 65535;  // images per launch (grid y of the multi-block form)
  const size_t ws = blur_workspace_bytes(std::min(n, per), height, width);
  if (ws && (rc = ensure_buf(h, &h->blur_ws, &h->blur_ws_cap, ws))) return rc;
  hipStream_t s = (hipStream_t)stream;
  for (int off = 0; off < n; off += per) {
    const int m = std::min(per, n - off);
    hipError_t e = launch_blur(crops + (size_t)off * img, m, height, width, channels, (double*)h->blur_out + off,
                               h->blur_ws, s);
    if (e != hipSuccess) return fail(h, FR_ERR_HIP, std::string("blur launch: ") + hipGetErrorString(e));
  }
  FR_HIP(h, hipMemcpyAsync(scores, h->blur_out, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s));
  FR_HIP(h, hipStreamSynchronize(s));
  return check_dev_err(h);
}

int fr_detect(fr_handle* h, const uint8_t* frames, int n, int height, int width, float det_thresh, int max_faces,
              float* dets, int32_t* counts, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (!h->detector) return fail(h, FR_ERR_STATE, "not a detector handle (fr_create(\"scrfd_10g\", \"scrfd\", ...))");
  if (!h->finalized) return fail(h, FR_ERR_STATE, "model not finalised (fr_finalize)");
  if (n < 0 || (n > 0 && (!frames || !counts || (max_faces > 0 && !dets))) || height < 2 || width < 2 ||
      max_faces < 0)
    return fail(h, FR_ERR_INVALID_ARGUMENT, "bad frames / sizes / output buffers");
  if (n == 0) return FR_OK;
  DeviceGuard dg(h->device);
  if (int rc = detector_run(h, frames, n, height, width, det_thresh, max_faces, dets, counts, (hipStream_t)stream))
    return rc;
  return check_dev_err(h);  // detector_run synchronised its stream
}

int fr_set_precision(fr_handle* h, int mode) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (mode != FR_PRECISION_F32 && mode != FR_PRECISION_BF16X3)
    return fail(h, FR_ERR_INVALID_ARGUMENT, "precision must be FR_PRECISION_F32 or FR_PRECISION_BF16X3");
  h->prec = mode == FR_PRECISION_BF16X3 ? PREC_BF16X3 : PREC_F32;
  DeviceGuard dg(h->device);
  clear_graphs(h);
  if (h->finalized) return ensure_winograd(h);
  return FR_OK;
}

int fr_set_conv_algorithm(fr_handle* h, int algo) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (algo != FR_CONV_DIRECT && algo != FR_CONV_WINOGRAD && algo != FR_CONV_WINOGRAD4)
    return fail(h, FR_ERR_INVALID_ARGUMENT, "algorithm must be FR_CONV_DIRECT, FR_CONV_WINOGRAD or FR_CONV_WINOGRAD4");
  h->winograd = algo != FR_CONV_DIRECT;
  h->wino_m = algo == FR_CONV_WINOGRAD ? 2 : 4;
  DeviceGuard dg(h->device);
  clear_graphs(h);
  if (h->finalized) return ensure_winograd(h);
  return FR_OK;
}

int fr_set_graph_batch(fr_handle* h, int max_n) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->detector) return fail(h, FR_ERR_STATE, "this handle is a detector (scrfd_10g)");
  if (max_n < 0 || max_n > h->max_batch) return fail(h, FR_ERR_INVALID_ARGUMENT, "max_n must be in [0, max_batch]");
  DeviceGuard dg(h->device);
  h->graph_max_n = max_n;
  clear_graphs(h);
  return FR_OK;
}

int fr_set_lanes(fr_handle* h, int min_n, int max_lanes) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (h->detector) return fail(h, FR_ERR_STATE, "this handle is a detector (scrfd_10g)");
  if (min_n < 0) return fail(h, FR_ERR_INVALID_ARGUMENT, "min_n must be >= 0 (0: one lane)");
  if (max_lanes < 1 || max_lanes > MAX_LANES) return fail(h, FR_ERR_INVALID_ARGUMENT, "max_lanes must be in [1, 4]");
  h->lane_min = min_n;
  h->lane_max = max_lanes;
  h->lanes_fallback = false;
  return FR_OK;
}

int fr_get_lanes(fr_handle* h, int* min_n, int* max_lanes, int* fell_back) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (min_n) *min_n = h->lane_min;
  if (max_lanes) *max_lanes = h->lane_max;
  if (fell_back) *fell_back = h->lanes_fallback ? 1 : 0;
  return FR_OK;
}

int fr_graph_count(fr_handle* h, int* count) {
  if (!h || !count) return fail(h, FR_ERR_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  *count = (int)h->graphs.size();
  return FR_OK;
}

int fr_profile_enable(fr_handle* h, int enable) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  h->prof = enable != 0;
  return FR_OK;
}

int fr_profile_read(fr_handle* h, double* conv_ms, double* conv_flop, int64_t* conv_launches, double* total_ms) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  double tms = 0;
  for (int k = 0; k < 3; ++k) {
    h->last_ms[k] = h->last_flop[k] = h->last_exec[k] = 0;
    h->last_n[k] = 0;
  }
  for (auto& e : h->events) {
    FR_HIP(h, hipEventSynchronize(e.b));
    float ms = 0.f;
    FR_HIP(h, hipEventElapsedTime(&ms, e.a, e.b));
    tms += ms;
    const int k = e.kind >= 0 && e.kind < 3 ? e.kind : 0;
    h->last_ms[k] += ms;
    h->last_flop[k] += e.flop;
    h->last_exec[k] += e.exec_flop;
    ++h->last_n[k];
    h->pool.push_back(e.a);
    h->pool.push_back(e.b);
  }
  h->events.clear();
  if (int rc = check_dev_err(h)) return rc;  // every profiled launch has completed
  if (conv_ms) *conv_ms = h->last_ms[1] + h->last_ms[2];
  if (conv_flop) *conv_flop = h->last_flop[1] + h->last_flop[2];
  if (conv_launches) *conv_launches = h->last_n[1] + h->last_n[2];
  if (total_ms) *total_ms = tms;
  return FR_OK;
}

int fr_profile_kernel(fr_handle* h, int kind, double* ms, double* flop, double* exec_flop, int64_t* launches) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  if (kind < 0 || kind > 2) return fail(h, FR_ERR_INVALID_ARGUMENT, "kind must be FR_PROF_OTHER/CONV_DIRECT/CONV_WINOGRAD");
  std::lock_guard<std::mutex> lk(h->mu);
  if (ms) *ms = h->last_ms[kind];
  if (flop) *flop = h->last_flop[kind];
  if (exec_flop) *exec_flop = h->last_exec[kind];
  if (launches) *launches = h->last_n[kind];
  return FR_OK;
}

const char* fr_last_error(fr_handle* h) { return h ? h->err.c_str() : g_create_error.c_str(); }

// content hash of the library's sources and flags (build.py build_id, a generated translation unit)
extern "C" const char* frhip_build_id(void);
const char* fr_version(void) {
  static const std::string v = std::string("frhip 0.1 gfx950 fp32-mfma build ") + frhip_build_id();
  return v.c_str();
}

int frt_conv2d(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout, int kh, int kw,
               int stride, int pad, const float* pre_scale, const float* pre_shift, const float* post_scale,
               const float* post_shift, const float* prelu, const float* res, int res_h, int res_w, int epi,
               int nsplit, int tile, int stream_k, int precision, void* stream) {
  static int t_cus = 0, t_cap = 0;
  static float* t_ws = nullptr;
  static long long t_wsf = 0;
  static int* t_cnt = nullptr;
  if (epi < 0 || epi > 4 || nsplit < 1 || (nsplit > 1 && epi != EPI_RAW) || (tile < 0 || tile >= TILE_COUNT) ||
      stride < 1 || kh < 1 || kw < 1 || B < 1)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d: bad arguments");
  ConvParams p{};
  p.x = x;
  p.w = w;
  p.y = y;
  p.pre_scale = pre_scale;
  p.pre_shift = pre_shift;
  p.post_scale = post_scale;
  p.post_shift = post_shift;
  p.prelu = prelu;
  p.res = res;
  p.B = B;
  p.H = H;
  p.W = W;
  p.Cin = cin;
  p.Cout = cout;
  p.KH = kh;
  p.KW = kw;
  p.stride = stride;
  p.pad = pad;
  p.Ho = (H + 2 * pad - kh) / stride + 1;
  p.Wo = (W + 2 * pad - kw) / stride + 1;
  p.res_H = res_h;
  p.res_W = res_w;
  p.M = B * p.Ho * p.Wo;
  p.steps_total = kh * kw * cin / 32;
  p.steps_per_split = (p.steps_total + nsplit - 1) / nsplit;
  p.split_stride = (long long)p.M * cout;
  if (stream_k) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (ensure_stream_k(dev, &t_cus, &t_ws, &t_wsf, &t_cnt, &t_cap) != FR_OK)
      return fail(nullptr, FR_ERR_HIP, "frt_conv2d: stream-K workspace allocation failed");
    p.sk_cus = t_cus;
    p.sk_ws = t_ws;
    p.sk_ws_floats = t_wsf;
    p.sk_cnt = t_cnt;
    p.sk_cnt_cap = t_cap;
  }
  hipError_t e = launch_conv(p, (ConvTile)tile, pre_scale != nullptr, (Epi)epi, nsplit, (hipStream_t)stream,
                             precision == 1 ? PREC_BF16X3 : PREC_F32);
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_conv2d: ") + hipGetErrorString(e));
  return FR_OK;
}

int frt_conv2d_winograd(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout,
                        const float* pre_scale, const float* pre_shift, const float* post_scale,
                        const float* post_shift, const float* prelu, const float* res, int epi, void* stream) {
  if (!wino_supported(cin, cout, 3, 3, 1, 1) || (epi != EPI_AFFINE_PRELU && epi != EPI_AFFINE_RES) ||
      (epi == EPI_AFFINE_PRELU && (!pre_scale || !pre_shift || !prelu)) || (epi == EPI_AFFINE_RES && (pre_scale || !res)) ||
      !post_scale || !post_shift || B < 1 || H < 1 || W < 1)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_winograd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  float* u = nullptr;
  if (hipMalloc((void**)&u, wino_weight_floats(cout, cin) * sizeof(float)) != hipSuccess)
    return fail(nullptr, FR_ERR_HIP, "frt_conv2d_winograd: allocation failed");
  hipError_t e = launch_wino_weights(w, u, cout, cin, s);
  if (e == hipSuccess) {
    WinoParams p{};
    p.x = x;
    p.u = u;
    p.y = y;
    p.pre_scale = pre_scale;
    p.pre_shift = pre_shift;
    p.post_scale = post_scale;
    p.post_shift = post_shift;
    p.prelu = prelu;
    p.res = res;
    p.B = B;
    p.H = H;
    p.W = W;
    p.Cin = cin;
    p.Cout = cout;
    e = launch_wino(p, pre_scale != nullptr, (Epi)epi, s);
  }
  const hipError_t se = hipStreamSynchronize(s);
  (void)hipFree(u);
  if (e == hipSuccess) e = se;
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_conv2d_winograd: ") + hipGetErrorString(e));
  return FR_OK;
}

static int g_frt_wino4_split = 1;
int frt_set_wino4_shapes(int mode) {
  if (mode < 0 || mode > 2) return FR_ERR_INVALID_ARGUMENT;
  g_wino4_shapes = mode;
  return FR_OK;
}
int frt_set_wino4_nbg(int nbg) {
  if (nbg < 0) return FR_ERR_INVALID_ARGUMENT;
  g_wino4_nbg = nbg;
  return FR_OK;
}
int frt_set_conv2sc_tile(int tile) {
  if (tile < -1 || tile >= TILE_COUNT) return FR_ERR_INVALID_ARGUMENT;
  g_conv2sc_tile = tile;
  return FR_OK;
}
int frt_set_wino4_max_split(int s) {
  g_wino4_max_split = s < 0 ? 0 : s;
  return FR_OK;
}
int frt_conv2d_s2band(const float* x, const float* w, float* y, int B, int H, int W, const float* post_scale,
                      const float* post_shift, const float* res, void* stream) {
  if (!s2c64_supported(64, 64, 3, 3, 2, 1, H, W) || B < 1)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_s2band: 64 -> 64 channels, even H, W <= 112");
  S2Params sp{};
  sp.x = x;
  sp.w = w;
  sp.post_scale = post_scale;
  sp.post_shift = post_shift;
  sp.res = res;
  sp.y = y;
  sp.B = B;
  sp.H = H;
  sp.W = W;
  const hipError_t e = launch_s2c64(sp, (hipStream_t)stream);
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_conv2d_s2band: ") + hipGetErrorString(e));
  return FR_OK;
}
int frt_set_s2_band(int on) {
  g_s2band = on != 0;
  return FR_OK;
}
int frt_set_wino4_poll_limit(int n) {
  g_wino4_poll = n < 0 ? WINO4_POLL_DEFAULT : n;
  return FR_OK;
}
int frt_conv2d_small(const float* x, const float* x2, const float* w, float* y, int B, int H, int W, int cin,
                     int cin2, int cout, int stride, const float* pre_scale, const float* pre_shift,
                     const float* post_scale, const float* post_shift, const float* prelu, const float* res, int epi,
                     void* stream) {
  if (B < 1 || H < 1 || W < 1 || (stride != 1 && stride != 2) || epi < 0 || epi > 3 || cin2 < 0 ||
      ((pre_scale != nullptr) != (epi == EPI_AFFINE_PRELU)) || (pre_scale && !pre_shift))
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_small: bad arguments");
  ConvParams p{};
  p.x = x;
  p.x2 = cin2 > 0 ? x2 : nullptr;
  p.Cin2 = cin2;
  p.w = w;
  p.y = y;
  p.pre_scale = pre_scale;
  p.pre_shift = pre_shift;
  p.post_scale = post_scale;
  p.post_shift = post_shift;
  p.prelu = prelu;
  p.res = res;
  p.B = B;
  p.H = H;
  p.W = W;
  p.Cin = cin;
  p.Cout = cout;
  p.KH = p.KW = 3;
  p.stride = stride;
  p.pad = 1;
  p.Ho = (H - 1) / stride + 1;
  p.Wo = (W - 1) / stride + 1;
  p.res_H = H;
  p.res_W = W;
  p.M = B * p.Ho * p.Wo;
  if (!w || cout % 16 || cin % 16 || cin2 % 16)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_small: bad arguments");
  // the kernel reads its filters in fragment order: a temporary copy (test entry point)
  float* wf = nullptr;
  const size_t wbytes = (size_t)cout * (9 * cin + cin2) * sizeof(float);
  hipError_t e = hipMalloc((void**)&wf, wbytes);
  if (e == hipSuccess) e = launch_convs_weights(w, wf, cout, 9 * cin + cin2, (hipStream_t)stream);
  if (e == hipSuccess) {
    p.w = wf;
    e = launch_convs(p, pre_scale != nullptr, (Epi)epi, (hipStream_t)stream);
  }
  if (wf) {
    const hipError_t e2 = hipStreamSynchronize((hipStream_t)stream);
    (void)hipFree(wf);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_conv2d_small: ") + hipGetErrorString(e));
  return FR_OK;
}
int frt_set_small_conv(fr_handle* h, int max_n) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->convs_max_n = std::max(0, max_n);
  clear_graphs(h);
  return FR_OK;
}
int frt_set_small_conv_pre_epilogue(fr_handle* h, int on) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->convs_pre_epilogue = on != 0;
  clear_graphs(h);
  return FR_OK;
}
int frt_set_small_conv_pixels(fr_handle* h, int max_m1) {
  if (!h || max_m1 < 0) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad handle or pixel limit");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->convs_max_m1 = max_m1;
  clear_graphs(h);
  return FR_OK;
}
int frt_set_wino4_blocked(fr_handle* h, int on) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->w4_blocked = on != 0;
  clear_graphs(h);
  return FR_OK;
}
int frt_set_small_conv_blocked(fr_handle* h, int on) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->convs_blocked = on != 0;
  clear_graphs(h);
  return FR_OK;
}
int frt_set_fuse_shortcut(fr_handle* h, int on) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  DeviceGuard dg(h->device);
  h->fuse_shortcut = on != 0;
  clear_graphs(h);
  return FR_OK;
}
int frt_set_wino4_split(int on) {
  g_frt_wino4_split = on != 0;
  return FR_OK;
}

int frt_conv2d_winograd4(const float* x, const float* w, float* y, int B, int H, int W, int cin, int cout,
                        const float* pre_scale, const float* pre_shift, const float* post_scale,
                        const float* post_shift, const float* prelu, const float* res, int epi, void* stream) {
  // epilogues: the IR body's (1 with pre-BN, 2) and the detector's (0, 1 without pre-BN, 5)
  const bool res_epi = epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_PRELU;
  const bool prelu_epi = epi == EPI_AFFINE_PRELU || epi == EPI_AFFINE_RES_PRELU;
  if (!wino4_supported(cin, cout, 3, 3, 1, 1) ||
      (epi != EPI_AFFINE && epi != EPI_AFFINE_PRELU && epi != EPI_AFFINE_RES && epi != EPI_AFFINE_RES_PRELU) ||
      (pre_scale && (epi != EPI_AFFINE_PRELU || !pre_shift)) || (prelu_epi && !prelu) || (res_epi != (res != nullptr)) ||
      !post_scale || !post_shift || B < 1 || H < 1 || W < 1)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_winograd4: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  ConvW cw;
  cw.cin = cin;
  cw.pre_scale = const_cast<float*>(pre_scale);
  cw.pre_shift = const_cast<float*>(pre_shift);
  std::vector<float> t;
  if (hipStreamSynchronize(s) != hipSuccess || !wino4_pre_fold(&cw, t))
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_conv2d_winograd4: pre-BN scale has a zero");
  float *u = nullptr, *part = nullptr, *pre_t = nullptr;
  if (hipMalloc((void**)&u, (wino4_weight_floats(cout, cin) + cin) * sizeof(float)) != hipSuccess)
    return fail(nullptr, FR_ERR_HIP, "frt_conv2d_winograd4: allocation failed");
  pre_t = u + wino4_weight_floats(cout, cin);
  hipError_t e = hipMemcpy(pre_t, t.data(), cin * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_wino4_weights(w, pre_scale, u, cout, cin, s);
  static int* frt_err = nullptr;  // this entry point's device error word (no handle to own one)
  if (e == hipSuccess && !frt_err) e = hipHostMalloc((void**)&frt_err, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) *(volatile int*)frt_err = 0;
  if (e == hipSuccess) {
    Wino4Params p{};
    p.x = x;
    p.u = u;
    p.y = y;
    p.pre_t = pre_scale ? pre_t : nullptr;
    p.post_scale = post_scale;
    p.post_shift = post_shift;
    p.prelu = prelu;
    p.res = res;
    p.B = B;
    p.H = H;
    p.W = W;
    p.Cin = cin;
    p.Cout = cout;
    p.no_split = !g_frt_wino4_split;
    p.poll_max = g_wino4_poll > 0 ? g_wino4_poll : -1;
    p.err = frt_err;
    p.shapes = g_wino4_shapes;
    if (g_frt_wino4_split) {  // split-K partial slots (64 KiB each)
      p.part_floats = 257ll * 2 * 16 * 16 * 64;
      if (hipMalloc((void**)&part, p.part_floats * sizeof(float)) != hipSuccess) e = hipErrorOutOfMemory;
      p.part = part;
    }
    if (e == hipSuccess) e = launch_wino4(p, pre_scale != nullptr, (Epi)epi, s);
  }
  const hipError_t se = hipStreamSynchronize(s);
  (void)hipFree(u);
  (void)hipFree(part);
  if (e == hipSuccess) e = se;
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_conv2d_winograd4: ") + hipGetErrorString(e));
  if (*(volatile int*)frt_err & FR_DEVERR_W4_HANDOFF)
    return fail(nullptr, FR_ERR_HIP, "frt_conv2d_winograd4: F(4x4) ring hand-off timed out in wino4_kernel");
  return FR_OK;
}

int frt_stem(const uint8_t* img, int B, const float* lut, const float* w27x64, const float* bn_scale,
             const float* bn_shift, const float* prelu, float* y, void* stream) {
  hipError_t e = launch_stem(img, B, lut, w27x64, bn_scale, bn_shift, prelu, y, (hipStream_t)stream);
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_stem: ") + hipGetErrorString(e));
  return FR_OK;
}

int frt_fit_similarity(const float* src, const float* dst, int n, double* M) {
  if (n < 2 || n > 8) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "n in [2, 8]");
  return fit_similarity(src, dst, n, M) ? FR_OK : fail(nullptr, FR_ERR_INVALID_ARGUMENT, "similarity fit failed");
}

int frt_detector_forward(fr_handle* h, const uint8_t* frames, int n, int height, int width, float* heads,
                         uint8_t* canvas, void* stream) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (!h->detector || !h->finalized) return fail(h, FR_ERR_STATE, "not a finalised detector handle");
  if (n < 1 || !frames || !heads || height < 2 || width < 2) return fail(h, FR_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard dg(h->device);
  return detector_forward(h, frames, n, height, width, heads, canvas, (hipStream_t)stream);
}

int frt_set_detector_row_reduction(fr_handle* h, int on) {
  if (!h) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "NULL handle");
  std::lock_guard<std::mutex> lk(h->mu);
  if (!h->detector || !h->det) return fail(h, FR_ERR_STATE, "not a finalised detector handle");
  detector_set_row_reduction(h->det, on != 0);
  return FR_OK;
}

int frt_maxpool3(const float* x, int B, int H, int W, int C, float* y, void* stream) {
  if (B < 1 || H < 1 || W < 1 || C < 4 || !x || !y)
    return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_maxpool3: bad arguments");
  const hipError_t e = launch_maxpool3(x, B, H, W, C, y, (hipStream_t)stream);
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_maxpool3: ") + hipGetErrorString(e));
  return FR_OK;
}

int frt_topk(const float* scores, int n, int G, int k, int32_t* idx, float* val, void* stream) {
  if (k < 1 || k > G) return fail(nullptr, FR_ERR_INVALID_ARGUMENT, "frt_topk: k must be in [1, G]");
  hipError_t e = launch_topk(scores, n, G, k, idx, val, (hipStream_t)stream);
  if (e != hipSuccess) return fail(nullptr, FR_ERR_HIP, std::string("frt_topk: ") + hipGetErrorString(e));
  return FR_OK;
}

}  // extern "C"
