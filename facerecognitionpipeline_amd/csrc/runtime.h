// Internals shared by the libfrhip runtime translation units (frhip_runtime.cpp,
// detector.cpp): the handle, folded-parameter types and the launch helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/frhip.h"
#include "frhip_kernels.h"

namespace frhip_rt {

struct BlockSpec {
  int cin, depth, stride;
};

// Device-side folded parameters of one conv.
struct ConvW {
  float* w = nullptr;  // [Cout][KH][KW][Cin]
  float* pre_scale = nullptr;
  float* pre_shift = nullptr;
  float* post_scale = nullptr;
  float* post_shift = nullptr;
  float* prelu = nullptr;
  float* wino = nullptr;  // Winograd-transformed filters (stride-1 3x3 only), or null
  float* wino4 = nullptr; // F(4x4,3x3) transformed filters G (g * pre_scale) G^T (built on demand), or null
  float* wino4_t = nullptr;  // F(4x4) folded pre-BN: pre_shift / pre_scale per input channel
  float* w_frag = nullptr;   // the serving conv kernel's copy of w in fragment order (launch_convs_weights), or null
  int cin = 0, cout = 0, kh = 0, kw = 0, stride = 1, pad = 0;
  int cin2 = 0;  // fused 1x1 shortcut input channels (w rows KH*KW*cin + cin2 long), else 0
};

struct BlockW {
  BlockSpec spec;
  ConvW conv1, conv2, sc;
  bool has_sc_conv = false;
  // conv2 and the conv shortcut as one GEMM (stride-2 blocks with a conv shortcut): both BN
  // scales folded into the weights [Cout][3][3][Cout | Cin], the two BN shifts summed
  ConvW conv2_sc;
};

// kind: 0 other launch, 1 direct implicit-GEMM conv, 2 Winograd conv (frhip.h FR_PROF_*)
struct ProfEvent {
  hipEvent_t a, b;
  double flop;       // algorithmic (direct-conv) FLOPs
  double exec_flop;  // FLOPs the MFMA pipe actually executes
  int kind;
};

// The buffers one running forward writes (a lane).  Lane 0 is the handle's own workspace; lanes
// 1 .. MAX_LANES - 1 (fr_set_lanes) are further sets, so the parts of a large batch run as
// concurrent forwards on their own streams and one part's part-empty last round of a layer fills
// with another part's work.
struct LaneWs {
  float* act[3] = {nullptr, nullptr, nullptr};
  float* sc_buf = nullptr;
  float* partial = nullptr;
  float* w4part = nullptr;
  float* sk_ws = nullptr;
  long long sk_ws_floats = 0;
  int* sk_cnt = nullptr;
  int sk_cnt_cap = 0;
};
constexpr int MAX_LANES = 4;

struct Detector;  // detector.cpp
void detector_destroy(Detector* d);
void detector_set_row_reduction(Detector* d, bool on);
// every conv of the detector (for the Winograd filter builds); no-op for d == nullptr
void detector_convs(Detector* d, std::vector<ConvW*>& out);

}  // namespace frhip_rt

struct fr_handle {
  std::mutex mu;
  std::string arch, model_type, err;
  bool arcface = false;
  bool detector = false;  // arch "scrfd_10g": a face detector, not an embedding model  // insightface IResNet keys/semantics (face_embedder.py:64-88)
  int device = 0;
  int max_batch = 256;
  bool finalized = false;
  std::vector<frhip_rt::BlockSpec> specs;
  std::map<std::string, size_t> expected;  // key -> numel
  std::map<std::string, std::vector<float>> params;

  // device arena with every folded weight
  float* arena = nullptr;
  size_t arena_floats = 0;
  float *lut = nullptr, *stem_w = nullptr, *stem_scale = nullptr, *stem_shift = nullptr, *stem_prelu = nullptr;
  std::vector<frhip_rt::BlockW> blocks;
  frhip_rt::ConvW head;  // BN2d pre-affine + FC as 7x7 valid conv
  float *fc_bias = nullptr, *bn1d_scale = nullptr, *bn1d_shift = nullptr;

  // workspace
  float *act[3] = {nullptr, nullptr, nullptr};
  float* sc_buf = nullptr;
  float* partial = nullptr;
  // head FC split-K parts: serving batches (4 n <= max_batch) / larger; partial buffers hold
  // HEAD_PARTS x max_batch rows (>= 98 n for the serving split at 4 n <= max_batch, >= 32 n for the other)
  static constexpr int HEAD_SPLIT_SMALL = 98, HEAD_SPLIT = 32, HEAD_PARTS = 49;
  uint8_t* in_stage = nullptr;
  float* emb_stage = nullptr;

  // resize branch of FaceEmbedder.preprocess (face_embedder.py:94-96): cv2.resize INTER_LINEAR
  // coefficient tables per source size ([112 x][4] then [112 y][4], device), resized crops of one
  // chunk, and host-API staging of the raw crops
  struct ResizeTab {
    int H, W, simd_end;
    int* tab;
    unsigned long long used;  // last use (LRU clock)
    hipEvent_t last;          // recorded after the table's last resize launch (on that call's stream)
  };
  static constexpr size_t RS_TABS_MAX = 16;  // coefficient tables kept per handle (LRU)
  std::vector<ResizeTab> rs_tabs;
  unsigned long long rs_clock = 0;
  uint8_t* rs_stage = nullptr;
  void* rs_src = nullptr;
  size_t rs_src_cap = 0;

  // gallery + match workspace
  float* gallery = nullptr;
  int G = 0;
  size_t gallery_cap = 0;
  float* qn = nullptr;
  size_t qn_cap = 0;
  float* scores = nullptr;
  size_t scores_cap = 0;
  void* match_io = nullptr;
  size_t match_io_cap = 0;
  void* gallery_tmp = nullptr;  // tail staging for row deletes
  size_t gallery_tmp_cap = 0;
  void* tpl_offsets = nullptr;  // CSR offsets of fr_build_templates
  size_t tpl_offsets_cap = 0;

  // alignment / quality workspace
  void* align_m = nullptr;  // [n][6] inverse affine maps (double)
  size_t align_m_cap = 0;
  void* blur_out = nullptr;  // [n] double
  size_t blur_out_cap = 0;
  void* blur_ws = nullptr;  // multi-block blur: per (image, chunk) int64 L sums + double values
  size_t blur_ws_cap = 0;

  // stream-K workspace shared by every body conv launch (launches are stream-ordered)
  int cus = 0;
  float* sk_ws = nullptr;
  long long sk_ws_floats = 0;
  int* sk_cnt = nullptr;
  int sk_cnt_cap = 0;
  bool stream_k = true;
  bool fuse_shortcut = true;  // conv2 + conv shortcut as one launch (frt_set_fuse_shortcut: A/B)
  frhip::Precision prec = frhip::PREC_F32;
  bool winograd = true;          // FR_CONV_WINOGRAD / _WINOGRAD4 for stride-1 3x3 convs
  int wino_m = 4;                // output tile of the Winograd algorithm: 4 = F(4x4,3x3) (default), 2 = F(2x2,3x3)
  float* wino_arena = nullptr;   // F(2x2) filters, built when that algorithm is selected
  float* wino4_arena = nullptr;  // F(4x4) filters, likewise
  float* convs_arena = nullptr;  // the serving conv kernel's filters (ConvW::w_frag), built at fr_finalize
  float* w4part = nullptr;         // F(4x4) split-K partial outputs (small batches), W4PART_FLOATS
  static constexpr long long W4PART_FLOATS = 16ll << 20;

  // lanes (fr_set_lanes): a forward of n crops runs as min(lane_max, n / lane_min) concurrent
  // parts, lane 0 on the caller's stream with the workspace above, lane l >= 1 on lane_stream[l]
  // with lane_ws[l]
  int lane_min = 0, lane_max = 1;
  bool lanes_fallback = false;  // lanes were turned off by a failed lane-workspace allocation
  frhip_rt::LaneWs lane_ws[frhip_rt::MAX_LANES];
  int lane_batch[frhip_rt::MAX_LANES] = {0, 0, 0, 0};  // crops lane l's buffers hold
  hipStream_t lane_stream[frhip_rt::MAX_LANES] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t lane_fork = nullptr;
  hipEvent_t lane_join[frhip_rt::MAX_LANES] = {nullptr, nullptr, nullptr, nullptr};

  // SCRFD detector (arch "scrfd_10g"): layers, workspace (detector.cpp)
  frhip_rt::Detector* det = nullptr;

  // hipGraph replay of small forwards (fr_set_graph_batch): one executable graph per
  // (n, normalize), captured on cap_stream from in_stage to emb_stage
  struct GraphEntry {
    int n, normalize;
    hipGraphExec_t exec;
  };
  int graph_max_n = 0;
  bool capturing = false;  // forwards captured into a graph run one lane
  hipStream_t cap_stream = nullptr;
  std::vector<GraphEntry> graphs;

  // forwards of n <= convs_max_n crops run every body 3x3 conv on conv_small.hip's kernel (one
  // launch per layer, whole K per 16x16 tile) instead of F(4x4) split-K + fixup / the split-K
  // direct convs (frt_set_small_conv)
  int convs_max_n = 2;
  // output-pixel limit of a batch-1 layer on that kernel (frt_set_small_conv_pixels; batch 2: 1,024)
  int convs_max_m1 = 4096;
  // a one-lane forward's conv2 on that kernel also writes the next block's pre-BN input into
  // convs_y2 (forward_lanes sets these three; run_conv sets convs_y2_done when it did), and that
  // block's conv1 then runs without pre-BN on it (frt_set_small_conv_pre_epilogue: A/B)
  float* convs_y2 = nullptr;
  const float *convs_y2_scale = nullptr, *convs_y2_shift = nullptr;
  bool convs_y2_done = false;
  bool convs_pre_epilogue = true;
  // activations passed between two serving-kernel layers of a one-lane forward are channel-blocked
  // (ConvParams::blk; forward_lanes sets convs_blk per launch); frt_set_small_conv_blocked: A/B
  int convs_blk = 0;
  bool convs_blocked = true;
  // channel-blocked activations between F(4x4) layers of larger forwards (forward_lanes sets w4_blk,
  // the Wino4Params::blk of the next launch); frt_set_wino4_blocked: A/B
  int w4_blk = 0;
  bool w4_blocked = true;

  // device-side error word (host-pinned, coherent): kernels that detect a broken invariant
  // store an FR_DEVERR_* code here (wino4_kernel: a ring hand-off that timed out); the runtime
  // reads it at its sync points and at the entry of every compute call (check_dev_err)
  int* dev_err = nullptr;

  // profiling
  bool prof = false;
  std::vector<frhip_rt::ProfEvent> events;
  std::vector<hipEvent_t> pool;
  double last_ms[3] = {0, 0, 0}, last_flop[3] = {0, 0, 0}, last_exec[3] = {0, 0, 0};
  int64_t last_n[3] = {0, 0, 0};

  ~fr_handle() {
    frhip_rt::detector_destroy(det);
    for (auto& e : events) {
      (void)hipEventDestroy(e.a);
      (void)hipEventDestroy(e.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
    for (auto& g : graphs) (void)hipGraphExecDestroy(g.exec);
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    if (lane_fork) (void)hipEventDestroy(lane_fork);
    for (int l = 1; l < frhip_rt::MAX_LANES; ++l) {
      if (lane_stream[l]) (void)hipStreamDestroy(lane_stream[l]);
      if (lane_join[l]) (void)hipEventDestroy(lane_join[l]);
      frhip_rt::LaneWs& L = lane_ws[l];
      for (auto p : L.act) (void)hipFree(p);
      (void)hipFree(L.sc_buf);
      (void)hipFree(L.partial);
      (void)hipFree(L.w4part);
      (void)hipFree(L.sk_ws);
      (void)hipFree(L.sk_cnt);
    }
    (void)hipFree(arena);
    (void)hipFree(wino_arena);
    (void)hipFree(wino4_arena);
    (void)hipFree(convs_arena);
    (void)hipFree(w4part);
    for (auto p : act) (void)hipFree(p);
    (void)hipFree(sc_buf);
    (void)hipFree(partial);
    (void)hipFree(in_stage);
    (void)hipFree(emb_stage);
    for (auto& t : rs_tabs) {
      (void)hipFree(t.tab);
      if (t.last) (void)hipEventDestroy(t.last);
    }
    (void)hipFree(rs_stage);
    (void)hipFree(rs_src);
    (void)hipFree(gallery);
    (void)hipFree(qn);
    (void)hipFree(scores);
    (void)hipFree(match_io);
    (void)hipFree(gallery_tmp);
    (void)hipFree(tpl_offsets);
    (void)hipFree(sk_ws);
    (void)hipFree(sk_cnt);
    (void)hipFree(align_m);
    (void)hipFree(blur_out);
    (void)hipFree(blur_ws);
    if (dev_err) (void)hipHostFree(dev_err);
  }
};

namespace frhip_rt {

int fail(fr_handle* h, int code, const std::string& msg);
// The handle's device error word: allocated (zeroed) on first use; FR_OK or FR_ERR_HIP.
int ensure_dev_err(fr_handle* h);
// FR_ERR_HIP (and the word cleared) if a kernel of work that has completed by now reported a
// broken invariant, else FR_OK.  Call after a stream sync to cover that call's own work.
int check_dev_err(fr_handle* h);

#define FR_HIP(h, call)                                                                          \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      return ::frhip_rt::fail(h, FR_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Host staging of every folded tensor before one upload into an arena.
struct Packer {
  std::vector<float> buf;
  std::vector<std::pair<float**, size_t>> fix;  // (destination pointer, float offset)
  void put(float** dst, const std::vector<float>& v) {
    size_t off = (buf.size() + 3) & ~size_t(3);  // 16-B alignment for float4 loads
    buf.resize(off);
    buf.insert(buf.end(), v.begin(), v.end());
    fix.push_back({dst, off});
  }
};

void add_bn(std::map<std::string, size_t>& m, const std::string& p, int c, bool affine = true);
void bn_fold(const std::vector<float>* gamma, const std::vector<float>* beta, const std::vector<float>& mean,
             const std::vector<float>& var, std::vector<float>& scale, std::vector<float>& shift);
std::vector<float> repack_oihw(const std::vector<float>& w, int O, int I, int kh, int kw);
int ensure_buf(fr_handle* h, void** p, size_t* cap, size_t bytes);
int ensure_stream_k(int device, int* cus, float** ws, long long* ws_floats, int** cnt, int* cnt_cap);
// L: the lane whose stream-K / split-K workspace the launch uses (nullptr: the handle's own)
// x2: the fused shortcut's input (cw.cin2 > 0)
int run_conv(fr_handle* h, const ConvW& cw, const float* x, float* y, int B, int H, int W, frhip::Epi epi,
             const float* res, int res_H, int res_W, int nsplit, long long split_stride, hipStream_t s,
             const LaneWs* L = nullptr, const float* x2 = nullptr);
const std::vector<float>* getp(fr_handle* h, const std::string& k);

// detector.cpp
// cv::resize INTER_LINEAR (uint8) coefficient table of one axis: (src0, src1, w0, w1) per output
void resize_axis_table(int dsize, int ssize, int* t);
// end of the SSE2-vectorised part of a resized row of row_elems bytes (the rest rounds as scalar code)
int resize_simd_end(int row_elems);
std::map<std::string, size_t> detector_schema();
int detector_finalize(fr_handle* h);
int detector_run(fr_handle* h, const uint8_t* frames, int n, int height, int width, float det_thresh, int max_faces,
                 float* dets, int32_t* counts, hipStream_t s);
int detector_forward(fr_handle* h, const uint8_t* frames, int n, int height, int width, float* heads,
                     uint8_t* canvas, hipStream_t s);

}  // namespace frhip_rt
