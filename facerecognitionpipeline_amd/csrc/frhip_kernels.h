// Internal kernel launch interface for libfrhip (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace frhip {

// Epilogue of the implicit-GEMM conv kernel.
enum Epi : int {
  EPI_AFFINE = 0,        // y = acc*scale + shift                      (shortcut conv1x1 + BN)
  EPI_AFFINE_PRELU = 1,  // y = prelu(acc*scale + shift)               (conv1 + BN + PReLU)
  EPI_AFFINE_RES = 2,    // y = acc*scale + shift + res[m]             (conv2 + BN + identity / conv shortcut)
  EPI_AFFINE_RES_SUB = 3,// y = acc*scale + shift + res[b, 2oy, 2ox]   (conv2 + BN + MaxPool2d(1,2) shortcut)
  EPI_RAW = 4,           // y[split] = acc                             (split-K partial / gallery scores)
  EPI_AFFINE_RES_PRELU = 5,  // y = prelu(acc*scale + shift + res[m])  (detector BasicBlock conv2 + BN + add + ReLU)
};

// One convolution (or GEMM, as a 1x1 conv over a 1x1 image) in NHWC f32.
//   x   [B][H][W][Cin]         w [Cout][KH][KW][Cin]        y [B][Ho][Wo][Cout]
// pre_scale/pre_shift: per-Cin affine applied to in-bounds input taps only (the
// pre-activation BatchNorm in front of a zero-padded conv), may be null.
struct ConvParams {
  const float* x;
  const float* w;
  float* y;
  const float* pre_scale;
  const float* pre_shift;
  const float* post_scale;
  const float* post_shift;
  const float* prelu;
  const float* res;
  int B, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad;
  int res_H, res_W;
  int M;                 // B*Ho*Wo
  int steps_total;       // KH*KW*Cin / 32
  int steps_per_split;   // K-steps per blockIdx.y slice
  long long split_stride;// elements between split-K partial slabs
  int mtiles, ntiles;
  // stream-K schedule (sk_cus > 0): persistent grid of sk_cus x blocks-per-CU blocks.
  int sk_cus;            // input: CUs to fill (0 = grid mode)
  int sk_blocks;         // set by the launcher: persistent grid size P
  int sk_dp_tiles;       // set by the launcher: tiles done whole, round-robin
  float* sk_ws;          // [P][2][BM*BN] partial-accumulator slabs
  long long sk_ws_floats;
  int* sk_cnt;           // per stream-K tile arrival counters, zero at allocation
  int sk_cnt_cap;
  // fused 1x1 shortcut (Cin2 > 0): K-steps [steps1, steps_total) read x2 [B][H][W][Cin2] at the
  // output's stride and no padding, 32 channels per step, against weight columns
  // KH*KW*Cin .. + Cin2 (w rows are KH*KW*Cin + Cin2 long): conv2 and the block's conv
  // shortcut as one GEMM (both BN scales folded into the weights, the shifts into post_shift)
  const float* x2;
  int Cin2, steps1;
  // serving conv kernel only (conv_small.hip): also y2 = y * y2_scale[c] + y2_shift[c] (the next
  // block's pre-activation BN, applied once here instead of per tap in its conv1); null: none
  float* y2;
  const float* y2_scale;
  const float* y2_shift;
  // serving conv kernel only: which activations are channel-blocked [B][C/16][H][W][16] instead
  // of NHWC (CONVS_BLK_* bits; y2 follows y)
  int blk;
};
constexpr int CONVS_BLK_X = 1, CONVS_BLK_X2 = 2, CONVS_BLK_RES = 4, CONVS_BLK_Y = 8;

// Tile family of a conv launch.
enum ConvTile : int {
  TILE_256x64 = 0,
  TILE_128x128 = 1,
  TILE_128x64 = 2,
  TILE_64x128 = 3,
  TILE_256x128 = 4,
  TILE_128x256 = 5,
  TILE_128x128_W8 = 6,  // 8 waves (512 threads)
  TILE_256x128_W8 = 7,
  TILE_128x64_W8 = 8,
  TILE_64x256_W8 = 9,
  TILE_256x64_W8 = 10,
  TILE_COUNT = 11
};

// Arithmetic of the conv GEMM: exact-f32 MFMA (default, the parity path) or the opt-in
// split-bf16 "bf16x3" (x = hi + lo, x.y ~= hi.hi + hi.lo + lo.hi, f32 accumulation).
enum Precision : int { PREC_F32 = 0, PREC_BF16X3 = 1 };

// y = epilogue(sum of S raw split-K slabs part[s][M][Cout], in split order) for EPI_AFFINE,
// EPI_AFFINE_RES and EPI_AFFINE_RES_SUB (conv_mfma.hip; serving-sized direct convs)
hipError_t launch_conv_split_fixup(const ConvParams& p, Epi epi, const float* part, int S, long long stride,
                                   hipStream_t s);
hipError_t launch_conv(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s,
                       Precision prec = PREC_F32);
int conv_tile_bm(ConvTile t);
int conv_tile_bn(ConvTile t);

// Winograd F(2x2,3x3) stride-1 pad-1 conv in f32 (conv_winograd.hip), NHWC like ConvParams.
//   u: transformed filters from launch_wino_weights (wino_weight_floats(Cout, Cin) floats).
// Epilogues: EPI_AFFINE_PRELU (with pre-BN) and EPI_AFFINE_RES (without).
struct WinoParams {
  const float* x;
  const float* u;
  float* y;
  const float* pre_scale;
  const float* pre_shift;
  const float* post_scale;
  const float* post_shift;
  const float* prelu;
  const float* res;  // same shape as y
  int B, H, W, Cin, Cout;
  int TH, TW, ntiles, mblocks, nblocks;  // set by launch_wino
};
bool wino_supported(int Cin, int Cout, int kh, int kw, int stride, int pad);
size_t wino_weight_floats(int Cout, int Cin);
// w: [Cout][3][3][Cin] f32 (device) -> u (device), fragment-ordered G g G^T.
hipError_t launch_wino_weights(const float* w, float* u, int Cout, int Cin, hipStream_t s);
hipError_t launch_wino(const WinoParams& p, bool pre, Epi epi, hipStream_t s);

// Winograd F(4x4,3x3) stride-1 pad-1 conv in f32 (conv_winograd4.hip), NHWC like ConvParams:
// one fused persistent kernel (transform waves -> LDS ring -> 16x16x4 MFMA waves with the
// output transform and the epilogue lane-local).  u: launch_wino4_weights output
// (wino4_weight_floats(Cout, Cin) floats).  Tiles are cut from a canvas of the batch (period
// Pr x Pc per image, NC images per canvas row, one zero separator row/column when 4 does not
// divide H/W).
struct Wino4Params {
  const float* x;
  const float* u;
  float* y;
  // pre-activation BN folded into the filters: U built from w * scale (launch_wino4_weights),
  // and t = shift / scale per input channel added to the in-image input pixels
  const float* pre_t;
  const float* post_scale;
  const float* post_shift;
  const float* prelu;
  const float* res;   // same shape as y
  int B, H, W, Cin, Cout;
  int Pr, Pc, NC, TWc, ntiles, mblocks, nblocks;  // set by launch_wino4 (wino4_canvas)
  int nbg;  // tile blocks per XCD group of items (set by launch_wino4)
  // split-K workspace (optional): compact raw partial outputs, one 16-tile x 16-pixel
  // x 64-cout slot (64 KiB) per item part; launch_wino4 splits the K loop of a small grid's items
  // when part_floats holds the slots
  float* part;
  long long part_floats;
  int ksplit, ks_per;      // set by launch_wino4
  int item0, nitem;        // set by launch_wino4: the launch's range of the layer's item order
  int no_split;  // 1: never split-K (tests compare the two schedules)
  int max_split;  // > 0: at most this many K parts per item in a split-K launch (serving sweeps)
  // ring hand-off guard: a wave that has polled its LDS counters poll_max times without seeing
  // the step it waits for stores FR_DEVERR_W4_HANDOFF into *err (a host-pinned word the
  // runtime reads at its sync points; nullable) and carries on, so a lost hand-off ends the
  // launch instead of hanging the GPU and is reported instead of passing as a result.
  // poll_max 0 means the default (WINO4_POLL_DEFAULT), < 0 no polls at all (tests).
  int* err;
  int poll_max;
  // layouts (W4_BLK_* bits): which of x, res, y are channel-blocked [B][C/16][H][W][16] instead of
  // NHWC (the same per-element arithmetic either way: outputs are bitwise the NHWC launch's)
  int blk;
  int nbg_override;  // > 0: tile blocks per XCD item group instead of the rule (A/B only)
  // item shapes of whole-item launches without pre-BN: 1 = a layer of 65..96 output channels runs
  // items of 16 tiles x 96 couts (wino4w_kernel), one of at most 32 channels items of 32 tiles x 32
  // couts (wino4t_kernel), when its 64-cout items take more than one round of workgroups; 2 = at
  // every grid size (tests); 0 = 64-cout items only
  int shapes;
};
constexpr int W4_BLK_X = 1, W4_BLK_RES = 2, W4_BLK_Y = 4;
constexpr int WINO4_POLL_DEFAULT = 1 << 16;
constexpr int FR_DEVERR_W4_HANDOFF = 1;
bool wino4_supported(int Cin, int Cout, int kh, int kw, int stride, int pad);  // Cin % 16, Cout % 16

// Serving-batch 3x3 convs (conv_small.hip): pad 1, stride 1 or 2, optional fused shortcut
// (Cin2 / x2, weight rows 9*Cin + Cin2), one workgroup per 16 pixels x 16 couts with the whole K
// reduction inside it (no split-K, no fixup).  pre: pre-BN + EPI_AFFINE_PRELU (conv1); else
// EPI_AFFINE / EPI_AFFINE_PRELU / EPI_AFFINE_RES / EPI_AFFINE_RES_SUB.  Reads p.x, w, y, pre_*,
// post_*, prelu, res, res_H/W, B, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, M, x2, Cin2, y2*.
// p.w is in fragment order (launch_convs_weights), not [Cout][9 Cin + Cin2].
bool convs_supported(const ConvParams& p, bool pre, Epi epi);
hipError_t launch_convs(const ConvParams& p, bool pre, Epi epi, hipStream_t s);
// w [Cout][KR] (KR = 9 Cin + Cin2, both % 16 == 0) -> wf, Cout * KR floats in fragment order:
// per 16-cout block cb and 16-wide K chunk kc, the 1 KiB one load instruction of a wave reads
// (lane l: couts cb * 16 + (l & 15), K kc * 16 + 4 (l >> 4) .. + 3).
hipError_t launch_convs_weights(const float* w, float* wf, int Cout, int KR, hipStream_t s);

// Stride-2 3x3 conv, 64 -> 64 channels, + BN + MaxPool2d(1,2) shortcut (conv_s2.hip): the first
// block of the AdaFace stage 1.  y[b][oy][ox] = conv(x)*scale + shift + res[b][2oy][2ox], NHWC f32;
// w [64][3][3][64]; res has x's shape.
struct S2Params {
  const float* x;
  const float* w;
  const float* post_scale;
  const float* post_shift;
  const float* res;
  float* y;
  int B, H, W;  // input
  int Ho, Wo;   // set by launch_s2c64
};
bool s2c64_supported(int Cin, int Cout, int kh, int kw, int stride, int pad, int H, int W);
hipError_t launch_s2c64(const S2Params& p, hipStream_t s);
size_t wino4_weight_floats(int Cout, int Cin);
void wino4_canvas(Wino4Params& p);
// w: [Cout][3][3][Cin] -> u = G (w * pre_scale[cin]) G^T in fragment order (pre_scale nullable)
hipError_t launch_wino4_weights(const float* w, const float* pre_scale, float* u, int Cout, int Cin, hipStream_t s);
hipError_t launch_wino4(const Wino4Params& p, bool pre, Epi epi, hipStream_t s);

// uint8 RGB HWC 112x112 -> (BGR, LUT normalise) -> conv3x3 3->64 -> BN -> PReLU, NHWC f32.
hipError_t launch_stem(const uint8_t* img, int B, const float* lut, const float* w27x64,
                       const float* bn_scale, const float* bn_shift, const float* prelu,
                       float* y, hipStream_t s);

// Sum split-K partials + FC bias -> BN1d(affine=False) -> x/||x|| -> optional e/(||e||+1e-8).
hipError_t launch_head_reduce(const float* partial, int nsplit, long long split_stride,
                              const float* fc_bias, const float* bn_scale, const float* bn_shift,
                              float* emb, int n, int normalize, int model_l2, hipStream_t s);

// q / (||q|| + 1e-8) row-wise over D=512 rows.
hipError_t launch_l2norm_rows(const float* q, float* out, int n, int d, hipStream_t s);
// serving-sized match scores (n <= 16 queries, D = 512): q / (||q|| + 1e-8) as l2norm_rows computes
// it, fused with the scores against the G x 512 gallery rows: scores [n][G]
hipError_t launch_scores_small(const float* q, const float* gallery, int G, float* scores, int n, hipStream_t s);

// Per row of a [n][G] score matrix: top-k by (score desc, index desc), k in [1, G].
hipError_t launch_topk(const float* scores, int n, int G, int k, int32_t* idx, float* val, hipStream_t s);

// warpAffine INTER_LINEAR / BORDER_CONSTANT 0 of n crops from one uint8 RGB frame;
// minv: device [n][6] inverse maps (double), out: [n][S][S][3].
hipError_t launch_warp_affine(const uint8_t* frame, int H, int W, const double* minv, int n, int S, uint8_t* out,
                              hipStream_t s);
// The same with up to WARP_MAPS_BY_VALUE host maps passed by value in the kernel arguments
// (2.3 KB of the 4 KB limit): nothing to copy, so nothing for the caller to wait on.
constexpr int WARP_MAPS_BY_VALUE = 48;
struct WarpMaps {
  double m[WARP_MAPS_BY_VALUE][6];
};
hipError_t launch_warp_affine_by_value(const uint8_t* frame, int H, int W, const double* host_minv, int n, int S,
                                       uint8_t* out, hipStream_t s);

// Laplacian variance (numpy's summation order) of the gray image of n uint8 images [n][H][W][C]
// (C = 3 / 4: RGB(A) -> gray; C = 1: gray) -> var[n] (double).  Images whose gray copy and
// summation trees fit BLUR_LDS_MAX bytes of LDS take one block each; larger ones take three
// launches over (chunk, image) blocks and blur_workspace_bytes(n, H, W) of device workspace ws.
constexpr size_t BLUR_LDS_MAX = 160 * 1024;
size_t blur_lds_bytes(int H, int W);
size_t blur_workspace_bytes(int n, int H, int W);
hipError_t launch_blur(const uint8_t* crops, int n, int H, int W, int C, double* var, void* ws, hipStream_t s);

// Gallery templates (GalleryManager._aggregate_embeddings) for n_students CSR slices of
// emb [total][512]; offsets: device [n_students + 1]; out: [n_students][512]; kept: [n] or NULL.
constexpr int TEMPLATE_MAX_SAMPLES = 1024;
enum TemplateMethod : int { TEMPLATE_MEAN = 0, TEMPLATE_MEDIAN = 1, TEMPLATE_WEIGHTED_MEAN = 2 };
hipError_t launch_templates(const float* emb, const int* offsets, int n_students, int method, float min_sim,
                            float* out, int* kept, hipStream_t s);

// ---- SCRFD detector glue (detect.hip)
constexpr int DET_MAX_CANDIDATES = 4096;  // per frame, above det_thresh, before NMS

struct DetDecodeParams {
  const float* head[3];  // per level [B][hw][32]
  int hw[3], w[3], stride[3], anchor_base[3];
  float thresh, det_scale;
  int cap;
  int* count;   // [B] candidates found (may exceed cap)
  float* cand;  // [B][cap][16]: score, anchor (int bits), x1 y1 x2 y2, 5 x (x, y)
};

// cv2.resize INTER_LINEAR (fixed point) of n frames into the top-left new_w x new_h of
// zero dw x dh canvases; xtab/ytab: device [new_w|new_h][4] = (src0, src1, w0, w1).
hipError_t launch_letterbox(const uint8_t* frames, int n, int H, int W, const int* xtab, const int* ytab, int new_w,
                            int new_h, int simd_end, int dw, int dh, uint8_t* out, hipStream_t s);
// (x - 127.5)/128 -> conv3x3 s2 p1 3->C (C % 8 == 0, <= 32; weights [27][C]) -> BN -> ReLU, NHWC.
hipError_t launch_det_stem(const uint8_t* img, int n, int H, int W, int C, const float* w27xC, const float* scale,
                           const float* shift, float* y, hipStream_t s);
hipError_t launch_maxpool3(const float* x, int B, int H, int W, int C, float* y, hipStream_t s);
hipError_t launch_upsample_add(float* big, const float* small, int B, int h, int w, int C, hipStream_t s);
// AvgPool2d(2, 2), NHWC, even H and W, C % 4 == 0.
hipError_t launch_avgpool2(const float* x, int B, int H, int W, int C, float* y, hipStream_t s);
// [B][Hs][W][C] -> [B][Hd][W][C]: rows [m, m + Hd - Hs) are copies of src row m (C % 4 == 0).
hipError_t launch_row_expand(const float* x, int B, int Hs, int W, int C, int m, int Hd, float* y, hipStream_t s);
hipError_t launch_decode(const DetDecodeParams& p, int n, hipStream_t s);
hipError_t launch_nms(const float* cand, const int* count, int n, int cap, float iou_thresh, int max_out, float* out,
                      int* out_count, hipStream_t s);

}  // namespace frhip
