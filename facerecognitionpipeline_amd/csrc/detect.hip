// SCRFD face detector glue kernels on gfx950 (FaceDetector.detect, face_recognition.py:31-48;
// insightface SCRFD.detect / forward / nms restated in oracle/scrfd.py).  The conv
// pyramid itself runs on the implicit-GEMM MFMA kernel (detector.cpp); these are the
// HBM-bound pieces around it:
//
//   letterbox_kernel   cv2.resize(INTER_LINEAR) of each frame into the top-left of a
//                      zero det_w x det_h canvas, in OpenCV's fixed point (11-bit
//                      coefficients from the host; SSE2 vertical rounding for the
//                      vectorised part of each row, scalar rounding for its tail)
//   det_stem_kernel    blobFromImage ((x - 127.5) / 128, RGB) fused into conv3x3 s2
//                      3->C + BN + ReLU; det_stem_mfma_kernel the same on MFMA (K = 27 -> 28)
//   maxpool3_kernel    MaxPool2d(3, 2, 1), NHWC
//   upsample_add       FPN top-down: big += nearest-2x(small), NHWC
//   decode_kernel      sigmoid(score) >= thresh -> distance2bbox / distance2kps at the
//                      anchor centres, / det_scale, appended to a per-frame list
//   nms_kernel         sort by (score desc, anchor asc), greedy IoU NMS (numpy f32
//                      arithmetic of SCRFD.nms), one workgroup per frame
#include "frhip_kernels.h"

#pragma clang fp contract(off)

namespace frhip {

// One thread per 4 consecutive canvas bytes of a row (one 32-bit store; a row is dw * 3 bytes,
// a multiple of 4 for the detector's 640-wide canvas -- launch_letterbox checks), 32-bit index
// arithmetic.  (One thread per byte with 64-bit div / mod took 114 us per 32-frame batch.)
__global__ __launch_bounds__(256) void letterbox_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                        const int* __restrict__ xtab, const int* __restrict__ ytab,
                                                        int new_w, int new_h, int simd_end, int dw, int dh,
                                                        uint8_t* __restrict__ out) {
  const int f = blockIdx.y;
  const int e4 = blockIdx.x * 256 + threadIdx.x;  // 4-byte group of the canvas
  const int row = dw * 3, row4 = row / 4;
  if (e4 >= dh * row4) return;
  const int y = e4 / row4;
  const int ex0 = (e4 - y * row4) * 4;
  const uint8_t* src = frames + (long long)f * H * W * 3;
  unsigned packed = 0;
  if (y < new_h) {
    const int ys0 = ytab[4 * y], ys1 = ytab[4 * y + 1], b0 = ytab[4 * y + 2], b1 = ytab[4 * y + 3];
    const uint8_t* r0 = src + (long long)ys0 * W * 3;
    const uint8_t* r1 = src + (long long)ys1 * W * 3;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ex = ex0 + q;
      const int x = ex / 3, c = ex - x * 3;
      unsigned v = 0;
      if (x < new_w) {
        const int xs0 = xtab[4 * x], xs1 = xtab[4 * x + 1], a0 = xtab[4 * x + 2], a1 = xtab[4 * x + 3];
        const int S0 = r0[xs0 * 3 + c] * a0 + r0[xs1 * 3 + c] * a1;
        const int S1 = r1[xs0 * 3 + c] * a0 + r1[xs1 * 3 + c] * a1;
        int r;
        if (ex < simd_end)
          r = ((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2;
        else
          r = (int)(((long long)S0 * b0 + (long long)S1 * b1 + (1 << 21)) >> 22);
        v = (unsigned)min(max(r, 0), 255);
      }
      packed |= v << (8 * q);
    }
  }
  reinterpret_cast<unsigned*>(out + (long long)f * dh * row)[e4] = packed;
}

// One block per (frame, output row); thread t: channel group t & 3 (8 channels), pixels (t >> 2) + 64 j.
__global__ __launch_bounds__(256) void det_stem_kernel(const uint8_t* __restrict__ img, int H, int W, int C,
                                                       const float* __restrict__ w27xC,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_w = smem;              // [27][C]
  float* s_in = smem + 27 * C;    // [3][W + 2][3]
  const int Ho = H / 2, Wo = W / 2;
  const int f = blockIdx.x / Ho;
  const int oy = blockIdx.x - f * Ho;
  const int tid = threadIdx.x;
  for (int i = tid; i < 27 * C; i += 256) s_w[i] = w27xC[i];
  const uint8_t* src = img + (long long)f * H * W * 3;
  for (int i = tid; i < 3 * (W + 2) * 3; i += 256) {
    const int r = i / ((W + 2) * 3);
    const int rem = i - r * (W + 2) * 3;
    const int xx = rem / 3, c = rem - xx * 3;
    const int iy = 2 * oy - 1 + r, ix = xx - 1;
    float v = 0.f;
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      v = ((float)src[((long long)iy * W + ix) * 3 + c] - 127.5f) * 0.0078125f;
    s_in[i] = v;
  }
  __syncthreads();
  const int cg = (tid & 3) * 8;
  if (cg >= C) return;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scale[cg + k];
    sh[k] = shift[cg + k];
  }
  for (int ox = tid >> 2; ox < Wo; ox += 64) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const float v = s_in[(ky * (W + 2) + 2 * ox + kx) * 3 + ci];
          // the tap's 8 weights as two 16-byte LDS reads (8 single-float reads made the kernel
          // LDS-issue bound: 320 us per 32-frame batch)
          const float4* wr = reinterpret_cast<const float4*>(s_w + ((ky * 3 + kx) * 3 + ci) * C + cg);
          const float4 w0 = wr[0], w1 = wr[1];
          const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] = __builtin_fmaf(v, wk[k], acc[k]);
        }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaxf(__builtin_fmaf(acc[k], sc[k], sh[k]), 0.f);
    float4* dst = reinterpret_cast<float4*>(y + (((long long)f * Ho + oy) * Wo + ox) * C + cg);
    dst[0] = make_float4(o[0], o[1], o[2], o[3]);
    dst[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// MaxPool2d(3, 2, 1) in NHWC, one thread per (output pixel, 4 channels): float4 loads of the 9
// taps, 32-bit index arithmetic.  (One thread per element with 64-bit div / mod took 519 us for
// a 32-frame 320x320x32 map, a fifth of the HBM rate.)  fmaxf per element as before: bit-exact.
// One thread per (4 channels, output column, strip of MP_R output rows): the strip's 2 MP_R + 1
// input rows are loaded once -- a row shared by two output rows is not loaded twice -- and each
// row's 3-column max is taken once.  (One thread per output pixel re-read the shared rows from
// other XCDs' workgroups: 1.43x the algorithmic bytes from HBM, 155 us for the 32-frame stem.)
// max is exact, so the result is the window max whatever the order.
constexpr int MP_R = 4;
__device__ __forceinline__ float4 max4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}
__global__ __launch_bounds__(256) void maxpool3_kernel(const float4* __restrict__ x, int B, int H, int W, int C4,
                                                       float4* __restrict__ y) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1, S = (Ho + MP_R - 1) / MP_R;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * S * Wo * C4) return;
  const int c = i % C4;
  const int pix = i / C4;
  const int ox = pix % Wo, t = pix / Wo;
  const int sy = t % S, b = t / S;
  const int oy0 = sy * MP_R;
  const float4* xb = x + b * H * W * C4 + c;
  float4 rm[2 * MP_R + 1];  // 3-column max of input rows 2 oy0 - 1 + r
#pragma unroll
  for (int r = 0; r < 2 * MP_R + 1; ++r) {
    const int iy = 2 * oy0 - 1 + r;
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if ((unsigned)iy < (unsigned)H)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = 2 * ox + dx;
        if ((unsigned)ix < (unsigned)W) m = max4(m, xb[(iy * W + ix) * C4]);
      }
    rm[r] = m;
  }
#pragma unroll
  for (int j = 0; j < MP_R; ++j)
    if (oy0 + j < Ho) y[((b * Ho + oy0 + j) * Wo + ox) * C4 + c] = max4(max4(rm[2 * j], rm[2 * j + 1]), rm[2 * j + 2]);
}

// FPN top-down: big += nearest-2x(small), NHWC, one thread per (pixel, 4 channels), 32-bit indices
__global__ __launch_bounds__(256) void upsample_add_kernel(float4* __restrict__ big, const float4* __restrict__ small,
                                                           int B, int h, int w, int C4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * 4 * h * w * C4) return;
  const int c = i % C4;
  const int pix = i / C4;
  const int x = pix % (2 * w), t = pix / (2 * w);
  const int yy = t % (2 * h), b = t / (2 * h);
  const float4 s = small[((b * h + yy / 2) * w + x / 2) * C4 + c];
  float4 v = big[i];
  v.x = v.x + s.x;
  v.y = v.y + s.y;
  v.z = v.z + s.z;
  v.w = v.w + s.w;
  big[i] = v;
}

// AvgPool2d(2, 2) in NHWC (SCRFD's downsample shortcut, before its 1x1 conv): ((a + b) + c) + d
// over the window in row-major order, times 1/4 (exact), one thread per (output pixel, 4 channels).
__global__ __launch_bounds__(256) void avgpool2_kernel(const float4* __restrict__ x, int B, int H, int W, int C4,
                                                       float4* __restrict__ y) {
  const int Ho = H / 2, Wo = W / 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * Ho * Wo * C4) return;
  const int c = i % C4;
  const int pix = i / C4;
  const int ox = pix % Wo, t = pix / Wo;
  const int oy = t % Ho, b = t / Ho;
  const int r0 = (b * H + 2 * oy) * W + 2 * ox;
  const float4 p = x[r0 * C4 + c], q = x[(r0 + 1) * C4 + c], u = x[(r0 + W) * C4 + c], v = x[(r0 + W + 1) * C4 + c];
  y[i] = make_float4((((p.x + q.x) + u.x) + v.x) * 0.25f, (((p.y + q.y) + u.y) + v.y) * 0.25f,
                     (((p.z + q.z) + u.z) + v.z) * 0.25f, (((p.w + q.w) + u.w) + v.w) * 0.25f);
}

// Row expansion of a reduced-height map (detector.cpp, row_plan): dst row r of each image is src
// row r above m, src row m for the Hd - Hs rows from m on (copies of a row inside the invariant
// run), src row r - (Hd - Hs) below them.  NHWC, one thread per (pixel, 4 channels).
__global__ __launch_bounds__(256) void row_expand_kernel(const float4* __restrict__ x, int B, int Hs, int W, int C4,
                                                         int m, int Hd, float4* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * Hd * W * C4) return;
  const int c = i % C4;
  const int pix = i / C4;
  const int col = pix % W, t = pix / W;
  const int r = t % Hd, b = t / Hd;
  const int ins = Hd - Hs;
  const int sr = r < m ? r : (r < m + ins ? m : r - ins);
  y[i] = x[((b * Hs + sr) * W + col) * C4 + c];
}

// Head outputs per level: [B][H*W][32] f32 = [cls a0, cls a1, bbox a0 (4), bbox a1 (4),
// kps a0 (10), kps a1 (10), pad 2] logits / distances in stride units.
__global__ __launch_bounds__(256) void decode_kernel(DetDecodeParams p) {
  const int f = blockIdx.y;
  int loc = blockIdx.x * 256 + threadIdx.x;
  int lv = 0;
  while (lv < 3 && loc >= p.hw[lv]) {
    loc -= p.hw[lv];
    ++lv;
  }
  if (lv >= 3) return;
  const int Wl = p.w[lv];
  const float stride = (float)p.stride[lv];
  const float* h = p.head[lv] + ((long long)f * p.hw[lv] + loc) * 32;
  const int gy = loc / Wl, gx = loc - gy * Wl;
  const float cx = (float)gx * stride, cy = (float)gy * stride;
  const float ds = p.det_scale;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float score = 1.0f / (1.0f + expf(-h[a]));
    if (!(score >= p.thresh)) continue;
    const int slot = atomicAdd(p.count + f, 1);
    if (slot >= p.cap) continue;
    float* o = p.cand + ((long long)f * p.cap + slot) * 16;
    o[0] = score;
    o[1] = __int_as_float(p.anchor_base[lv] + loc * 2 + a);
    const float* bp = h + 2 + 4 * a;
    o[2] = (cx - bp[0] * stride) / ds;
    o[3] = (cy - bp[1] * stride) / ds;
    o[4] = (cx + bp[2] * stride) / ds;
    o[5] = (cy + bp[3] * stride) / ds;
    const float* kp = h + 10 + 10 * a;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      o[6 + 2 * k] = (cx + kp[2 * k] * stride) / ds;
      o[7 + 2 * k] = (cy + kp[2 * k + 1] * stride) / ds;
    }
  }
}

// One workgroup (1024 threads) per frame.  Key = (~score_bits << 32) | (anchor << 12 | slot):
// ascending order = score descending, then anchor ascending (scores are positive, so their
// bits order like the values); the slot (arrival order of decode_kernel) rides along.
__global__ __launch_bounds__(1024) void nms_kernel(const float* __restrict__ cand, const int* __restrict__ count,
                                                   int cap, float iou_thresh, int max_out,
                                                   float* __restrict__ out, int* __restrict__ out_count) {
  __shared__ unsigned long long keys[DET_MAX_CANDIDATES];
  __shared__ unsigned char removed[DET_MAX_CANDIDATES];
  __shared__ int s_nkeep;
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const int n = min(count[f], cap);
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  const float* C = cand + (long long)f * cap * 16;
  for (int i = tid; i < np2; i += 1024) {
    if (i < n) {
      const unsigned sb = __float_as_uint(C[i * 16]);
      const unsigned anchor = (unsigned)__float_as_int(C[i * 16 + 1]);
      keys[i] = ((unsigned long long)(~sb) << 32) | (anchor << 12) | (unsigned)i;
    } else {
      keys[i] = ~0ull;
    }
    removed[i] = 0;
  }
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = keys[i], b = keys[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            keys[i] = b;
            keys[l] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = 0; i < n; ++i) {
    if (removed[i]) continue;  // uniform: removed[] is stable between barriers
    const float* bi = C + (keys[i] & 0xfffu) * 16;
    const float x1 = bi[2], y1 = bi[3], x2 = bi[4], y2 = bi[5];
    const float area_i = (x2 - x1 + 1.f) * (y2 - y1 + 1.f);
    if (tid == 0) {
      const int k = s_nkeep;
      if (k < max_out) {
        float* o = out + ((long long)f * max_out + k) * 15;
        o[0] = x1;
        o[1] = y1;
        o[2] = x2;
        o[3] = y2;
        o[4] = bi[0];
        for (int q = 0; q < 10; ++q) o[5 + q] = bi[6 + q];
      }
      s_nkeep = k + 1;
    }
    for (int j = i + 1 + tid; j < n; j += 1024) {
      if (removed[j]) continue;
      const float* bj = C + (keys[j] & 0xfffu) * 16;
      const float area_j = (bj[4] - bj[2] + 1.f) * (bj[5] - bj[3] + 1.f);
      const float xx1 = fmaxf(x1, bj[2]), yy1 = fmaxf(y1, bj[3]);
      const float xx2 = fminf(x2, bj[4]), yy2 = fminf(y2, bj[5]);
      const float w = fmaxf(0.f, xx2 - xx1 + 1.f), h = fmaxf(0.f, yy2 - yy1 + 1.f);
      const float inter = w * h;
      const float ovr = inter / (area_i + area_j - inter);
      if (!(ovr <= iou_thresh)) removed[j] = 1;
    }
    __syncthreads();
  }
  if (tid == 0) out_count[f] = s_nkeep;
}

hipError_t launch_letterbox(const uint8_t* frames, int n, int H, int W, const int* xtab, const int* ytab, int new_w,
                            int new_h, int simd_end, int dw, int dh, uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const long long elems = (long long)dh * dw * 3;
  if ((dw * 3) % 4 || elems >= (1ll << 31) || (reinterpret_cast<uintptr_t>(out) & 3)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(letterbox_kernel, dim3((unsigned)((elems / 4 + 255) / 256), n), dim3(256), 0, s, frames, H, W,
                     xtab, ytab, new_w, new_h, simd_end, dw, dh, out);
  return hipGetLastError();
}

// The same stem on v_mfma_f32_16x16x4_f32 (as the embedding stem_kernel): K = 27 taps padded to
// 28, the weights the A operand (16 channels x 4 taps per fragment, CB x 7 registers per lane),
// 16 output pixels the B operand read from the normalised input rows staged in LDS; an f32 MFMA
// chains its 4 products as fmaf, so with K in (ky, kx, ci) order every output is bitwise the
// scalar kernel's.  One block per (frame, 2 output rows): 5 input rows loaded as whole-row dwords
// and unpacked through a 256-entry table of (x - 127.5) / 128.
typedef float dst_f4 __attribute__((ext_vector_type(4)));
template <int CB>
__global__ __launch_bounds__(256) void det_stem_mfma_kernel(const uint8_t* __restrict__ img, int H, int W,
                                                            const float* __restrict__ w27xC,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, float* __restrict__ y) {
  constexpr int C = 16 * CB, R = 2, NROW = 2 * R + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_lut = smem;
  float* s_in = smem + 256;  // [NROW][W + 2][3] + one zero cell
  const int SW = W + 2, NIN = NROW * SW * 3;
  const int Ho = H / 2, Wo = W / 2, RB = Ho / R;
  const int f = blockIdx.x / RB, oy0 = (blockIdx.x - f * RB) * R;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  s_lut[tid] = ((float)tid - 127.5f) * 0.0078125f;
  const int m = lane & 15, kk = lane >> 4;
  float wa[CB][7];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = 4 * st + kk;
      wa[cb][st] = k < 27 ? w27xC[k * C + 16 * cb + m] : 0.f;
    }
  const int RDW = W * 3 / 4;  // dwords per input row
  const unsigned* src = reinterpret_cast<const unsigned*>(img + (size_t)f * H * W * 3);
  for (int i = tid; i < NROW * 2 * 3 + 1; i += 256) {  // halo columns and the zero cell
    const int r = i / 6, e = i - r * 6;
    s_in[i < NROW * 6 ? (r * SW + (e < 3 ? 0 : SW - 1)) * 3 + e % 3 : NIN] = 0.f;
  }
  __syncthreads();  // s_lut
  for (int i = tid; i < NROW * RDW; i += 256) {
    const int r = i / RDW, q = 4 * (i - r * RDW);
    const int iy = 2 * oy0 - 1 + r;
    const bool in = (unsigned)iy < (unsigned)H;
    const unsigned raw = in ? src[iy * RDW + (i - r * RDW)] : 0u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int xb = q + e, ix = xb / 3;
      s_in[(r * SW + ix + 1) * 3 + (xb - ix * 3)] = in ? s_lut[(raw >> (8 * e)) & 255u] : 0.f;
    }
  }
  __syncthreads();
  int koff[7];
#pragma unroll
  for (int st = 0; st < 7; ++st) {
    const int k = 4 * st + kk;
    const int ky = k / 9, kx = (k / 3) % 3, c = k % 3;
    koff[st] = k < 27 ? (ky * SW + kx) * 3 + c : -1;
  }
  const int rg = lane >> 4;
  dst_f4 sc[CB], sh[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    sc[cb] = *reinterpret_cast<const dst_f4*>(scale + 16 * cb + 4 * rg);
    sh[cb] = *reinterpret_cast<const dst_f4*>(shift + 16 * cb + 4 * rg);
  }
  const int GPR = Wo / 16;  // 16-pixel groups per output row
  for (int grp = wv; grp < R * GPR; grp += 4) {
    const int r = grp / GPR, ox = (grp - r * GPR) * 16 + m;
    const int base = (2 * r * SW + 2 * ox) * 3;
    float bv[7];
#pragma unroll
    for (int st = 0; st < 7; ++st) bv[st] = s_in[koff[st] < 0 ? NIN : base + koff[st]];
    float* out = y + (((size_t)f * Ho + oy0 + r) * Wo + ox) * C;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      dst_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 7; ++st) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[cb][st], bv[st], acc, 0, 0, 0);
      // lane (pixel m, row group rg) holds channels 16 cb + 4 rg .. + 3 of its pixel
      dst_f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaxf(__builtin_fmaf(acc[e], sc[cb][e], sh[cb][e]), 0.f);
      *reinterpret_cast<dst_f4*>(out + 16 * cb + 4 * rg) = o;
    }
  }
}

hipError_t launch_det_stem(const uint8_t* img, int n, int H, int W, int C, const float* w27xC, const float* scale,
                           const float* shift, float* y, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (C % 8 != 0 || C > 32 || H % 2 || W % 2) return hipErrorInvalidValue;
  if ((C == 16 || C == 32) && W % 32 == 0 && (H / 2) % 2 == 0) {
    const size_t lds = (256 + 5 * (W + 2) * 3 + 1) * sizeof(float);
    if (C == 32)
      hipLaunchKernelGGL(det_stem_mfma_kernel<2>, dim3(n * (H / 4)), dim3(256), lds, s, img, H, W, w27xC, scale, shift,
                         y);
    else
      hipLaunchKernelGGL(det_stem_mfma_kernel<1>, dim3(n * (H / 4)), dim3(256), lds, s, img, H, W, w27xC, scale, shift,
                         y);
    return hipGetLastError();
  }
  const size_t lds = (27 * C + 3 * (W + 2) * 3) * sizeof(float);
  hipLaunchKernelGGL(det_stem_kernel, dim3(n * (H / 2)), dim3(256), lds, s, img, H, W, C, w27xC, scale, shift, y);
  return hipGetLastError();
}

hipError_t launch_maxpool3(const float* x, int B, int H, int W, int C, float* y, hipStream_t s) {
  const long long total = (long long)B * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1) * C;
  if (total <= 0) return hipSuccess;
  if (C % 4 || (long long)B * H * W * C >= (1ll << 31) ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15))
    return hipErrorInvalidValue;
  const long long threads = (long long)B * (((H - 1) / 2 + 1 + MP_R - 1) / MP_R) * ((W - 1) / 2 + 1) * (C / 4);
  hipLaunchKernelGGL(maxpool3_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(x), B, H, W, C / 4, reinterpret_cast<float4*>(y));
  return hipGetLastError();
}

hipError_t launch_avgpool2(const float* x, int B, int H, int W, int C, float* y, hipStream_t s) {
  if (C % 4 || H % 2 || W % 2 || (long long)B * H * W * C >= (1ll << 31)) return hipErrorInvalidValue;
  const int n = B * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(avgpool2_kernel, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<const float4*>(x), B, H,
                     W, C / 4, reinterpret_cast<float4*>(y));
  return hipGetLastError();
}

hipError_t launch_row_expand(const float* x, int B, int Hs, int W, int C, int m, int Hd, float* y, hipStream_t s) {
  if (C % 4 || Hs < 1 || Hd < Hs || m < 0 || m >= Hs || (long long)B * Hd * W * C >= (1ll << 31))
    return hipErrorInvalidValue;
  const int n = B * Hd * W * (C / 4);
  hipLaunchKernelGGL(row_expand_kernel, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<const float4*>(x), B,
                     Hs, W, C / 4, m, Hd, reinterpret_cast<float4*>(y));
  return hipGetLastError();
}

hipError_t launch_upsample_add(float* big, const float* small, int B, int h, int w, int C, hipStream_t s) {
  const long long total = (long long)B * 4 * h * w * C;
  if (total <= 0) return hipSuccess;
  if (C % 4 || total >= (1ll << 31) || ((reinterpret_cast<uintptr_t>(big) | reinterpret_cast<uintptr_t>(small)) & 15))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(upsample_add_kernel, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<float4*>(big), reinterpret_cast<const float4*>(small), B, h, w, C / 4);
  return hipGetLastError();
}

hipError_t launch_decode(const DetDecodeParams& p, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int locs = p.hw[0] + p.hw[1] + p.hw[2];
  hipLaunchKernelGGL(decode_kernel, dim3((locs + 255) / 256, n), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_nms(const float* cand, const int* count, int n, int cap, float iou_thresh, int max_out, float* out,
                      int* out_count, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (cap > DET_MAX_CANDIDATES) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nms_kernel, dim3(n), dim3(1024), 0, s, cand, count, cap, iou_thresh, max_out, out, out_count);
  return hipGetLastError();
}

}  // namespace frhip
