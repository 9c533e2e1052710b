// Implicit-GEMM NHWC convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces every Conv2d of the AdaFace IR body (net.BasicBlockIR res_layer[1],
// res_layer[4], shortcut_layer[0]) and the output Linear (as a 7x7 "valid" conv
// over the NHWC feature map), reached by the reference through
// `self.model(batch)` (face_embedder.py:157) on PyTorch CPU fp32.
//
// GEMM view:  C[m][n] = sum_k A[m][k] * Wt[n][k]
//   m = (b, oy, ox)            M = B*Ho*Wo      (output pixels, NHWC row)
//   n = output channel         N = Cout
//   k = (ky, kx, ci)           K = KH*KW*Cin    (one K-step = one tap x 32 channels)
//
// Tiles: 256 threads = 4 waves; each wave owns TM x TN 32x32 accumulators.
// LDS holds A as [BM][32+4] and B as [BN][32+4] floats (4-float pad -> the
// ds_read_b128 of 32 consecutive rows hits 16 distinct 16-B slots: conflict free).
// Lane (i = l&31, h = l>>5) reads 4 consecutive k (4h..4h+3 of an 8-k group) of
// its A row and B row with one ds_read_b128 each; MFMA s of the group uses
// element s, so the pair {h=0, h=1} of one MFMA covers k = 4h+s.
//
// Pipeline (register staging, one barrier per K-step): global loads of step
// s+1 are issued before the MFMAs of step s and written to the other LDS
// buffer after them (pre-BN affine + zero padding applied on the way).
// Numerics: exact f32 products, f32 accumulation (MFMA = fmaf chain), only the
// k summation order differs from the CPU reference.
#include "frhip_kernels.h"

namespace frhip {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDK = BK + 4;
constexpr int NTHREADS = 256;

template <int BM, int BN, int WM, int WN, bool PRE, int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void conv_mfma_kernel(ConvParams p) {
  static_assert(WM * WN == 4, "4 waves per block");
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  constexpr int A_IT = BM / 32;  // A rows staged per thread (8 float4 per row, 32 rows per pass)
  constexpr int B_IT = BN / 32;

  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LDK];
  float* As0 = lds;
  float* Bs0 = lds + BM * LDK;
  constexpr int BUF = (BM + BN) * LDK;

  // ---- block -> tile, XCD-aware (blocks b, b+8, ... share an XCD: give each XCD a
  // contiguous run of tiles so neighbouring M-tiles and one weight panel share its L2).
  const int nwg = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int mt = wg % p.mtiles;
  const int nt = wg / p.mtiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int split = blockIdx.y;
  const int s_begin = split * p.steps_per_split;
  int s_end = s_begin + p.steps_per_split;
  if (s_end > p.steps_total) s_end = p.steps_total;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int k4 = tid & 7;       // which float4 of the 32-channel K-step
  const int rsub = tid >> 3;    // 0..31

  const int H = p.H, W = p.W, Cin = p.Cin;
  const int cchunks = Cin / BK;
  const int Ktot = p.KH * p.KW * Cin;

  // ---- per-row im2col bases for the A rows this thread stages
  int a_base[A_IT], a_iy[A_IT], a_ix[A_IT];
  const int HoWo = p.Ho * p.Wo;
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    const int m = m0 + rsub + 32 * i;
    if (m < p.M) {
      const int b = m / HoWo;
      const int rem = m - b * HoWo;
      const int oy = rem / p.Wo;
      const int ox = rem - oy * p.Wo;
      a_iy[i] = oy * p.stride - p.pad;
      a_ix[i] = ox * p.stride - p.pad;
      a_base[i] = ((b * H + a_iy[i]) * W + a_ix[i]) * Cin + 4 * k4;
    } else {
      a_iy[i] = -(1 << 20);
      a_ix[i] = 0;
      a_base[i] = 0;
    }
  }
  int b_off[B_IT];
  bool b_ok[B_IT];
#pragma unroll
  for (int j = 0; j < B_IT; ++j) {
    const int n = n0 + rsub + 32 * j;
    b_ok[j] = n < p.Cout;
    b_off[j] = (b_ok[j] ? n : 0) * Ktot + 4 * k4;
  }

  float4 ra[A_IT], rb[B_IT];
  float4 psc = make_float4(1.f, 1.f, 1.f, 1.f), psh = make_float4(0.f, 0.f, 0.f, 0.f);
  bool a_ok[A_IT];

  auto load_step = [&](int s) {
    const int tap = s / cchunks;
    const int c0 = (s - tap * cchunks) * BK;
    const int ky = tap / p.KW;
    const int kx = tap - ky * p.KW;
    const int tap_off = (ky * W + kx) * Cin + c0;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
      a_ok[i] = ((unsigned)iy < (unsigned)H) && ((unsigned)ix < (unsigned)W);
      ra[i] = a_ok[i] ? *reinterpret_cast<const float4*>(p.x + a_base[i] + tap_off)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int koff = tap * Cin + c0;
#pragma unroll
    for (int j = 0; j < B_IT; ++j)
      rb[j] = b_ok[j] ? *reinterpret_cast<const float4*>(p.w + b_off[j] + koff)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (PRE) {
      psc = *reinterpret_cast<const float4*>(p.pre_scale + c0 + 4 * k4);
      psh = *reinterpret_cast<const float4*>(p.pre_shift + c0 + 4 * k4);
    }
  };

  auto store_step = [&](int buf) {
    float* As = As0 + buf * BUF;
    float* Bs = Bs0 + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      float4 v = ra[i];
      if constexpr (PRE) {
        // BN(x) only where the tap is inside the image: padded zeros stay zero.
        if (a_ok[i]) {
          v.x = v.x * psc.x + psh.x;
          v.y = v.y * psc.y + psh.y;
          v.z = v.z * psc.z + psh.z;
          v.w = v.w * psc.w + psh.w;
        }
      }
      *reinterpret_cast<float4*>(As + (rsub + 32 * i) * LDK + 4 * k4) = v;
    }
#pragma unroll
    for (int j = 0; j < B_IT; ++j)
      *reinterpret_cast<float4*>(Bs + (rsub + 32 * j) * LDK + 4 * k4) = rb[j];
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int frag_row = lane & 31;
  const int frag_k = 4 * (lane >> 5);

  if (s_begin < s_end) {
    load_step(s_begin);
    store_step(0);
    __syncthreads();
    int buf = 0;
    for (int s = s_begin; s < s_end; ++s) {
      const bool more = (s + 1) < s_end;
      if (more) load_step(s + 1);
      const float* Ab = As0 + buf * BUF + (wm * TM * 32 + frag_row) * LDK + frag_k;
      const float* Bb = Bs0 + buf * BUF + (wn * TN * 32 + frag_row) * LDK + frag_k;
#pragma unroll
      for (int g = 0; g < BK / 8; ++g) {
        float4 fa[TM], fb[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) fa[a] = *reinterpret_cast<const float4*>(Ab + a * 32 * LDK + g * 8);
#pragma unroll
        for (int b = 0; b < TN; ++b) fb[b] = *reinterpret_cast<const float4*>(Bb + b * 32 * LDK + g * 8);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].x, fb[b].x, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].y, fb[b].y, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].z, fb[b].z, acc[a][b], 0, 0, 0);
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[a].w, fb[b].w, acc[a][b], 0, 0, 0);
          }
      }
      if (more) store_step(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int HrWr = p.res_H * p.res_W;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int n = n0 + (wn * TN + b) * 32 + (lane & 31);
    if (n >= p.Cout) continue;
    float sc = 1.f, sh = 0.f, al = 0.f;
    if constexpr (EPI != EPI_RAW) {
      sc = p.post_scale[n];
      sh = p.post_shift[n];
    }
    if constexpr (EPI == EPI_AFFINE_PRELU) al = p.prelu[n];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + (wm * TM + a) * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        float v = acc[a][b][e];
        if constexpr (EPI == EPI_RAW) {
          p.y[(long long)split * p.split_stride + (long long)m * p.Cout + n] = v;
        } else {
          v = v * sc + sh;
          if constexpr (EPI == EPI_AFFINE_PRELU) v = v > 0.f ? v : v * al;
          if constexpr (EPI == EPI_AFFINE_RES) v += p.res[(long long)m * p.Cout + n];
          if constexpr (EPI == EPI_AFFINE_RES_SUB) {
            const int bb = m / HoWo;
            const int rem = m - bb * HoWo;
            const int oy = rem / p.Wo;
            const int ox = rem - oy * p.Wo;
            v += p.res[((long long)(bb * p.res_H + 2 * oy) * p.res_W + 2 * ox) * p.Cout + n];
            (void)HrWr;
          }
          p.y[(long long)m * p.Cout + n] = v;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_tile(const ConvParams& p0, bool pre, Epi epi, int nsplit, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (p.Cout + BN - 1) / BN;
  dim3 grid(p.mtiles * p.ntiles, nsplit), block(NTHREADS);
#define FR_CONV_CASE(PRE_, EPI_)                                                                    \
  if (pre == PRE_ && epi == EPI_) {                                                                 \
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, PRE_, EPI_>), grid, block, 0, s, p);      \
    return hipGetLastError();                                                                       \
  }
  FR_CONV_CASE(true, EPI_AFFINE_PRELU)
  FR_CONV_CASE(false, EPI_AFFINE_RES)
  FR_CONV_CASE(false, EPI_AFFINE_RES_SUB)
  FR_CONV_CASE(false, EPI_AFFINE)
  FR_CONV_CASE(true, EPI_RAW)
  FR_CONV_CASE(false, EPI_RAW)
#undef FR_CONV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_conv(const ConvParams& p, ConvTile tile, bool pre, Epi epi, int nsplit, hipStream_t s) {
  if (p.Cin % BK != 0 || p.steps_total != p.KH * p.KW * p.Cin / BK || nsplit < 1 ||
      (long long)p.steps_per_split * nsplit < p.steps_total || p.M <= 0 || p.Cout <= 0)
    return hipErrorInvalidValue;
  if (tile == TILE_256x64) return launch_tile<256, 64, 4, 1>(p, pre, epi, nsplit, s);
  return launch_tile<128, 128, 2, 2>(p, pre, epi, nsplit, s);
}

}  // namespace frhip
