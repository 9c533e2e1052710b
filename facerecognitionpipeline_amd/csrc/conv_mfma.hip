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
  const int taps = p.KH * p.KW;
  const int Ktot = taps * Cin;

  // Buffer descriptors: an out-of-range offset returns zeros, so padding taps,
  // rows past M and columns past N need no branches (OOB = 0x80000000).
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.B * H * W * Cin * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.Cout * Ktot * 4, 0x00020000);
  constexpr int OOB = 0x80000000;

  // ---- per-row im2col bases (bytes) for the A rows this thread stages
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
      a_base[i] = (((b * H + a_iy[i]) * W + a_ix[i]) * Cin + 4 * k4) * 4;
    } else {
      a_iy[i] = -(1 << 20);
      a_ix[i] = 0;
      a_base[i] = 0;
    }
  }
  int b_base[B_IT];
#pragma unroll
  for (int j = 0; j < B_IT; ++j) {
    const int n = n0 + rsub + 32 * j;
    b_base[j] = n < p.Cout ? (n * Ktot + 4 * k4) * 4 : OOB;
  }

  // K-step s = cc * taps + tap: channel chunk outer, tap inner, so the 9 taps of
  // one 32-channel slice are consecutive steps (the shifted im2col rows re-hit L1/L2).
  int tap = s_begin % taps;
  int cc = s_begin / taps;
  int ky = tap / p.KW;
  int kx = tap - ky * p.KW;

  float4 ra[A_IT], rb[B_IT];
  float4 psc = make_float4(1.f, 1.f, 1.f, 1.f), psh = make_float4(0.f, 0.f, 0.f, 0.f);
  unsigned a_okm = 0;

  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto ld4 = [](__amdgpu_buffer_rsrc_t rs, int off) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
  };

  auto load_step = [&](bool live) {
    const int c0 = cc * BK;
    const int tap_off = ((ky * W + kx) * Cin + c0) * 4;
    a_okm = 0;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
      const unsigned ok = (unsigned)live & (unsigned)((unsigned)iy < (unsigned)H) & (unsigned)((unsigned)ix < (unsigned)W);
      a_okm |= ok << i;
      ra[i] = ld4(xr, ok ? a_base[i] + tap_off : OOB);
    }
    const int koff = (tap * Cin + c0) * 4;
#pragma unroll
    for (int j = 0; j < B_IT; ++j) rb[j] = ld4(wr, (b_base[j] == OOB || !live) ? OOB : b_base[j] + koff);
    if constexpr (PRE) {
      psc = *reinterpret_cast<const float4*>(p.pre_scale + c0 + 4 * k4);
      psh = *reinterpret_cast<const float4*>(p.pre_shift + c0 + 4 * k4);
    }
  };
  // Step counters of s+1; frozen on the last step (its loads are OOB no-ops).
  auto advance = [&](bool live) {
    const int kx1 = kx + 1 == p.KW ? 0 : kx + 1;
    const int ky1 = kx + 1 == p.KW ? (ky + 1 == p.KH ? 0 : ky + 1) : ky;
    const int tap1 = tap + 1 == taps ? 0 : tap + 1;
    const int cc1 = tap + 1 == taps ? cc + 1 : cc;
    kx = live ? kx1 : kx;
    ky = live ? ky1 : ky;
    tap = live ? tap1 : tap;
    cc = live ? cc1 : cc;
  };

  auto store_step = [&](int buf) {
    float* As = As0 + buf * BUF;
    float* Bs = Bs0 + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      float4 v = ra[i];
      if constexpr (PRE) {
        // BN(x) only where the tap is inside the image: padded zeros stay zero.
        if (a_okm & (1u << i)) {
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
    load_step(true);
    store_step(0);
    __syncthreads();
    int buf = 0;
    // Branch-free body (one basic block) so the schedule below can interleave the next
    // step's global loads and LDS writes with this step's MFMAs.
    for (int s = s_begin; s < s_end; ++s) {
      const bool live = (s + 1) < s_end;
      advance(live);
      load_step(live);
      const float* Ab = As0 + buf * BUF + (wm * TM * 32 + frag_row) * LDK + frag_k;
      const float* Bb = Bs0 + buf * BUF + (wn * TN * 32 + frag_row) * LDK + frag_k;
      float4 fa[BK / 8][TM], fb[BK / 8][TN];
#pragma unroll
      for (int g = 0; g < BK / 8; ++g) {
#pragma unroll
        for (int a = 0; a < TM; ++a) fa[g][a] = *reinterpret_cast<const float4*>(Ab + a * 32 * LDK + g * 8);
#pragma unroll
        for (int b = 0; b < TN; ++b) fb[g][b] = *reinterpret_cast<const float4*>(Bb + b * 32 * LDK + g * 8);
      }
#pragma unroll
      for (int g = 0; g < BK / 8; ++g) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[g][a][e], fb[g][b][e], acc[a][b], 0, 0, 0);
      }
      store_step(buf ^ 1);
      // Schedule (MFMA f32 = 64 pipe cycles; other instructions issue in its shadow):
      //   fragments of groups 0-1 | 1 MFMA + 1 global load, x loads | fragments of groups 2-3 |
      //   MFMAs | 2 MFMA + 1 LDS write, x writes (the loads had the whole step to land)
      constexpr int NMFMA = (BK / 2) * TM * TN;
      constexpr int NLD = A_IT + B_IT + (PRE ? 2 : 0);
      constexpr int NDSR = (BK / 8) * (TM + TN);
      constexpr int NDSW = A_IT + B_IT;
      constexpr int NMID = NMFMA - NLD - 2 * NDSW;
      static_assert(NMID >= 0, "tile too small for the interleave");
      __builtin_amdgcn_sched_group_barrier(0x100, NDSR / 2, 0);
#pragma unroll
      for (int i = 0; i < NLD; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, NDSR - NDSR / 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NMID, 0);
#pragma unroll
      for (int i = 0; i < NDSW; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
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
      (long long)p.steps_per_split * nsplit < p.steps_total || p.M <= 0 || p.Cout <= 0 ||
      (long long)p.B * p.H * p.W * p.Cin * 4 >= (1ll << 31) || (long long)p.Cout * p.KH * p.KW * p.Cin * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  switch (tile) {
    case TILE_256x64: return launch_tile<256, 64, 4, 1>(p, pre, epi, nsplit, s);
    case TILE_128x128: return launch_tile<128, 128, 2, 2>(p, pre, epi, nsplit, s);
    case TILE_128x64: return launch_tile<128, 64, 4, 1>(p, pre, epi, nsplit, s);
    case TILE_64x128: return launch_tile<64, 128, 1, 4>(p, pre, epi, nsplit, s);
    case TILE_256x128: return launch_tile<256, 128, 2, 2>(p, pre, epi, nsplit, s);
    case TILE_128x256: return launch_tile<128, 256, 2, 2>(p, pre, epi, nsplit, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace frhip
