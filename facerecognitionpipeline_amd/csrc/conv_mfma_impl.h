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
//   k = (ci, ky, kx)           K = KH*KW*Cin    (one K-step = one tap x 32 channels;
//                                                channel chunk outer, tap inner)
//
// Tiles: 256 threads = 4 waves; each wave owns TM x TN 32x32 accumulators.
// LDS holds A as [BM][32+4] and B as [BN][32+4] floats (4-float pad -> the
// ds_read_b128 of 32 consecutive rows hits 16 distinct 16-B slots: conflict free).
// Lane (i = l&31, h = l>>5) reads 4 consecutive k (4h..4h+3 of an 8-k group) of
// its A row and B row with one ds_read_b128 each; MFMA e of the group uses
// element e, so the pair {h=0, h=1} of one MFMA covers k = 4h+e.
//
// Pipeline (register staging, one barrier per K-step, branch-free body): the
// global loads of step s+1 (buffer loads; an out-of-range offset returns 0, which
// is the zero padding) are interleaved with the MFMAs of step s and written to the
// other LDS buffer during its last MFMAs (pre-BN affine applied on the way).
//
// Two schedules over the same body:
//   grid mode       one block per (tile, K-split): blockIdx.x = tile (XCD-aware),
//                   blockIdx.y = split (EPI_RAW writes split-K partial slabs).
//   stream-K mode   (p.sk_blocks > 0) a persistent grid of sk_blocks = CUs x
//                   blocks/CU.  The first sk_dp_tiles tiles go round-robin whole;
//                   the remaining tiles' K-steps are cut into equal contiguous
//                   ranges, one per block, so every block gets the same work and
//                   no half-empty last round exists.  A tile cut across blocks is
//                   finished by the last block to arrive (agent-scope release /
//                   acquire + ticket counter, cdna_hip_programming.md G16): it sums
//                   every contributor's slab in block order, so the result does not
//                   depend on arrival order.
// Numerics: exact f32 products, f32 accumulation (MFMA = fmaf chain), only the
// k summation order differs from the CPU reference.
#pragma once
#include <type_traits>

#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDK = BK + 4;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// bf16x3 staging: x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (both round-to-nearest-even);
// writes 4 hi halves at row[k4] and 4 lo halves 80 B further (row = 40 floats).
__device__ __forceinline__ void split_store(float* row, int k4, float4 v) {
  bf16x4 h, l;
  h[0] = (__bf16)v.x;
  h[1] = (__bf16)v.y;
  h[2] = (__bf16)v.z;
  h[3] = (__bf16)v.w;
  l[0] = (__bf16)(v.x - (float)h[0]);
  l[1] = (__bf16)(v.y - (float)h[1]);
  l[2] = (__bf16)(v.z - (float)h[2]);
  l[3] = (__bf16)(v.w - (float)h[3]);
  char* base = reinterpret_cast<char*>(row) + 8 * k4;
  *reinterpret_cast<bf16x4*>(base) = h;
  *reinterpret_cast<bf16x4*>(base + 80) = l;
}

// XCD-aware bijection: blocks b, b+8, ... share an XCD; give each XCD a contiguous run
// of work items so neighbouring M-tiles and one weight panel share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int BM, int BN, int WM, int WN, bool PRE, int EPI, bool SPLIT>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_mfma_kernel(ConvParams p) {
  constexpr int NTHREADS = 64 * WM * WN;  // one wave per (wm, wn) sub-tile
  constexpr int RPP = NTHREADS / 8;       // staged rows per pass (8 float4 per 32-channel row)
  static_assert(BM % RPP == 0 && BN % RPP == 0, "tile rows must be a multiple of the staging pass");
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  constexpr int A_IT = BM / RPP;  // A rows staged per thread
  constexpr int B_IT = BN / RPP;
  constexpr int ACC = TM * TN * 16;  // accumulator floats per lane

  // fp32 path: rows of 32+4 floats.  SPLIT (bf16x3) path: per row 32+8 bf16 "hi" then
  // 32+8 bf16 "lo" halves = 40 floats; 80-B half-rows keep the b128 fragment reads of 32
  // consecutive rows on 16 distinct 16-B slots (row r starts at slot 5r mod 16).
  constexpr int ROWF = SPLIT ? 40 : LDK;
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * ROWF];
  __shared__ int s_flag;
  float* As0 = lds;
  float* Bs0 = lds + BM * ROWF;
  constexpr int BUF = (BM + BN) * ROWF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int k4 = tid & 7;       // which float4 of the 32-channel K-step
  const int rsub = tid >> 3;    // 0..RPP-1

  const int H = p.H, W = p.W, Cin = p.Cin;
  const int taps = p.KH * p.KW;
  const int Ktot = taps * Cin + p.Cin2;  // weight row length (fused shortcut columns last)
  const int ncc = Cin / BK;              // channel chunks of the main conv
  const int HoWo = p.Ho * p.Wo;

  // Buffer descriptors: an out-of-range offset returns zeros, so padding taps,
  // rows past M and columns past N need no branches (OOB = 0x80000000).
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.B * H * W * Cin * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr2 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.Cin2 ? p.x2 : p.x), (short)0, p.Cin2 ? p.B * H * W * p.Cin2 * 4 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, (short)0, p.Cout * Ktot * 4, 0x00020000);
  constexpr int OOB = 0x80000000;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto ld4 = [](__amdgpu_buffer_rsrc_t rs, int off) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
  };

  floatx16 acc[TM][TN];
  const int frag_row = lane & 31;
  const int frag_k = 4 * (lane >> 5);

  // ---- one tile, K-steps [s_begin, s_end) -> acc (zeroed first) ---------------------
  auto run_segment = [&](int m0, int n0, int s_begin, int s_end) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    if (s_begin >= s_end) return;

    // per-row im2col bases (bytes) for the A rows this thread stages
    int a_base[A_IT], a_iy[A_IT], a_ix[A_IT], a_base2[A_IT];
    unsigned a_row = 0;  // rows inside M
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int m = m0 + rsub + RPP * i;
      if (m < p.M) {
        const int b = m / HoWo;
        const int rem = m - b * HoWo;
        const int oy = rem / p.Wo;
        const int ox = rem - oy * p.Wo;
        a_iy[i] = oy * p.stride - p.pad;
        a_ix[i] = ox * p.stride - p.pad;
        a_base[i] = (((b * H + a_iy[i]) * W + a_ix[i]) * Cin + 4 * k4) * 4;
        a_base2[i] = (((b * H + oy * p.stride) * W + ox * p.stride) * p.Cin2 + 4 * k4) * 4;
        a_row |= 1u << i;
      } else {
        a_iy[i] = -(1 << 20);
        a_ix[i] = 0;
        a_base[i] = 0;
        a_base2[i] = 0;
      }
    }
    int b_base[B_IT];
#pragma unroll
    for (int j = 0; j < B_IT; ++j) {
      const int n = n0 + rsub + RPP * j;
      b_base[j] = n < p.Cout ? (n * Ktot + 4 * k4) * 4 : OOB;
    }

    // counters of the next step to load (cc >= ncc: fused shortcut chunk cc - ncc, tap 0)
    const bool in_sc = p.Cin2 > 0 && s_begin >= p.steps1;
    int tap = in_sc ? 0 : s_begin % taps;
    int cc = in_sc ? ncc + (s_begin - p.steps1) : s_begin / taps;
    int ky = tap / p.KW;
    int kx = tap - ky * p.KW;
    // DEEP (tiles with <= 32 accumulators per lane, where the registers are there): global loads
    // run two K-steps ahead of the MFMAs: step t is loaded into register set (t - s_begin) & 1
    // two iterations before it is computed and written to LDS buffer (t - s_begin) & 1 at the end
    // of the iteration before (the layers with the largest inputs stream them from HBM, whose
    // latency under load is more than one step of MFMAs).  Otherwise one set, one step ahead.
    constexpr bool DEEP = ACC <= 32;
    float4 ra[2][A_IT], rb[2][B_IT];
    float4 psc[2] = {make_float4(1.f, 1.f, 1.f, 1.f), make_float4(1.f, 1.f, 1.f, 1.f)};
    float4 psh[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    unsigned a_okm[2] = {0, 0};

    auto load_step = [&](int r, bool live) {
      if (p.Cin2 > 0 && cc >= ncc) {  // fused shortcut step: x2 at the output's stride
        const int c2 = (cc - ncc) * BK;
        a_okm[r] = 0;
#pragma unroll
        for (int i = 0; i < A_IT; ++i) {
          const unsigned ok = (unsigned)live & ((a_row >> i) & 1u);
          a_okm[r] |= ok << i;
          ra[r][i] = ld4(xr2, ok ? a_base2[i] + c2 * 4 : OOB);
        }
        const int koff2 = (taps * Cin + c2) * 4;
#pragma unroll
        for (int j = 0; j < B_IT; ++j) rb[r][j] = ld4(wr, (b_base[j] == OOB || !live) ? OOB : b_base[j] + koff2);
        return;
      }
      const int c0 = cc * BK;
      const int tap_off = ((ky * W + kx) * Cin + c0) * 4;
      a_okm[r] = 0;
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
        const unsigned ok =
            (unsigned)live & (unsigned)((unsigned)iy < (unsigned)H) & (unsigned)((unsigned)ix < (unsigned)W);
        a_okm[r] |= ok << i;
        ra[r][i] = ld4(xr, ok ? a_base[i] + tap_off : OOB);
      }
      const int koff = (tap * Cin + c0) * 4;
#pragma unroll
      for (int j = 0; j < B_IT; ++j) rb[r][j] = ld4(wr, (b_base[j] == OOB || !live) ? OOB : b_base[j] + koff);
      if constexpr (PRE) {
        psc[r] = *reinterpret_cast<const float4*>(p.pre_scale + c0 + 4 * k4);
        psh[r] = *reinterpret_cast<const float4*>(p.pre_shift + c0 + 4 * k4);
      }
    };
    // counters of the next step; frozen past the segment's end (those loads are OOB no-ops)
    auto advance = [&](bool live) {
      const bool sc = p.Cin2 > 0 && cc >= ncc;  // shortcut chunks: one step each, tap 0
      const int kx1 = sc ? 0 : kx + 1 == p.KW ? 0 : kx + 1;
      const int ky1 = sc ? 0 : kx + 1 == p.KW ? (ky + 1 == p.KH ? 0 : ky + 1) : ky;
      const int tap1 = sc ? 0 : tap + 1 == taps ? 0 : tap + 1;
      const int cc1 = sc || tap + 1 == taps ? cc + 1 : cc;
      kx = live ? kx1 : kx;
      ky = live ? ky1 : ky;
      tap = live ? tap1 : tap;
      cc = live ? cc1 : cc;
    };
    auto store_step = [&](int r, int buf) {
      float* As = As0 + buf * BUF;
      float* Bs = Bs0 + buf * BUF;
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        float4 v = ra[r][i];
        if constexpr (PRE) {
          // BN(x) only where the tap is inside the image: padded zeros stay zero.
          if (a_okm[r] & (1u << i)) {
            v.x = v.x * psc[r].x + psh[r].x;
            v.y = v.y * psc[r].y + psh[r].y;
            v.z = v.z * psc[r].z + psh[r].z;
            v.w = v.w * psc[r].w + psh[r].w;
          }
        }
        if constexpr (SPLIT)
          split_store(As + (rsub + RPP * i) * ROWF, k4, v);
        else
          *reinterpret_cast<float4*>(As + (rsub + RPP * i) * LDK + 4 * k4) = v;
      }
#pragma unroll
      for (int j = 0; j < B_IT; ++j) {
        if constexpr (SPLIT)
          split_store(Bs + (rsub + RPP * j) * ROWF, k4, rb[r][j]);
        else
          *reinterpret_cast<float4*>(Bs + (rsub + RPP * j) * LDK + 4 * k4) = rb[r][j];
      }
    };

    load_step(0, true);  // step s_begin
    advance(s_begin + 1 < s_end);
    if constexpr (DEEP) {
      load_step(1, s_begin + 1 < s_end);  // step s_begin + 1
      advance(s_begin + 2 < s_end);
    }
    store_step(0, 0);
    __syncthreads();
    // iteration for step s from LDS buffer `buf`; DEEP: register set R = buf = (s - s_begin) & 1
    // (compile time), else set 0
    auto iteration = [&](auto Rc, int s, int buf) {
      constexpr int R = decltype(Rc)::value;
      const int cb = DEEP ? R : buf;
      if constexpr (DEEP) {
        load_step(R, s + 2 < s_end);  // step s + 2 into the set step s was staged from
        advance(s + 3 < s_end);
      } else {
        load_step(0, s + 1 < s_end);
        advance(s + 2 < s_end);
      }
      if constexpr (!SPLIT) {
        const float* Ab = As0 + cb * BUF + (wm * TM * 32 + frag_row) * LDK + frag_k;
        const float* Bb = Bs0 + cb * BUF + (wn * TN * 32 + frag_row) * LDK + frag_k;
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
      } else {
        // bf16x3: x = hi + lo (bf16 each); x.y ~= hi.hi + hi.lo + lo.hi, f32 accumulation.
        // Lane (r, h) reads 8 consecutive k (16 B) of hi and of lo for each 16-k group.
        const char* Ab = reinterpret_cast<const char*>(As0 + cb * BUF + (wm * TM * 32 + frag_row) * ROWF) +
                         16 * (lane >> 5);
        const char* Bb = reinterpret_cast<const char*>(Bs0 + cb * BUF + (wn * TN * 32 + frag_row) * ROWF) +
                         16 * (lane >> 5);
        bf16x8 ah[BK / 16][TM], al[BK / 16][TM], bh[BK / 16][TN], bl[BK / 16][TN];
#pragma unroll
        for (int g = 0; g < BK / 16; ++g) {
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            ah[g][a] = *reinterpret_cast<const bf16x8*>(Ab + a * 32 * ROWF * 4 + g * 32);
            al[g][a] = *reinterpret_cast<const bf16x8*>(Ab + a * 32 * ROWF * 4 + 80 + g * 32);
          }
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            bh[g][b] = *reinterpret_cast<const bf16x8*>(Bb + b * 32 * ROWF * 4 + g * 32);
            bl[g][b] = *reinterpret_cast<const bf16x8*>(Bb + b * 32 * ROWF * 4 + 80 + g * 32);
          }
        }
#pragma unroll
        for (int g = 0; g < BK / 16; ++g) {
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[g][a], bh[g][b], acc[a][b], 0, 0, 0);
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[g][a], bl[g][b], acc[a][b], 0, 0, 0);
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[g][a], bh[g][b], acc[a][b], 0, 0, 0);
        }
      }
      // step s + 1 (loaded one iteration ago) into the other LDS buffer, free since the barrier
      // that closed step s - 1
      store_step(DEEP ? R ^ 1 : 0, cb ^ 1);
      // Schedule (MFMA f32 = 64 pipe cycles; other instructions issue in its shadow):
      //   fragments of groups 0-1 | 1 MFMA + 1 global load, x loads | fragments of groups 2-3 |
      //   MFMAs | 2 MFMA + 1 LDS write, x writes (the loads have two steps to land)
      constexpr int NMFMA = SPLIT ? (BK / 16) * 3 * TM * TN : (BK / 2) * TM * TN;
      constexpr int NLD = A_IT + B_IT + (PRE ? 2 : 0);
      constexpr int NDSR = SPLIT ? (BK / 16) * 2 * (TM + TN) : (BK / 8) * (TM + TN);
      constexpr int NDSW = (A_IT + B_IT) * (SPLIT ? 2 : 1);
      constexpr int WPM = SPLIT ? 2 : 1;  // LDS writes per MFMA in the tail of the step
      constexpr int NMID = NMFMA - NLD - (NDSW + WPM - 1) / WPM;
      if constexpr (NMID >= 0) {
        __builtin_amdgcn_sched_group_barrier(0x100, NDSR / 2, 0);
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, NDSR - NDSR / 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NMID, 0);
#pragma unroll
        for (int i = 0; i < (NDSW + WPM - 1) / WPM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x200, WPM, 0);
        }
      }
      __syncthreads();
    };
    if constexpr (DEEP) {
      for (int s = s_begin; s < s_end; s += 2) {
        iteration(std::integral_constant<int, 0>(), s, 0);
        if (s + 1 < s_end) iteration(std::integral_constant<int, 1>(), s + 1, 1);
      }
    } else {
      int buf = 0;
      for (int s = s_begin; s < s_end; ++s) {
        iteration(std::integral_constant<int, 0>(), s, buf);
        buf ^= 1;
      }
    }
  };

  // ---- epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  // Output (and residual) addresses are 32-bit byte offsets into buffer descriptors sized to the
  // tensors: rows past M are dropped by the range check (no per-element branch), and a lane's
  // 16 rows of a 32x32 block sit at compile-time row steps r_e from its first row, so each
  // element's offset is that row's base plus a wave-uniform r_e * Cout * 4 (an SGPR operand).
  constexpr bool RESM = EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU;
  const __amdgpu_buffer_rsrc_t rres = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.res ? p.res : p.y), (short)0,
      p.res ? (RESM ? p.M * p.Cout * 4 : p.B * p.res_H * p.res_W * p.Cout * 4) : 0, 0x00020000);
  auto epilogue = [&](int m0, int n0, int split) {
    const int rowb = p.Cout * 4;  // bytes per output row
    // the output (EPI_RAW: split-K slab `split`), M rows exactly (launch_conv: < 2 GiB)
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.y + (EPI == EPI_RAW ? (long long)split * p.split_stride : 0ll)), (short)0, p.M * rowb, 0x00020000);
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + (wn * TN + b) * 32 + (lane & 31);
      if (n >= p.Cout) continue;
      float sc = 1.f, sh = 0.f, al = 0.f;
      if constexpr (EPI != EPI_RAW) {
        sc = p.post_scale[n];
        sh = p.post_shift[n];
      }
      if constexpr (EPI == EPI_AFFINE_PRELU || EPI == EPI_AFFINE_RES_PRELU) al = p.prelu[n];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        // the lane's first row of this 32x32 block; element e is row m1 + (e & 3) + 8 (e >> 2)
        const int m1 = m0 + (wm * TM + a) * 32 + 4 * (lane >> 5);
        const int vb = m1 * rowb + n * 4;
        // EPI_AFFINE_RES_SUB: (b, oy, ox) of row m1 once; the 16 rows follow by carries
        int sb = 0, soy = 0, sox = 0;
        if constexpr (EPI == EPI_AFFINE_RES_SUB) {
          sb = m1 / HoWo;
          const int rem = m1 - sb * HoWo;
          soy = rem / p.Wo;
          sox = rem - soy * p.Wo;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = (e & 3) + 8 * (e >> 2);  // compile time
          const int so = r * rowb;               // wave-uniform
          float v = acc[a][b][e];
          if constexpr (EPI != EPI_RAW) {
            v = v * sc + sh;
            if constexpr (EPI == EPI_AFFINE_PRELU) v = v > 0.f ? v : v * al;
            if constexpr (RESM) {
              v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rres, vb, so, 0));
              if constexpr (EPI == EPI_AFFINE_RES_PRELU) v = v > 0.f ? v : v * al;
            }
            if constexpr (EPI == EPI_AFFINE_RES_SUB) {
              int bb = sb, oy = soy, ox = sox + r;
              while (ox >= p.Wo) {  // once at most when Wo >= 32 (every stride-2 layer here)
                ox -= p.Wo;
                if (++oy == p.Ho) {
                  oy = 0;
                  ++bb;
                }
              }
              const int ro = (((bb * p.res_H + 2 * oy) * p.res_W + 2 * ox) * p.Cout + n) * 4;
              v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rres, bb < p.B ? ro : 0x80000000, 0, 0));
            }
          }
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), yr, vb, so, 0);
        }
      }
    }
  };

  const int ntile = p.mtiles * p.ntiles;
  if (p.sk_blocks == 0) {
    // ---------------- grid mode ----------------
    const int t = xcd_remap(blockIdx.x, ntile);
    const int mt = t % p.mtiles, nt = t / p.mtiles;
    const int split = blockIdx.y;
    const int s_begin = split * p.steps_per_split;
    const int s_end = min(s_begin + p.steps_per_split, p.steps_total);
    run_segment(mt * BM, nt * BN, s_begin, s_end);
    epilogue(mt * BM, nt * BN, split);
    return;
  }

  // ---------------- stream-K mode ----------------
  const int P = p.sk_blocks;
  const int bid = xcd_remap(blockIdx.x, P);
  const int S = p.steps_total;
  // (1) whole tiles, round-robin; within a round the XCD remap keeps tiles contiguous
  for (int t = bid; t < p.sk_dp_tiles; t += P) {
    const int mt = t % p.mtiles, nt = t / p.mtiles;
    run_segment(mt * BM, nt * BN, 0, S);
    epilogue(mt * BM, nt * BN, 0);
  }
  // (2) the remaining tiles as one flat range of K-steps, cut evenly over the P blocks
  const long long U = (long long)(ntile - p.sk_dp_tiles) * S;
  if (U <= 0) return;
  auto lo_of = [&](int b) { return (long long)b * U / P; };
  const long long lo = lo_of(bid), hi = lo_of(bid + 1);
  float* ws = p.sk_ws;
  for (long long it = lo; it < hi;) {
    const int tl = (int)(it / S);                // tile within the stream-K region
    const int k0 = (int)(it - (long long)tl * S);
    const int k1 = (int)min((long long)S, (long long)k0 + (hi - it));
    const int t = p.sk_dp_tiles + tl;
    const int mt = t % p.mtiles, nt = t / p.mtiles;
    run_segment(mt * BM, nt * BN, k0, k1);
    it += k1 - k0;
    if (k0 == 0 && k1 == S) {
      epilogue(mt * BM, nt * BN, 0);
      continue;
    }
    // slab of this block for this tile: slot 1 if the block had an earlier segment
    const int slot = (lo < (long long)tl * S) ? 1 : 0;
    // write-through (sc1) slab stores: the release below then has no dirty slab lines to write
    // back from L2 before the ticket (the last arriver may sit on another XCD)
    float* mine = ws + ((long long)bid * 2 + slot) * (ACC * NTHREADS);
    const __amdgpu_buffer_rsrc_t mr =
        __builtin_amdgcn_make_buffer_rsrc((void*)mine, (short)0, ACC * NTHREADS * 4, 0x00020000);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e]), mr,
                                                (((a * TN + b) * 16 + e) * NTHREADS + tid) * 4, 0, 16);
    // blocks holding a segment of tile tl: first..last (block ranges are contiguous)
    const long long t_lo = (long long)tl * S, t_hi = t_lo + S;
    int first = (int)((t_lo * P) / U);
    while (first + 1 < P && lo_of(first + 1) <= t_lo) ++first;
    while (first > 0 && lo_of(first) > t_lo) --first;
    int last = (int)(((t_hi - 1) * P) / U);
    while (last + 1 < P && lo_of(last + 1) <= t_hi - 1) ++last;
    while (last > 0 && lo_of(last) > t_hi - 1) --last;
    const int nseg = last - first + 1;
    // publish: every wave drains its stores, then one release + ticket (G16 counter form)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(p.sk_cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = ticket == nseg - 1;
      if (is_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p.sk_cnt[tl] = 0;  // re-arm for the next launch (counters start zeroed at allocation)
      }
      s_flag = is_last;
    }
    __syncthreads();
    if (!s_flag) continue;
    // last arriver: sum every contributor's slab in block order (arrival-order independent)
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
    for (int c = first; c <= last; ++c) {
      const int cslot = (lo_of(c) < t_lo) ? 1 : 0;
      const float* src = ws + ((long long)c * 2 + cslot) * (ACC * NTHREADS);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[a][b][e] += src[((a * TN + b) * 16 + e) * NTHREADS + tid];
    }
    epilogue(mt * BM, nt * BN, 0);
  }
}

// SET selects the (PRE, EPI) instances a translation unit compiles: 0 = the embedding
// network's, 1 = the detector's (no pre-BN; ReLU via zero PReLU slopes).
template <int BM, int BN, int WM, int WN, bool SPLIT, int SET = 0>
static hipError_t launch_tile(const ConvParams& p0, bool pre, Epi epi, int nsplit, hipStream_t s) {
  constexpr int NTHREADS = 64 * WM * WN;
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (p.Cout + BN - 1) / BN;
  p.sk_blocks = 0;
  p.sk_dp_tiles = 0;
  if (p.sk_cus > 0) {
    static int occ[8][2] = {};  // blocks per CU per (PRE, EPI) instance of this tile
    int& o = occ[epi][pre ? 1 : 0];
    if (o == 0) {
      hipError_t e = hipSuccess;
#define FR_OCC_CASE(PRE_, EPI_) \
  if (pre == PRE_ && epi == EPI_) \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, conv_mfma_kernel<BM, BN, WM, WN, PRE_, EPI_, SPLIT>, NTHREADS, 0);
      if constexpr (SET == 0) {
        FR_OCC_CASE(true, EPI_AFFINE_PRELU)
        FR_OCC_CASE(false, EPI_AFFINE_RES)
        FR_OCC_CASE(false, EPI_AFFINE_RES_SUB)
        FR_OCC_CASE(false, EPI_AFFINE)
        FR_OCC_CASE(true, EPI_RAW)
        FR_OCC_CASE(false, EPI_RAW)
      } else {
        FR_OCC_CASE(false, EPI_AFFINE)
        FR_OCC_CASE(false, EPI_AFFINE_PRELU)
        FR_OCC_CASE(false, EPI_AFFINE_RES)
        FR_OCC_CASE(false, EPI_AFFINE_RES_PRELU)
      }
#undef FR_OCC_CASE
      if (e != hipSuccess || o < 1) o = 1;
    }
    const long long ntile = (long long)p.mtiles * p.ntiles;
    const long long P0 = (long long)p.sk_cus * o;
    // at least ~8 K-steps per block: a tile's last arriver sums one slab per contributor, so
    // cutting a small grid (batch 1: 2-4 tiles) over every CU would make that fixup the
    // critical path; large grids are unaffected (ntile * steps / 8 >> CUs)
    p.sk_blocks = (int)min(P0, ntile * max(1, p.steps_total / 8));
  }
  dim3 grid(p.sk_blocks > 0 ? p.sk_blocks : p.mtiles * p.ntiles, p.sk_blocks > 0 ? 1 : nsplit), block(NTHREADS);
  if (p.sk_blocks > 0) {
    const int ntile = p.mtiles * p.ntiles;
    // whole tiles round-robin except the last (1 + fractional) rounds, which go stream-K
    const int rounds = ntile / p.sk_blocks;
    const int rem = ntile - rounds * p.sk_blocks;
    p.sk_dp_tiles = rem == 0 ? ntile : (rounds >= 1 ? (rounds - 1) * p.sk_blocks : 0);
    if ((long long)(ntile - p.sk_dp_tiles) * p.steps_total < p.sk_blocks && p.sk_dp_tiles < ntile)
      p.sk_blocks = (ntile - p.sk_dp_tiles) * p.steps_total;
    grid.x = p.sk_blocks;
    if (p.sk_dp_tiles < ntile && (!p.sk_ws || !p.sk_cnt || ntile - p.sk_dp_tiles > p.sk_cnt_cap ||
                                  (long long)p.sk_blocks * 2 * BM * BN > p.sk_ws_floats))
      return hipErrorInvalidValue;
  }
#define FR_CONV_CASE(PRE_, EPI_)                                                                    \
  if (pre == PRE_ && epi == EPI_) {                                                                 \
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, PRE_, EPI_, SPLIT>), grid, block, 0, s, p); \
    return hipGetLastError();                                                                       \
  }
  if constexpr (SET == 0) {
    FR_CONV_CASE(true, EPI_AFFINE_PRELU)
    FR_CONV_CASE(false, EPI_AFFINE_RES)
    FR_CONV_CASE(false, EPI_AFFINE_RES_SUB)
    FR_CONV_CASE(false, EPI_AFFINE)
    FR_CONV_CASE(true, EPI_RAW)
    FR_CONV_CASE(false, EPI_RAW)
  } else {
    FR_CONV_CASE(false, EPI_AFFINE)
    FR_CONV_CASE(false, EPI_AFFINE_PRELU)
    FR_CONV_CASE(false, EPI_AFFINE_RES)
    FR_CONV_CASE(false, EPI_AFFINE_RES_PRELU)
  }
#undef FR_CONV_CASE
  return hipErrorInvalidValue;
}

}  // namespace
}  // namespace frhip
