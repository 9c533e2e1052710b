// Winograd F(6x6, 3x3) convolution in f32 on gfx950 (v_mfma_f32_16x16x4_f32): an EXPERIMENT, not
// in the library (tools/w6_bench.cpp checks it against a float64 direct conv and times it against
// wino4_kernel).  Measured and dropped in round 5: 0.97-1.11x F(4x4) at B = 256, 4-10x at serving
// sizes (profiles/r05/w6_*.txt).
//
// Per 6x6 output tile and (cin, cout) pair the algorithm does 64 products instead of 324 (F(4x4):
// 36 per 16 outputs).  At IR-101 stage 3 (14x14 maps, 52% of the forward) both tile sizes waste
// the same canvas share (period 15: 15^2/14^2), so F(6x6) executes 21% fewer MFMA products there.
// Points 0, +-1, +-2, +-1/2, inf (the NNPACK set):
//   B^T = [1 0 -21/4 0 21/4 0 -1 0; 0 1 1 -17/4 -17/4 1 1 0; 0 -1 1 17/4 -17/4 -1 1 0;
//          0 1/2 1/4 -5/2 -5/4 2 1 0; 0 -1/2 1/4 5/2 -5/4 -2 1 0; 0 2 4 -5/2 -5 1/2 1 0;
//          0 -2 4 5/2 -5 -1/2 1 0; 0 -1 0 21/4 0 -21/4 0 1]
//   G   = [1 0 0; -2/9 -2/9 -2/9; -2/9 2/9 -2/9; 1/90 1/45 2/45; 1/90 -1/45 2/45;
//          32/45 16/45 8/45; 32/45 -16/45 8/45; 0 0 1]
//   A^T = [1 1 1 1 1 1 1 0; 0 1 -1 2 -2 1/2 -1/2 0; 0 1 1 4 4 1/4 1/4 0; 0 1 -1 8 -8 1/8 -1/8 0;
//          0 1 1 16 16 1/16 1/16 0; 0 1 -1 32 -32 1/32 -1/32 1]
// fp32 error per layer, simulated against a float64 direct conv (256 channels, U built in double):
// 2.8x F(4x4)'s; measured 7-16e-5 at |y| ~ 5 (F(4x4): 2-9e-5).
//
// Structure (not F(4x4)'s warp specialisation): 64 transform elements x 16 tiles x 16 couts of
// accumulators are 256 registers per lane, which only a wave alone on its SIMD can hold (512
// VGPR + AGPR), so each of the 4 waves of a workgroup does both jobs for its 16 couts: per K-step
// (16 input channels) it transforms 4 of the item's 16 tiles into the LDS ring slot of the NEXT
// K-step while it runs this K-step's 256 MFMAs from the current slot; one workgroup barrier per
// K-step hands the slots over (two slots of 64 KiB).  The transform runs as 14 pieces placed
// between MFMA pairs (W6_PSTART / W6_PSTRIDE) or as one burst (W6_BURST); U is loaded W6_UR xi
// ahead.  What the single-wave form cannot do is hide its own VALU and dependency bubbles behind a
// second wave's MFMAs: a K-step costs ~14k cycles against 8.2k of MFMA issue even without global
// loads (W6_NOLOAD / W6_NOULOAD timing variants).  The pre-BN masks are taken from the patch
// offsets; a form with float mask registers gave wrong values on the last canvas row.
//
// Work item = 16 tiles x 64 couts x 64 xi; wave w owns couts 16w .. 16w+15.  Fragment layouts as in
// conv_winograd4.hip (v_mfma_f32_16x16x4_f32: A[l&15][k=l>>4] = U, B[k=l>>4][l&15] = V; a lane's
// accumulator holds 4 consecutive couts of one tile): V slot [64 xi][64 lanes (vslot)][4] (64 KiB),
// U [64 xi][Cout/16][Cin/16][64 lanes][4].
#include <algorithm>
#include <cmath>

#include "frhip_kernels.h"

namespace frhip {

// canvas + items of an F(6x6) layer (w6_setup fills the geometry fields)
struct Wino6Params {
  const float* x;
  const float* u;
  float* y;
  const float* pre_t;  // pre-BN folded: t = shift / scale per input channel (scale in U), or null
  const float* post_scale;
  const float* post_shift;
  const float* prelu;
  const float* res;
  int B, H, W, Cin, Cout;
  int Pr, Pc, NC, TWc, ntiles, mblocks, nblocks, nbg;
};

bool wino6_supported(int Cin, int Cout, int kh, int kw, int stride, int pad);
size_t wino6_weight_floats(int Cout, int Cin);
hipError_t launch_wino6_weights(const float* w, const float* pre_scale, float* u, int Cout, int Cin, hipStream_t s);
hipError_t launch_wino6(const Wino6Params& p, bool pre, Epi epi, hipStream_t s);
void wino6_canvas(Wino6Params& p);

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int NXI6 = 64;
constexpr int FT6 = 16;
constexpr int FN6 = 64;
constexpr int KC6 = 16;
constexpr int VSTEP6 = NXI6 * FT6 * KC6;  // floats of one ring slot (16,384 = 64 KiB)
#ifndef W6_UR
#define W6_UR 8
#endif
constexpr int UR6 = W6_UR;  // xi of U in flight per wave (64 % UR6 == 0)
constexpr int BIGOFF6 = 0x7F000000;
#ifndef W6_PSTART  // MFMA pair after which the first transform piece runs, and the pairs between pieces
#define W6_PSTART 4
#endif
#ifndef W6_PSTRIDE
#define W6_PSTRIDE 2
#endif
static_assert(NXI6 % UR6 == 0, "U ring phase must repeat every K-step");
static_assert(2 * VSTEP6 * 4 <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int xcd_remap6(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc6(const void* ptr, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(ptr);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), (short)0, n,
                                           0x00020000);
}

__device__ __forceinline__ f4 ld4_6(__amdgpu_buffer_rsrc_t r, int off, int soff = 0) {
#ifndef W6_NOULOAD
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
#else  // timing only: no U loads (the residual loads of the epilogue go too)
  const u32x4 v = {(unsigned)off, (unsigned)soff, 0u, 0u};
#endif
  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

// the ring's conflict-free 16-byte slot of fragment lane l (as conv_winograd4.hip's vslot)
__device__ __forceinline__ int vslot6(int l) {
  const int k = l >> 4;
  return l ^ ((k & 1) * 2 + (k >> 1) * 12);
}

// canvas coordinate -> in-image coordinate (or -1) and the image slot (base or base + 1)
__device__ __forceinline__ int canvas_coord6(int v, int base, int P, int H, bool sep, int& slot) {
  const int y = v - base * P, y1 = y - P;
  const bool in0 = (unsigned)y < (unsigned)H;
  const bool in1 = sep && (unsigned)y1 < (unsigned)H;
  slot = base + (in1 ? 1 : 0);
  return in0 ? y : (in1 ? y1 : -1);
}

// 1-D input transform B^T d (8 -> 8) on two channels, 26 packed ops
__device__ __forceinline__ void bt8v(const f2 (&d)[8], f2 (&t)[8]) {
  const f2 c214 = {5.25f, 5.25f}, m174 = {-4.25f, -4.25f}, c025 = {0.25f, 0.25f}, m125 = {-1.25f, -1.25f};
  const f2 c05 = {0.5f, 0.5f}, m25 = {-2.5f, -2.5f}, c2 = {2.f, 2.f}, c4 = {4.f, 4.f}, m5 = {-5.f, -5.f};
  t[0] = __builtin_elementwise_fma(c214, d[4] - d[2], d[0] - d[6]);
  t[7] = __builtin_elementwise_fma(c214, d[3] - d[5], d[7] - d[1]);
  const f2 a = __builtin_elementwise_fma(m174, d[4], d[2] + d[6]);
  const f2 b = __builtin_elementwise_fma(m174, d[3], d[1] + d[5]);
  t[1] = a + b;
  t[2] = a - b;
  const f2 c = __builtin_elementwise_fma(m125, d[4], __builtin_elementwise_fma(c025, d[2], d[6]));
  const f2 e = __builtin_elementwise_fma(c2, d[5], __builtin_elementwise_fma(m25, d[3], c05 * d[1]));
  t[3] = c + e;
  t[4] = c - e;
  const f2 f = __builtin_elementwise_fma(m5, d[4], __builtin_elementwise_fma(c4, d[2], d[6]));
  const f2 h = __builtin_elementwise_fma(c05, d[5], __builtin_elementwise_fma(m25, d[3], c2 * d[1]));
  t[5] = f + h;
  t[6] = f - h;
}

// 1-D output transform A^T m (8 -> 6) on four couts
__device__ __forceinline__ void at8q(const f4 (&m)[8], f4 (&o)[6]) {
  const f4 p12 = m[1] + m[2], d12 = m[1] - m[2];
  const f4 p34 = m[3] + m[4], d34 = m[3] - m[4];
  const f4 p56 = m[5] + m[6], d56 = m[5] - m[6];
  const f4 c2 = {2.f, 2.f, 2.f, 2.f}, c4 = {4.f, 4.f, 4.f, 4.f}, c8 = {8.f, 8.f, 8.f, 8.f};
  const f4 c16 = {16.f, 16.f, 16.f, 16.f}, c32 = {32.f, 32.f, 32.f, 32.f};
  const f4 h2 = {0.5f, 0.5f, 0.5f, 0.5f}, h4 = {0.25f, 0.25f, 0.25f, 0.25f}, h8 = {0.125f, 0.125f, 0.125f, 0.125f};
  const f4 h16 = {0.0625f, 0.0625f, 0.0625f, 0.0625f}, h32 = {0.03125f, 0.03125f, 0.03125f, 0.03125f};
  o[0] = m[0] + p12 + p34 + p56;
  o[1] = __builtin_elementwise_fma(h2, d56, __builtin_elementwise_fma(c2, d34, d12));
  o[2] = __builtin_elementwise_fma(h4, p56, __builtin_elementwise_fma(c4, p34, p12));
  o[3] = __builtin_elementwise_fma(h8, d56, __builtin_elementwise_fma(c8, d34, d12));
  o[4] = __builtin_elementwise_fma(h16, p56, __builtin_elementwise_fma(c16, p34, p12));
  o[5] = __builtin_elementwise_fma(h32, d56, __builtin_elementwise_fma(c32, d34, d12)) + m[7];
}

struct Item6 {
  int mb, nb;
};
__device__ __forceinline__ Item6 item6_of(const Wino6Params& p, int gi) {
  const int NB = p.nblocks, GM = p.nbg;
  const int grp = gi / (GM * NB), rem = gi - grp * GM * NB;
  const int gm = min(GM, p.mblocks - grp * GM);
  Item6 it;
  it.nb = rem / gm;
  it.mb = grp * GM + (rem - it.nb * gm);
  return it;
}

// PRE: pre-BN folded into U + shift t at in-image pixels (IR conv1, EPI_AFFINE_PRELU); otherwise
// EPI_AFFINE_RES (IR conv2: BN + identity residual) or EPI_AFFINE_PRELU without pre-BN.
template <bool PRE, int EPI>
__global__ __launch_bounds__(256, 1) void wino6_kernel(Wino6Params p) {
  __shared__ __attribute__((aligned(16))) float ring[2 * VSTEP6];
  constexpr bool RES = EPI == EPI_AFFINE_RES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout;
  const int KST = Cin / KC6;
  const int nitems = p.mblocks * p.nblocks;
  const int bid = blockIdx.x, nblk = gridDim.x;
  const int nloc = (nitems - bid + nblk - 1) / nblk;
  if (nloc <= 0) return;
  const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
  auto item_at = [&](int j) { return item6_of(p, xcd_remap6(bid + min(j, nloc - 1) * nblk, nitems)); };

  // ---- transform side: this wave's tiles 4w .. 4w+3 of the item; lane (half h, tile ii, channel
  // pair pr) holds patch columns 4h .. 4h+3 (8 rows) of channels 2pr, 2pr+1
  const int half = lane >> 5, ii = (lane >> 3) & 3, pr = lane & 7;
  const int ti = 4 * w + ii, ch = 2 * pr;
  const __amdgpu_buffer_rsrc_t xr = rsrc6(p.x, p.B * H * W * Cin * 4);
  int roff[8], coff[4];
  auto enter_item = [&](int j) {
    const Item6 it = item_at(j);
    const int T = it.mb * FT6 + ti;
    const int tr = T / p.TWc, tc = T - tr * p.TWc;
    const int ir0 = (6 * tr) / p.Pr, ic0 = (6 * tc) / p.Pc;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int rs;
      const int y = canvas_coord6(6 * tr - 1 + e, ir0, p.Pr, H, sep_r, rs);
      const bool in = y >= 0 && rs * p.NC < p.B && T < p.ntiles;
      roff[e] = in ? (rs * p.NC * H + y) * W * Cin * 4 : BIGOFF6;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int cs;
      const int x = canvas_coord6(6 * tc - 1 + 4 * half + e, ic0, p.Pc, W, sep_c, cs);
      const bool in = x >= 0 && cs < p.NC;
      coff[e] = in ? ((cs * H * W + x) * Cin + ch) * 4 : BIGOFF6;
    }
  };
  f2 d[8][4];
  f2 tsh = {0.f, 0.f};
  auto load = [&](int step) {
    const int soff = __builtin_amdgcn_readfirstlane(step * KC6 * 4);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#ifndef W6_NOLOAD
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, (int)((unsigned)roff[a] + (unsigned)coff[b]), soff, 0);
#else  // timing only: no patch loads
        const u32x2 v = {(unsigned)(roff[a] + soff), (unsigned)coff[b]};
#endif
        d[a][b] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
      }
    if constexpr (PRE) tsh = *reinterpret_cast<const f2*>(p.pre_t + step * KC6 + ch);
  };
  // ring address of (tile ti, channels ch, ch+1): fragment lane 16 (ch / 4) + ti, elements ch % 4 ..
  // +1; half h holds transform rows 4h .. 4h+3, i.e. xi from 32 h
  // The transform in 14 pieces the K-step places between its MFMAs (piece q after MFMA pair
  // W6_PSTART + W6_PSTRIDE q): pre-BN shift (2), four column transforms, the partner exchange (4),
  // four row transforms with their ring writes.
  const int dst_off = vslot6(16 * (ch >> 2) + ti) * 4 + (ch & 3) + half * 32 * 256;
  auto transform_piece = [&](int q, float* slot) {
    if (q < 2) {
#ifndef W6_NO_SHIFT_PIECE
      if constexpr (PRE)
#else
      if constexpr (false)
#endif
#pragma unroll
        for (int a = 4 * q; a < 4 * q + 4; ++a) {  // in-image taps: both offsets real
          const f2 trow = roff[a] != BIGOFF6 ? tsh : f2{0.f, 0.f};
#pragma unroll
          for (int b = 0; b < 4; ++b) d[a][b] += coff[b] != BIGOFF6 ? trow : f2{0.f, 0.f};
        }
    } else if (q < 6) {  // column b: d[.][b] <- (B^T d)[.][b]
      const int b = q - 2;
      f2 c[8], o[8];
#pragma unroll
      for (int a = 0; a < 8; ++a) c[a] = d[a][b];
      bt8v(c, o);
#pragma unroll
      for (int a = 0; a < 8; ++a) d[a][b] = o[a];
    } else if (q < 10) {
      // partner exchange: half 0 keeps transform rows 0-3, half 1 rows 4-7; after it d[k][b] holds
      // row 4h + k of column b and d[4 + k][b] row 4h + k of column 4 + b
      const int k = q - 6;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(d[k][b][e]), __float_as_uint(d[4 + k][b][e]),
                                                          false, false);
          d[k][b][e] = __uint_as_float(r[0]);
          d[4 + k][b][e] = __uint_as_float(r[1]);
        }
    } else {
      const int k = q - 10;
      const f2 row[8] = {d[k][0], d[k][1], d[k][2], d[k][3], d[4 + k][0], d[4 + k][1], d[4 + k][2], d[4 + k][3]};
      f2 v[8];
      bt8v(row, v);
      float* dst = slot + dst_off;
#pragma unroll
      for (int c = 0; c < 8; ++c) *reinterpret_cast<f2*>(dst + (8 * k + c) * 256) = v[c];
    }
  };
  auto transform_store = [&](float* slot) {
#pragma unroll
    for (int q = 0; q < 14; ++q) transform_piece(q, slot);
  };

  // ---- MFMA side: couts 16w .. 16w+15 of every item
  const __amdgpu_buffer_rsrc_t ur = rsrc6(p.u, NXI6 * Cout * Cin * 4);
  const int NB16 = Cout / 16;
  const int XS = NB16 * KST * 1024;  // bytes between the xi planes of U
  auto ubase = [&](int j) {
    const Item6 it = item_at(j);
    return (min(it.nb * 4 + w, NB16 - 1) * KST) * 1024;
  };
  const int lo = lane * 16;
  const float* vrd = ring + vslot6(lane) * 4;
  const __amdgpu_buffer_rsrc_t yr = rsrc6(p.y, p.B * H * W * Cout * 4);
  const __amdgpu_buffer_rsrc_t rr = rsrc6(p.res, RES ? p.B * H * W * Cout * 4 : 0);
  const int n = lane & 15, rg = lane >> 4;

  // One K-step of stream step g (ring slot g % 2): the patch loads of the next stream step (K-step
  // `lstep` of the geometry in roff / coff) go out first, then the 256 MFMAs in pairs of xi with
  // their fragment reads and U refills, the transform pieces of those patches placed between them
  // (f32 MFMA and VALU do not co-issue on a SIMD, so the point is only that no piece waits for its
  // loads: the first runs a few MFMA pairs after they were issued).  Branch-free; one barrier.
  f4 uring[UR6];
  f4 acc[NXI6];
  auto kstep = [&](int g, int lstep, int cur, int nxt) {
    load(lstep);
    __builtin_amdgcn_sched_barrier(0);  // the patch loads go out first
    const float* vb = vrd + (g & 1) * VSTEP6;
    float* nslot = ring + ((g + 1) & 1) * VSTEP6;
    f4 a0n = *reinterpret_cast<const f4*>(vb), a1n = *reinterpret_cast<const f4*>(vb + 256);
#pragma unroll
    for (int x = 0; x < NXI6; x += 2) {
      const f4 a0 = a0n, a1 = a1n;
      if (x + 2 < NXI6) {
        a0n = *reinterpret_cast<const f4*>(vb + (x + 2) * 256);
        a1n = *reinterpret_cast<const f4*>(vb + (x + 3) * 256);
      }
      const f4 u0 = uring[x % UR6], u1 = uring[(x + 1) % UR6];
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(u0.x, a0.x, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u1.x, a1.x, acc[x + 1], 0, 0, 0);
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(u0.y, a0.y, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u1.y, a1.y, acc[x + 1], 0, 0, 0);
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(u0.z, a0.z, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u1.z, a1.z, acc[x + 1], 0, 0, 0);
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(u0.w, a0.w, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u1.w, a1.w, acc[x + 1], 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int y = x + e;
        uring[y % UR6] = y + UR6 < NXI6 ? ld4_6(ur, lo, (y + UR6) * XS + cur) : ld4_6(ur, lo, (y + UR6 - NXI6) * XS + nxt);
      }
      // the next stream step's transform into the other slot (its last readers finished before the
      // previous barrier), a piece at a time
#ifndef W6_BURST
      const int pq = x / 2 - W6_PSTART;
      if (pq >= 0 && pq % W6_PSTRIDE == 0 && pq / W6_PSTRIDE < 14) transform_piece(pq / W6_PSTRIDE, nslot);
#else  // the whole transform as one run of VALU after MFMA pair W6_PSTART
      if (x / 2 == W6_PSTART)
#pragma unroll
        for (int q = 0; q < 14; ++q) transform_piece(q, nslot);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: item 0's geometry, step 0 loaded and transformed into slot 0
  enter_item(0);
  load(0);
  int ub = ubase(0);
#pragma unroll
  for (int r = 0; r < UR6; ++r) uring[r] = ld4_6(ur, lo, r * XS + ub);
  transform_store(ring);
  __syncthreads();

  for (int j = 0; j < nloc; ++j) {
    const Item6 it = item_at(j);
    const bool live = it.nb * 64 + w * 16 < Cout;
    const int ub_next = ubase(j + 1);
#pragma unroll
    for (int x = 0; x < NXI6; ++x) acc[x] = f4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s + 1 < KST; ++s) kstep(j * KST + s, s + 1, ub + s * 1024, ub + (s + 1) * 1024);
    // the last K-step loads the next item's step 0 (past the last item: the last item's again,
    // transformed into a slot nobody reads)
    enter_item(j + 1);
    kstep(j * KST + KST - 1, 0, ub + (KST - 1) * 1024, ub_next);
    ub = ub_next;
    // ---- epilogue: lane (tile n, cout quad rg) holds couts 4rg .. 4rg+3 of tile n for all 64 xi
    const int T = it.mb * FT6 + n;
    const int tr = T / p.TWc, tc = T - tr * p.TWc;
    const int ir0 = (6 * tr) / p.Pr, ic0 = (6 * tc) / p.Pc;
    const int cout0 = min(it.nb * 64 + w * 16, Cout - 16) + 4 * rg;
    int ro[6], co[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      int rs, cs;
      const int y = canvas_coord6(6 * tr + e, ir0, p.Pr, H, sep_r, rs);
      const int x = canvas_coord6(6 * tc + e, ic0, p.Pc, W, sep_c, cs);
      ro[e] = (y >= 0 && rs * p.NC < p.B && T < p.ntiles && live) ? ((rs * p.NC * H + y) * W * Cout + cout0) * 4 : BIGOFF6;
      co[e] = (x >= 0 && cs < p.NC) ? (cs * H * W + x) * Cout * 4 : BIGOFF6;
    }
    const f4 sc = *reinterpret_cast<const f4*>(p.post_scale + cout0);
    const f4 sh = *reinterpret_cast<const f4*>(p.post_shift + cout0);
    f4 al = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_AFFINE_PRELU) al = *reinterpret_cast<const f4*>(p.prelu + cout0);
    // A^T M A in three passes of two output columns (each pass re-reads the accumulators and
    // redoes the shared sums of its rows: 96 fewer live registers than all six at once)
#pragma unroll
    for (int xp = 0; xp < 3; ++xp) {
      f4 t2[8][2];
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const f4 m8[8] = {acc[8 * a], acc[8 * a + 1], acc[8 * a + 2], acc[8 * a + 3],
                          acc[8 * a + 4], acc[8 * a + 5], acc[8 * a + 6], acc[8 * a + 7]};
        f4 o6[6];
        at8q(m8, o6);
        t2[a][0] = o6[2 * xp];
        t2[a][1] = o6[2 * xp + 1];
      }
#pragma unroll
      for (int xh = 0; xh < 2; ++xh) {
        const int xq = 2 * xp + xh;
        const f4 c8[8] = {t2[0][xh], t2[1][xh], t2[2][xh], t2[3][xh], t2[4][xh], t2[5][xh], t2[6][xh], t2[7][xh]};
        f4 o6[6];
        at8q(c8, o6);
        f4 rv[6];
        if constexpr (RES)
#pragma unroll
          for (int yq = 0; yq < 6; ++yq) rv[yq] = ld4_6(rr, (int)((unsigned)ro[yq] + (unsigned)co[xq]));
#pragma unroll
        for (int yq = 0; yq < 6; ++yq) {
          f4 v = __builtin_elementwise_fma(o6[yq], sc, sh);
          if constexpr (EPI == EPI_AFFINE_PRELU)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * al[r];
          if constexpr (RES) v += rv[yq];
          const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
          __builtin_amdgcn_raw_buffer_store_b128(bits, yr, (int)((unsigned)ro[yq] + (unsigned)co[xq]), 0, 0);
        }
      }
    }
  }
}

// G g G^T of every (cout, cin) filter in double, rounded once to f32, in the U fragment order
__global__ void wino6_weight_kernel(const float* __restrict__ w, const float* __restrict__ pre_scale,
                                    float* __restrict__ u, int Cout, int Cin) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Cout * Cin) return;
  const int o = idx / Cin, i = idx - o * Cin;
  const double G[8][3] = {{1.0, 0.0, 0.0},
                          {-2.0 / 9, -2.0 / 9, -2.0 / 9},
                          {-2.0 / 9, 2.0 / 9, -2.0 / 9},
                          {1.0 / 90, 1.0 / 45, 2.0 / 45},
                          {1.0 / 90, -1.0 / 45, 2.0 / 45},
                          {32.0 / 45, 16.0 / 45, 8.0 / 45},
                          {32.0 / 45, -16.0 / 45, 8.0 / 45},
                          {0.0, 0.0, 1.0}};
  double g[3][3];
#pragma unroll
  for (int y = 0; y < 3; ++y)
#pragma unroll
    for (int x = 0; x < 3; ++x)
      g[y][x] = (double)w[((long long)(o * 3 + y) * 3 + x) * Cin + i] * (pre_scale ? (double)pre_scale[i] : 1.0);
  double tg[8][3];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int x = 0; x < 3; ++x) tg[a][x] = G[a][0] * g[0][x] + G[a][1] * g[1][x] + G[a][2] * g[2][x];
  const int NB16 = Cout / 16, KS = Cin / KC6;
  const int nb16 = o >> 4, nn = o & 15;
  const int s = i / KC6, c = i % KC6;
  const int ln = 16 * (c >> 2) + nn, m = c & 3;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const double v = tg[a][0] * G[b][0] + tg[a][1] * G[b][1] + tg[a][2] * G[b][2];
      const int xi = 8 * a + b;
      u[(((long long)(xi * NB16 + nb16) * KS + s) * 64 + ln) * 4 + m] = (float)v;
    }
}

int w6_cus() {
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus > 0 ? cus : 256;
}

}  // namespace

bool wino6_supported(int Cin, int Cout, int kh, int kw, int stride, int pad) {
  return kh == 3 && kw == 3 && stride == 1 && pad == 1 && Cin % 16 == 0 && Cin >= 16 && Cout % 64 == 0;
}

size_t wino6_weight_floats(int Cout, int Cin) { return (size_t)NXI6 * Cout * Cin; }

hipError_t launch_wino6_weights(const float* w, const float* pre_scale, float* u, int Cout, int Cin, hipStream_t s) {
  if (Cout % 16 || Cin % KC6) return hipErrorInvalidValue;
  const int n = Cout * Cin;
  hipLaunchKernelGGL(wino6_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, pre_scale, u, Cout, Cin);
  return hipGetLastError();
}

// Canvas for 6x6 tiles: P = H when 6 | H, else H + 1 (one zero separator row / column between
// images), NC images per canvas row so that NC * P is a multiple of 6.
void wino6_canvas(Wino6Params& p) {
  auto period = [](int h) { return h % 6 == 0 ? h : h + 1; };
  p.Pr = period(p.H);
  p.Pc = period(p.W);
  p.NC = 1;
  while ((p.NC * p.Pc) % 6) ++p.NC;
  if (p.NC > p.B) p.NC = p.B;
  const int crow = (p.B + p.NC - 1) / p.NC;
  p.TWc = (p.NC * p.Pc + 5) / 6;
  const int TRc = (crow * p.Pr + 5) / 6;
  p.ntiles = TRc * p.TWc;
}

hipError_t launch_wino6(const Wino6Params& p0, bool pre, Epi epi, hipStream_t s) {
  Wino6Params p = p0;
  if (!wino6_supported(p.Cin, p.Cout, 3, 3, 1, 1) || p.B < 1 || (pre && !p.pre_t) ||
      (long long)p.B * p.H * p.W * p.Cin * 4 >= BIGOFF6 || (long long)p.B * p.H * p.W * p.Cout * 4 >= (1ll << 31) ||
      (long long)NXI6 * p.Cout * p.Cin * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  wino6_canvas(p);
  if (pre && p.NC > 1 && p.B % p.NC && p.Pr == p.H) {
    p.Pr = p.H + 1;  // absent images of a partial last canvas row stay outside every window
    p.ntiles = ((((p.B + p.NC - 1) / p.NC) * p.Pr + 5) / 6) * p.TWc;
  }
  p.mblocks = (p.ntiles + FT6 - 1) / FT6;
  p.nblocks = p.Cout / FN6;
  p.nbg = std::max(1, std::min(p.mblocks, std::max(32 / p.nblocks, 8)));
  const int nT = p.mblocks * p.nblocks;
  const dim3 grid(std::min(nT, w6_cus()));
  if (pre && epi == EPI_AFFINE_PRELU)
    hipLaunchKernelGGL((wino6_kernel<true, EPI_AFFINE_PRELU>), grid, dim3(256), 0, s, p);
  else if (!pre && epi == EPI_AFFINE_RES)
    hipLaunchKernelGGL((wino6_kernel<false, EPI_AFFINE_RES>), grid, dim3(256), 0, s, p);
  else if (!pre && epi == EPI_AFFINE_PRELU)
    hipLaunchKernelGGL((wino6_kernel<false, EPI_AFFINE_PRELU>), grid, dim3(256), 0, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace frhip
