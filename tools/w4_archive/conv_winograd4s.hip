// Winograd F(4x4, 3x3) in f32 on gfx950 with symmetric waves: the launches of whole items (grids of
// at least one 16-tile x 64-cout item per CU; the batch-256 forward's layers).
//
// Same algorithm, U and canvas as conv_winograd4.hip (see there for the matrices, the canvas and the
// fragment layouts); what differs is how a workgroup's 8 waves share the work.  The shipping
// split there gives each SIMD an MFMA wave (all 36 xi of 16 couts: 144 accumulators) and a
// transform wave that hand V over through LDS counters; its K-step runs 6,400-6,800 cycles against
// 4,608 of MFMA issue, ~1,300-1,700 of them waiting for the transform's data or for epilogues
// (DESIGN.md section 4).  Here every wave does both jobs for half the xi: wave w owns couts
// 16 (w & 3) .. +15 and xi rows 3 (w >> 2) .. +2 (18 xi, 72 accumulators, ~230 VGPRs), so two
// waves share each SIMD and one's VALU and waits run beside the other's MFMAs.
//   * Transform: wave w transforms tiles 2w, 2w+1 of the item for the K-step's 16 channels, one
//     channel per lane (lane = column half h, tile, channel): 18 4-byte patch loads (a patch row's
//     16 channels are 64 contiguous bytes), B^T down its 3 columns, 9 values traded with the
//     partner half (v_permlane32_swap), B^T along its 3 rows, 18 ring writes.  The loads of step
//     s + 1 go out at the start of step s; the transform runs in pieces between the MFMA pairs of
//     step s, the two xi halves at different pairs (W4S_P0 / W4S_P1), into the other of 2 ring
//     slots.  One workgroup barrier per K-step.
//   * MFMA: per K-step and xi one ds_read_b128 of V, one 1-KiB load of U (a ring W4S_UR xi ahead),
//     4 MFMAs; xi in pairs.
//   * Epilogue: each wave forms the partial A^T M A of its 3 xi rows for the 16 pixels of its
//     lane's tile, hands its partner the 2 output rows the partner stores (16 KiB of LDS per wave
//     pair), adds the partner's half of its own 2 rows, and applies BN (+ PReLU | + residual).
//   * Layouts: NHWC or channel-blocked x / res / y (W4_BLK_* bits, addresses only).
// Deterministic: each output is one item's own K loop and one fixed two-term sum.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "frhip_kernels.h"

namespace frhip {

namespace {

struct Wino4sParams {
  const float* x;
  const float* u;
  float* y;
  const float* pre_t;
  const float* post_scale;
  const float* post_shift;
  const float* prelu;
  const float* res;
  int B, H, W, Cin, Cout;
  int blk;  // W4_BLK_* bits: x / res / y channel-blocked [B][C/16][H][W][16] instead of NHWC
  int Pr, Pc, NC, TWc, ntiles, mblocks, nblocks, nbg;
};


typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NXI_S = 36;
constexpr int FT_S = 16;
constexpr int KC_S = 16;
constexpr int VSTEP_S = NXI_S * FT_S * KC_S;  // 9,216 floats
constexpr int XCH_S = 8 * 64 * 32;            // partial-output exchange: 8 waves x 64 lanes x 32 floats
constexpr int BIGOFF_S = 0x7F000000;
#ifndef W4S_UR
#define W4S_UR 6
#endif
constexpr int UR_S = W4S_UR;  // xi of U in flight per wave (18 % UR_S == 0)
static_assert(18 % UR_S == 0, "U ring phase must repeat every K-step");
static_assert((2 * VSTEP_S + XCH_S) * 4 <= 160 * 1024, "LDS budget");
// MFMA pair (of 9) after which a wave's transform pieces start: the two waves of a SIMD (xi
// halves 0 and 1) run theirs at different points of the K-step
#ifndef W4S_P0
#define W4S_P0 1
#endif
#ifndef W4S_P1
#define W4S_P1 5
#endif

__device__ __forceinline__ int xcd_remap_s(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_s(const void* ptr, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(ptr);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), (short)0, n,
                                           0x00020000);
}

__device__ __forceinline__ f4 ld4_s(__amdgpu_buffer_rsrc_t r, int off, int soff = 0) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

__device__ __forceinline__ int vslot_s(int l) {
  const int k = l >> 4;
  return l ^ ((k & 1) * 2 + (k >> 1) * 12);
}

__device__ __forceinline__ int canvas_coord_s(int v, int base, int P, int H, bool sep, int& slot) {
  const int y = v - base * P, y1 = y - P;
  const bool in0 = (unsigned)y < (unsigned)H;
  const bool in1 = sep && (unsigned)y1 < (unsigned)H;
  slot = base + (in1 ? 1 : 0);
  return in0 ? y : (in1 ? y1 : -1);
}

__device__ __forceinline__ void bt6_s(const float (&d)[6], float (&t)[6]) {
  const float r = d[4] - d[2], u = d[3] - d[1];
  const float pp = __builtin_fmaf(-4.f, d[2], d[4]), q = __builtin_fmaf(-4.f, d[1], d[3]);
  t[0] = __builtin_fmaf(4.f, d[0] - d[2], r);
  t[1] = pp + q;
  t[2] = pp - q;
  t[3] = __builtin_fmaf(2.f, u, r);
  t[4] = __builtin_fmaf(-2.f, u, r);
  t[5] = __builtin_fmaf(-4.f, u, d[5] - d[3]);
}

__device__ __forceinline__ void at6q_s(const f4 (&m)[6], f4 (&o)[4]) {
  const f4 c2 = {2.f, 2.f, 2.f, 2.f}, c4 = {4.f, 4.f, 4.f, 4.f}, c8 = {8.f, 8.f, 8.f, 8.f};
  const f4 p12 = m[1] + m[2], m12 = m[1] - m[2];
  const f4 p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = __builtin_elementwise_fma(c2, m34, m12);
  o[2] = __builtin_elementwise_fma(c4, p34, p12);
  o[3] = __builtin_elementwise_fma(c8, m34, m12 + m[5]);
}

struct ItemS {
  int mb, nb;
};
__device__ __forceinline__ ItemS item_s(const Wino4sParams& p, int gi) {
  const int NB = p.nblocks, GM = p.nbg;
  const int grp = gi / (GM * NB), rem = gi - grp * GM * NB;
  const int gm = min(GM, p.mblocks - grp * GM);
  ItemS it;
  it.nb = rem / gm;
  it.mb = grp * GM + (rem - it.nb * gm);
  return it;
}

template <bool PRE, int EPI>
__global__ __launch_bounds__(512, 1) void wino4s_kernel(Wino4sParams p) {
  __shared__ __attribute__((aligned(16))) float lds[2 * VSTEP_S + XCH_S];
  float* ring = lds;
  float* xch = lds + 2 * VSTEP_S;
  constexpr bool RES = EPI == EPI_AFFINE_RES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = w & 3, xh = w >> 2;
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout;
  const int KST = Cin / KC_S;
  const int nitems = p.mblocks * p.nblocks;
  const int bid = blockIdx.x, nblk = gridDim.x;
  const int nloc = (nitems - bid + nblk - 1) / nblk;
  if (nloc <= 0) return;
  const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
  auto item_at = [&](int j) { return item_s(p, xcd_remap_s(bid + min(j, nloc - 1) * nblk, nitems)); };

  // ---- transform: tiles 2w, 2w+1 of the item; lane (column half h, tile t, channel ch) holds patch
  // columns 3h .. 3h+2 (6 rows) of channel ch
  const int half = lane >> 5, tt = (lane >> 4) & 1, ch = lane & 15;
  const int ti = 2 * w + tt;
  const __amdgpu_buffer_rsrc_t xr = rsrc_s(p.x, p.B * H * W * Cin * 4);
  // x layout: pixel pitch and per-K-step stride (the image base is the same in both layouts)
  const int xppx = (p.blk & W4_BLK_X) ? 16 : Cin;
  const int xstep = (p.blk & W4_BLK_X) ? H * W * KC_S * 4 : KC_S * 4;
  int roff[6], coff[3];
  auto enter_item = [&](int j) {
    const ItemS it = item_at(j);
    const int T = it.mb * FT_S + ti;
    const int tr = T / p.TWc, tc = T - tr * p.TWc;
    const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      int rs;
      const int y = canvas_coord_s(4 * tr - 1 + e, ir0, p.Pr, H, sep_r, rs);
      const bool in = y >= 0 && rs * p.NC < p.B && T < p.ntiles;
      roff[e] = in ? (rs * p.NC * H * W * Cin + y * W * xppx) * 4 : BIGOFF_S;
    }
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      int cs;
      const int x = canvas_coord_s(4 * tc - 1 + 3 * half + e, ic0, p.Pc, W, sep_c, cs);
      const bool in = x >= 0 && cs < p.NC;
      coff[e] = in ? (cs * H * W * Cin + x * xppx + ch) * 4 : BIGOFF_S;
    }
  };
  float d[6][3];
  float tsh = 0.f;
  auto load = [&](int step) {
    const int soff = __builtin_amdgcn_readfirstlane(step * xstep);
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        d[a][b] = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(xr, (int)((unsigned)roff[a] + (unsigned)coff[b]), soff, 0));
    if constexpr (PRE) tsh = p.pre_t[step * KC_S + ch];
  };
  // ring address of (tile ti, channel ch): fragment lane 16 (ch / 4) + ti, element ch % 4; half h
  // writes transform rows 3h .. 3h+2 (xi from 18 h)
  const int dst_off = vslot_s(16 * (ch >> 2) + ti) * 4 + (ch & 3) + half * 18 * 256;
  // pieces: 0 pre-BN shift, 1-3 column transforms, 4 partner exchange, 5-7 row transforms + writes
  auto piece = [&](int q, float* slot) {
    if (q == 0) {
      if constexpr (PRE)
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) d[a][b] += (roff[a] != BIGOFF_S && coff[b] != BIGOFF_S) ? tsh : 0.f;
    } else if (q < 4) {
      const int b = q - 1;
      float c[6], o[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) c[a] = d[a][b];
      bt6_s(c, o);
#pragma unroll
      for (int a = 0; a < 6; ++a) d[a][b] = o[a];
    } else if (q == 4) {
      // half 0 keeps transform rows 0-2, half 1 rows 3-5: d[k][b] <- row 3h + k of column b,
      // d[3 + k][b] <- row 3h + k of column 3 + b
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(d[k][b]), __float_as_uint(d[3 + k][b]), false,
                                                          false);
          d[k][b] = __uint_as_float(r[0]);
          d[3 + k][b] = __uint_as_float(r[1]);
        }
    } else {
      const int k = q - 5;
      const float row[6] = {d[k][0], d[k][1], d[k][2], d[3 + k][0], d[3 + k][1], d[3 + k][2]};
      float v[6];
      bt6_s(row, v);
      float* dst = slot + dst_off;
#pragma unroll
      for (int c = 0; c < 6; ++c) dst[(6 * k + c) * 256] = v[c];
    }
  };

  // ---- MFMA: couts 16 cb .. +15, xi 18 xh .. +17
  const __amdgpu_buffer_rsrc_t ur = rsrc_s(p.u, NXI_S * Cout * Cin * 4);
  const int NB16 = Cout / 16;
  const int XS = NB16 * KST * 1024;
  const int xb = 18 * xh;
  auto ubase = [&](int j) {
    const ItemS it = item_at(j);
    return xb * XS + (min(it.nb * 4 + cb, NB16 - 1) * KST) * 1024;
  };
  const int lo = lane * 16;
  const float* vrd = ring + vslot_s(lane) * 4 + xb * 256;
  f4 uring[UR_S];
  f4 acc[18];
  auto kstep = [&](auto PS, int g, int lstep, int cur, int nxt) {
    constexpr int pstart = decltype(PS)::value;
    load(lstep);
    __builtin_amdgcn_sched_barrier(0);
    const float* vb = vrd + (g & 1) * VSTEP_S;
    float* nslot = ring + ((g + 1) & 1) * VSTEP_S;
    f4 a0n = *reinterpret_cast<const f4*>(vb), a1n = *reinterpret_cast<const f4*>(vb + 256);
#pragma unroll
    for (int x = 0; x < 18; x += 2) {
      const f4 a0 = a0n, a1 = a1n;
      if (x + 2 < 18) {
        a0n = *reinterpret_cast<const f4*>(vb + (x + 2) * 256);
        a1n = *reinterpret_cast<const f4*>(vb + (x + 3) * 256);
      }
      const f4 u0 = uring[x % UR_S], u1 = uring[(x + 1) % UR_S];
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
        uring[y % UR_S] = y + UR_S < 18 ? ld4_s(ur, lo, (y + UR_S) * XS + cur) : ld4_s(ur, lo, (y + UR_S - 18) * XS + nxt);
      }
      // transform pieces: 8 of them over the pairs from pstart (pairs 0..8), the last pair takes the rest
      const int pr = x / 2;
      if (pr >= pstart) {
        const int q0 = pr - pstart, q1 = pr == 8 ? 8 : q0 + 1;
        for (int q = q0; q < q1 && q < 8; ++q) piece(q, nslot);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  };

  enter_item(0);
  load(0);
  int ub = ubase(0);
#pragma unroll
  for (int r = 0; r < UR_S; ++r) uring[r] = ld4_s(ur, lo, r * XS + ub);
#pragma unroll
  for (int q = 0; q < 8; ++q) piece(q, ring);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t yr = rsrc_s(p.y, p.B * H * W * Cout * 4);
  const __amdgpu_buffer_rsrc_t rr = rsrc_s(p.res, RES ? p.B * H * W * Cout * 4 : 0);
  const int n = lane & 15, rg = lane >> 4;
  for (int j = 0; j < nloc; ++j) {
    const ItemS it = item_at(j);
    const bool live = it.nb * 64 + cb * 16 < Cout;
    const int ub_next = ubase(j + 1);
#pragma unroll
    for (int x = 0; x < 18; ++x) acc[x] = f4{0.f, 0.f, 0.f, 0.f};
    // the two xi halves place their transform pieces at different points of the K-step
    auto run = [&](auto PS) {
      for (int s = 0; s + 1 < KST; ++s) kstep(PS, j * KST + s, s + 1, ub + s * 1024, ub + (s + 1) * 1024);
      enter_item(j + 1);
      kstep(PS, j * KST + KST - 1, 0, ub + (KST - 1) * 1024, ub_next);
    };
    if (xh == 0)
      run(std::integral_constant<int, W4S_P0>{});
    else
      run(std::integral_constant<int, W4S_P1>{});
    ub = ub_next;

    // ---- epilogue: partial A^T M A over this wave's 3 xi rows (a = 3 xh + k) for all 16 pixels
    f4 t[3][4];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const f4 m6[6] = {acc[6 * k], acc[6 * k + 1], acc[6 * k + 2], acc[6 * k + 3], acc[6 * k + 4], acc[6 * k + 5]};
      at6q_s(m6, t[k]);
    }
    // A^T columns: rows 0-2 -> (1,0,0,0), (1,1,1,1), (1,-1,1,-1); rows 3-5 -> (1,2,4,8), (1,-2,4,-8), (0,0,0,1)
    f4 P[4][4];
    const f4 c2 = {2.f, 2.f, 2.f, 2.f}, c4 = {4.f, 4.f, 4.f, 4.f}, c8 = {8.f, 8.f, 8.f, 8.f};
#pragma unroll
    for (int xq = 0; xq < 4; ++xq) {
      if (xh == 0) {
        const f4 s12 = t[1][xq] + t[2][xq], d12 = t[1][xq] - t[2][xq];
        P[0][xq] = t[0][xq] + s12;
        P[1][xq] = d12;
        P[2][xq] = s12;
        P[3][xq] = d12;
      } else {
        const f4 s34 = t[0][xq] + t[1][xq], d34 = t[0][xq] - t[1][xq];
        P[0][xq] = s34;
        P[1][xq] = c2 * d34;
        P[2][xq] = c4 * s34;
        P[3][xq] = __builtin_elementwise_fma(c8, d34, t[2][xq]);
      }
    }
    // xh 0 stores output rows 0-1, xh 1 rows 2-3: hand the partner its two rows
    const int mine = 2 * xh;
    float* xo = xch + (w * 64 + lane) * 4;  // [wave][i][lane][4], i = 0..7
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
      for (int xq = 0; xq < 4; ++xq)
        *reinterpret_cast<f4*>(xo + (r2 * 4 + xq) * 8 * 64 * 4) = xh ? P[r2][xq] : P[2 + r2][xq];
    __syncthreads();
    const float* xi = xch + ((w ^ 4) * 64 + lane) * 4;
    const int T = it.mb * FT_S + n;
    const int tr = T / p.TWc, tc = T - tr * p.TWc;
    const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
    const int cout0 = min(it.nb * 64 + cb * 16, Cout - 16) + 4 * rg;
    const f4 sc = *reinterpret_cast<const f4*>(p.post_scale + cout0);
    const f4 sh = *reinterpret_cast<const f4*>(p.post_shift + cout0);
    f4 al = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_AFFINE_PRELU) al = *reinterpret_cast<const f4*>(p.prelu + cout0);
    // output / residual layouts: pixel pitch and the cout quad's offset inside a pixel row
    const bool yb = (p.blk & W4_BLK_Y) != 0, rb = (p.blk & W4_BLK_RES) != 0;
    const int yppx = yb ? 16 : Cout, rppx = rb ? 16 : Cout;
    const int ycb = yb ? (cout0 >> 4) * H * W * 16 + (cout0 & 15) : cout0;
    const int rcb = rb ? (cout0 >> 4) * H * W * 16 + (cout0 & 15) : cout0;
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      int rs;
      const int yy = canvas_coord_s(4 * tr + mine + r2, ir0, p.Pr, H, sep_r, rs);
      const bool rin = yy >= 0 && rs * p.NC < p.B && T < p.ntiles && live;
      const int ro = rin ? (rs * p.NC * H * W * Cout + yy * W * yppx + ycb) * 4 : BIGOFF_S;
      const int rro = rin ? (rs * p.NC * H * W * Cout + yy * W * rppx + rcb) * 4 : BIGOFF_S;
      f4 rv[4];
      int oo[4];
#pragma unroll
      for (int xq = 0; xq < 4; ++xq) {
        int cs;
        const int xx = canvas_coord_s(4 * tc + xq, ic0, p.Pc, W, sep_c, cs);
        const bool cin_ = xx >= 0 && cs < p.NC;
        oo[xq] = (int)((unsigned)ro + (unsigned)(cin_ ? (cs * H * W * Cout + xx * yppx) * 4 : BIGOFF_S));
        if constexpr (RES)
          rv[xq] = ld4_s(rr, (int)((unsigned)rro + (unsigned)(cin_ ? (cs * H * W * Cout + xx * rppx) * 4 : BIGOFF_S)));
      }
#pragma unroll
      for (int xq = 0; xq < 4; ++xq) {
        const f4 other = *reinterpret_cast<const f4*>(xi + (r2 * 4 + xq) * 8 * 64 * 4);
        f4 v = __builtin_elementwise_fma((xh ? P[2 + r2][xq] : P[r2][xq]) + other, sc, sh);
        if constexpr (EPI == EPI_AFFINE_PRELU)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * al[r];
        if constexpr (RES) v += rv[xq];
        const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[xq], 0, 0);
      }
    }
    // the exchange area is rewritten only after the next item's K-step barriers
  }
}

int w4s_cus() {
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus > 0 ? cus : 256;
}


// canvas and items as conv_winograd4.hip's wino4_canvas (periods H or H + 1, NC images per canvas row)
void w4s_canvas(Wino4sParams& p, bool pre) {
  auto period = [](int h) { return h % 4 == 0 ? h : h + 1; };
  p.Pr = period(p.H);
  p.Pc = period(p.W);
  p.NC = 1;
  while ((p.NC * p.Pc) % 4) ++p.NC;
  if (p.NC > p.B) p.NC = p.B;
  // pre-BN: absent images of a part-filled last canvas row must stay outside every patch window
  if (pre && p.NC > 1 && p.B % p.NC && p.Pr == p.H) p.Pr = p.H + 1;
  const int crow = (p.B + p.NC - 1) / p.NC;
  p.TWc = (p.NC * p.Pc + 3) / 4;
  p.ntiles = ((crow * p.Pr + 3) / 4) * p.TWc;
  p.mblocks = (p.ntiles + FT_S - 1) / FT_S;
  p.nblocks = p.Cout / 64;
  p.nbg = std::max(1, std::min(p.mblocks, std::max(32 / p.nblocks, 8)));
}

Wino4sParams w4s_params(const Wino4Params& q, bool pre) {
  Wino4sParams p{};
  p.x = q.x;
  p.u = q.u;
  p.y = q.y;
  p.pre_t = q.pre_t;
  p.post_scale = q.post_scale;
  p.post_shift = q.post_shift;
  p.prelu = q.prelu;
  p.res = q.res;
  p.B = q.B;
  p.H = q.H;
  p.W = q.W;
  p.Cin = q.Cin;
  p.Cout = q.Cout;
  p.blk = q.blk;
  w4s_canvas(p, pre);
  return p;
}

}  // namespace

bool wino4s_takes(const Wino4Params& q, bool pre, Epi epi, int cus) {
  const bool epi_ok = pre ? (epi == EPI_AFFINE_PRELU && q.pre_t) : (epi == EPI_AFFINE_RES || epi == EPI_AFFINE_PRELU);
  if (!epi_ok || q.Cin % 16 || q.Cin < 16 || q.Cout % 64 || q.B < 1 || q.sk_mode == 2 ||
      (epi == EPI_AFFINE_RES && !q.res) || (long long)q.B * q.H * q.W * q.Cin * 4 >= BIGOFF_S ||
      (long long)q.B * q.H * q.W * q.Cout * 4 >= (1ll << 31) || (long long)NXI_S * q.Cout * q.Cin * 4 >= (1ll << 31))
    return false;
  const Wino4sParams p = w4s_params(q, pre);
  return (long long)p.mblocks * p.nblocks >= cus;  // whole items only: at least one per CU
}

hipError_t launch_wino4s(const Wino4Params& q, bool pre, Epi epi, hipStream_t s) {
  if (!wino4s_takes(q, pre, epi, 1)) return hipErrorInvalidValue;
  const Wino4sParams p = w4s_params(q, pre);
  const int nT = p.mblocks * p.nblocks;
  const dim3 grid(std::min(nT, w4s_cus()));
  if (pre)
    hipLaunchKernelGGL((wino4s_kernel<true, EPI_AFFINE_PRELU>), grid, dim3(512), 0, s, p);
  else if (epi == EPI_AFFINE_RES)
    hipLaunchKernelGGL((wino4s_kernel<false, EPI_AFFINE_RES>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((wino4s_kernel<false, EPI_AFFINE_PRELU>), grid, dim3(512), 0, s, p);
  return hipGetLastError();
}

}  // namespace frhip
