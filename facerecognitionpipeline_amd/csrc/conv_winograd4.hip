// Winograd F(4x4, 3x3) convolution in f32 on gfx950, in two passes:
//
//   1. wino4g_itrans_kernel: every 6x6 input patch of the layer is transformed ONCE,
//      V = B^T d B (with the pre-activation BatchNorm applied to the in-image pixels first),
//      and written to a V buffer laid out in MFMA A-fragment order.
//   2. wino4g_gemm_kernel: per transform element xi (36) the layer is the GEMM
//      M_xi[tile][cout] = sum_cin V_xi[tile][cin] U_xi[cin][cout] on v_mfma_f32_32x32x2_f32,
//      with the output transform A^T M A and BN (+PReLU | +residual) fused in the epilogue.
//
// Replaces the stride-1 3x3 Conv2d of net.BasicBlockIR (res_layer[1] and the stride-1
// res_layer[4], reached through `self.model(batch)`, face_embedder.py:157) and the
// detector's stride-1 3x3 convs.  The one-pass kernel before it (round 1) transformed each
// input patch again for every 32-output-channel block (8x at 256 channels) on VALU that
// competes with the f32 MFMA pipe for the SIMD; here the transform costs one streaming pass
// over the activations and the GEMM kernel is MFMA + loads only.
//
// Transforms (Lavin & Gray 2016, points 0, +-1, +-2, inf):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// Filters U = G g G^T are built once per model in double (launch_wino4_weights, no pre-BN
// folding: the pre-BN is applied to the input in pass 1).
//
// Tiles are cut from a "canvas" of the batch (wino4_canvas): images laid out NC per canvas
// row with a period of P rows / columns.  P = H when 4 | H (every tile inside one image);
// otherwise P = H + 1 -- one zero separator row/column between neighbouring images is all a
// 3x3 pad-1 conv needs, so a 4x4 tile may straddle two images and 14x14 images cost 15^2/14^2
// of the products instead of 16^2/14^2.  Patch pixels on a separator or outside the canvas
// load as 0.
//
// Layouts (floats):
//   V  [mblocks][KST][36 xi][2 q][64 lane][4]   one (tile block, K-step) chunk = 73,728 B;
//      lane = 32 h + m holds channels 8h + 4q .. +3 of tile m of the block (the
//      32x32x2 A-operand fragment: lane (m, h) supplies A[m][k = h])
//   U  [36 xi][Cout/32][KST][2 q][64 lane][4]   lane = 32 h + n: channels 8h + 4q .. of cout n
// with KST = Cin / 16 K-steps of 16 channels; MFMA j (0..7) of a K-step multiplies channel
// 8h + j.
//
// GEMM workgroup: 32 tiles x 64 couts x all 36 xi, 12 waves (768 threads, 3 per SIMD):
// wave w owns transform row a = w % 6 (xi = 6a .. 6a+5) for cout half w / 6, i.e. six
// 32x32 accumulator blocks (96 registers).  The K loop is branch-free streaming: each wave
// loads its A fragments (V) and B fragments (U) straight from L2 / the Infinity Cache in
// fragment order (1 KiB coalesced loads; the other cout half's wave of the same row reads
// the same V lines), three (K-step, xi) slots ahead in a register ring, no LDS, no barrier.
// Owning whole rows lets the epilogue apply the b-direction of A^T M A in registers
// (6 -> 4 per row) before the LDS exchange; the a-direction runs after it, per
// (tile, column, cout), followed by BN / PReLU / residual and the stores.
#include <algorithm>

#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NXI = 36;                  // transform elements
constexpr int WT = 32;                   // 4x4 output tiles per tile block (MFMA M)
constexpr int KC = 16;                   // input channels per K-step
constexpr int CHUNK = NXI * WT * KC;     // floats of one V chunk (18,432)
constexpr int GEMM_THREADS = 768;        // 12 waves: 6 transform rows x 2 cout halves
constexpr int RING = 3;                  // (K-step, xi) slots of operands in flight per wave
constexpr int MROW = 33;                 // epilogue staging row (32 couts + 1)
constexpr int EPI_FLOATS = 24 * WT * MROW;  // [6 a][4 b'][32 tiles][33]
constexpr int BIGOFF = 0x7F000000;       // row/column offset of padding: any sum with it is past the range
static_assert(EPI_FLOATS * 4 <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* ptr, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(ptr);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), (short)0, n,
                                           0x00020000);
}

// 16-byte buffer load: per-lane byte offset `off` + wave-uniform byte offset `soff` (an SGPR)
__device__ __forceinline__ f4 ld4(__amdgpu_buffer_rsrc_t r, int off, int soff = 0) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0);
  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

// Canvas coordinate v (a row or a column) of a tile whose origin lies in image slot `base`:
// returns the in-image coordinate and sets `slot` (base or base + 1), or -1 for padding.
__device__ __forceinline__ int canvas_coord(int v, int base, int P, int H, bool sep, int& slot) {
  const int y = v - base * P, y1 = y - P;
  const bool in0 = (unsigned)y < (unsigned)H;
  const bool in1 = sep && (unsigned)y1 < (unsigned)H;
  slot = base + (in1 ? 1 : 0);
  return in0 ? y : (in1 ? y1 : -1);
}

// 1-D input transform B^T d (6 -> 6) of four channels
__device__ __forceinline__ void bt6(const f4 (&d)[6], f4 (&t)[6]) {
  const f4 s1 = d[3] + d[4], s2 = d[1] + d[2];
  const f4 s3 = d[4] - d[3], s4 = d[1] - d[2];
  const f4 s5 = d[4] - d[2], s6 = d[3] - d[1];
  t[0] = 4.f * d[0] + (-5.f * d[2] + d[4]);
  t[1] = -4.f * s2 + s1;
  t[2] = 4.f * s4 + s3;
  t[3] = 2.f * s6 + s5;
  t[4] = -2.f * s6 + s5;
  t[5] = 4.f * d[1] + (-5.f * d[3] + d[5]);
}

// 1-D output transform A^T m (6 -> 4)
__device__ __forceinline__ void at6(const float (&m)[6], float (&o)[4]) {
  const float p12 = m[1] + m[2], m12 = m[1] - m[2];
  const float p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = m12 + 2.f * m34;
  o[2] = p12 + 4.f * p34;
  o[3] = m12 + 8.f * m34 + m[5];
}

// ---- pass 1: input transform ------------------------------------------------------------
// Block (tile block mb, 32-channel group g): 4 waves x (8 tiles x 8 channel quads).  Each
// thread loads its 6x6 patch as 36 16-byte loads (a wave covers 8 pixels x 128 B = whole
// lines), applies the pre-BN at in-image pixels, transforms and stores 36 float4 of V (per
// (K-step, h, q) group a wave writes 8 tiles x 16 B = one 128-B segment).
template <bool PRE>
__global__ __launch_bounds__(256) void wino4g_itrans_kernel(Wino4Params p) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c4 = lane & 7, m = 8 * wv + (lane >> 3);
  const int mb = blockIdx.x, g = blockIdx.y;
  const int H = p.H, W = p.W, Cin = p.Cin, KST = Cin / KC;
  const int T = mb * WT + m;
  const int tr = T / p.TWc, tc = T - tr * p.TWc;
  const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
  const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
  const int c0 = 32 * g + 4 * c4;
  int roff[6], coff[6];
  bool rin[6], cin[6];
  int rslot[6], cslot[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int y = canvas_coord(4 * tr - 1 + i, ir0, p.Pr, H, sep_r, rslot[i]);
    const int x = canvas_coord(4 * tc - 1 + i, ic0, p.Pc, W, sep_c, cslot[i]);
    rin[i] = y >= 0 && T < p.ntiles;
    cin[i] = x >= 0 && cslot[i] < p.NC;
    roff[i] = rin[i] ? (rslot[i] * p.NC * H + y) * W * Cin * 4 : BIGOFF;
    coff[i] = cin[i] ? ((cslot[i] * H * W + x) * Cin + c0) * 4 : BIGOFF;
  }
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x, p.B * H * W * Cin * 4);
  f4 d[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) d[i][j] = ld4(xr, (int)((unsigned)roff[i] + (unsigned)coff[j]));
  if constexpr (PRE) {
    // BN(x) = x * scale + shift at in-image pixels only: the conv's zero padding (and the
    // canvas separators / the images past B) stay 0, as in BN -> zero-padded Conv2d
    const f4 sc = *reinterpret_cast<const f4*>(p.pre_scale + c0);
    const f4 sh = *reinterpret_cast<const f4*>(p.pre_shift + c0);
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const bool in = rin[i] && cin[j] && (rslot[i] * p.NC + cslot[j]) < p.B;
        const f4 v = d[i][j] * sc + sh;
        d[i][j] = in ? v : f4{0.f, 0.f, 0.f, 0.f};
      }
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {  // columns: d[.][j] <- (B^T d)[.][j]
    f4 c[6], o[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) c[i] = d[i][j];
    bt6(c, o);
#pragma unroll
    for (int i = 0; i < 6; ++i) d[i][j] = o[i];
  }
  const int s = 2 * g + (c4 >> 2), h = (c4 & 3) >> 1, q = c4 & 1;
  float* vbase = p.v + ((size_t)mb * KST + s) * CHUNK + q * 256 + (32 * h + m) * 4;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    f4 v[6];
    bt6(d[a], v);
#pragma unroll
    for (int b = 0; b < 6; ++b) *reinterpret_cast<f4*>(vbase + (6 * a + b) * 512) = v[b];
  }
}

// ---- pass 2: transform-domain GEMM + output transform ----------------------------------
// SPLIT (small grids): workgroup (item, split) runs K-steps [s0, s0 + KS) and writes its raw
// inverse-transformed partial output to slab `split`; wino4g_split_reduce_kernel finishes.
template <int EPI, bool SPLIT>
__global__ __launch_bounds__(GEMM_THREADS, 1) void wino4g_gemm_kernel(Wino4Params p) {
  __shared__ __attribute__((aligned(16))) float lds[EPI_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: operand offsets stay scalar
  const int ra = wid % 6, ch = wid / 6;  // transform row, cout half
  const int NB = p.nblocks;              // 64-cout blocks
  const int nT = p.mblocks * NB;
  const int tt = xcd_remap(blockIdx.x, SPLIT ? nT * p.ksplit : nT);
  const int split = SPLIT ? tt / nT : 0;
  const int t = SPLIT ? tt - split * nT : tt;
  // item t -> (tile block mb, cout block nb): one XCD's contiguous run of items covers GM tile
  // blocks x all NB cout blocks, so the V chunks and U blocks it streams are shared in its L2
  const int GM = p.nbg;
  const int grp = t / (GM * NB), rem = t - grp * GM * NB;
  const int gm = min(GM, p.mblocks - grp * GM);
  const int nb = rem / gm, mb = grp * GM + (rem - (rem / gm) * gm);
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout;
  const int KST = Cin / KC;
  const int s0 = SPLIT ? split * p.ks_per : 0;
  const int KS = SPLIT ? min(p.ks_per, KST - s0) : KST;
  const int cout0 = nb * 64 + ch * 32;
  const bool active = cout0 < Cout;  // Cout % 64 == 32: the last block's second half idles

  floatx16 acc[6];
#pragma unroll
  for (int b = 0; b < 6; ++b)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;

  if (active) {
    const __amdgpu_buffer_rsrc_t vr = uniform_rsrc(p.v + (size_t)mb * KST * CHUNK, KST * CHUNK * 4);
    const __amdgpu_buffer_rsrc_t ur = uniform_rsrc(p.u, NXI * Cout * Cin * 4);
    const int NB32 = Cout / 32, nb32 = cout0 / 32;
    // slot (K-step s, b) = (s, xi = 6 ra + b): the fragment of lane l sits at 16 l bytes (q = 0)
    // and 1 KiB + 16 l (q = 1) of a wave-uniform 2-KiB block
    const int lo = lane * 16;
    f4 va[RING][2], ub[RING][2];
    auto load = [&](int slot, int rs) {  // slot counts (K-step, b) pairs from s0; clamped at the end
      const int s = s0 + min(slot / 6, KS - 1), b = slot % 6;
      const int vo = (s * NXI + 6 * ra + b) * 2048;
      const int uo = (((6 * ra + b) * NB32 + nb32) * KST + s) * 2048;
      va[rs][0] = ld4(vr, lo, vo);
      va[rs][1] = ld4(vr, lo, vo + 1024);
      ub[rs][0] = ld4(ur, lo, uo);
      ub[rs][1] = ld4(ur, lo, uo + 1024);
    };
#pragma unroll
    for (int r = 0; r < RING; ++r) load(r, r);
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int rs = b % RING;  // 6 slots per K-step, RING | 6: the ring phase is static
        const f4 a0 = va[rs][0], a1 = va[rs][1], b0 = ub[rs][0], b1 = ub[rs][1];
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b0.x, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b0.y, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b0.z, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b0.w, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b1.x, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b1.y, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, b1.z, acc[b], 0, 0, 0);
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, b1.w, acc[b], 0, 0, 0);
        load(6 * s + b + RING, rs);
        // keep slot order: without this the scheduler clusters three slots' MFMAs and issues
        // their refills together right before they are consumed (vmcnt(0) every half step)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- epilogue -------------------------------------------------------------------------
  // b-direction of A^T M A in registers: lane (n, h) register r holds (tile 8(r/4) + 4h + r%4,
  // cout n) of all six b of row ra; z[b'] = (A^T m)[b'].  Staged per cout half as
  // lds[a][b'][tile][cout] (row 33: conflict-free), then each thread finishes (tile, b', cout)
  // columns along a and writes 4 output pixels.
  const int ntile_cols = WT * 4 * 32;  // (tile, b', cout) columns of one cout half
  const __amdgpu_buffer_rsrc_t yr =
      uniform_rsrc(SPLIT ? p.part + split * p.part_stride : p.y, p.B * H * W * Cout * 4);
  constexpr bool RES = !SPLIT && (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU);
  const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.res, RES ? p.B * H * W * Cout * 4 : 0);
  const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();  // the previous half's columns are read
    if (ch == pass && active) {
      const int n = lane & 31, h = lane >> 5;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float m6[6] = {acc[0][r], acc[1][r], acc[2][r], acc[3][r], acc[4][r], acc[5][r]};
        float z[4];
        at6(m6, z);
        const int tile = 8 * (r >> 2) + 4 * h + (r & 3);
#pragma unroll
        for (int bq = 0; bq < 4; ++bq) lds[((ra * 4 + bq) * WT + tile) * MROW + n] = z[bq];
      }
    }
    __syncthreads();
    if (nb * 64 + pass * 32 >= Cout) continue;  // uniform: this half has no couts
    const int cout = nb * 64 + pass * 32 + (tid & 31);
    const float sc = SPLIT ? 1.f : p.post_scale[cout], sh = SPLIT ? 0.f : p.post_shift[cout];
    float al = 0.f;
    if constexpr (!SPLIT && (EPI == EPI_AFFINE_PRELU || EPI == EPI_AFFINE_RES_PRELU)) al = p.prelu[cout];
    for (int col = tid; col < ntile_cols; col += GEMM_THREADS) {
      const int tb = col >> 5;  // (tile, b') pair
      const int tile = tb >> 2, bq = tb & 3;
      float m6[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) m6[a] = lds[((a * 4 + bq) * WT + tile) * MROW + (col & 31)];
      float o[4];
      at6(m6, o);
      const int T = mb * WT + tile;
      const int tr = T / p.TWc, tc = T - tr * p.TWc;
      const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
      int cs;
      const int xx = canvas_coord(4 * tc + bq, ic0, p.Pc, W, sep_c, cs);
      const int ocol = (xx >= 0 && cs < p.NC) ? cs * H * W + xx : -1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int rsl;
        const int y = canvas_coord(4 * tr + r, ir0, p.Pr, H, sep_r, rsl);
        const int nimg = rsl * p.NC;
        const int orow = (y >= 0 && nimg < p.B && T < p.ntiles) ? (nimg * H + y) * W : -1;
        const int pix = orow + ocol;
        const bool ok = orow >= 0 && ocol >= 0 && pix < p.B * H * W;
        const int oo = ok ? (pix * Cout + cout) * 4 : BIGOFF;  // BIGOFF: the store is dropped
        float v = o[r];
        if constexpr (!SPLIT) {
          v = v * sc + sh;
          if constexpr (EPI == EPI_AFFINE_PRELU) v = v > 0.f ? v : v * al;
          if constexpr (RES) {
            v += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, oo, 0, 0));
            if constexpr (EPI == EPI_AFFINE_RES_PRELU) v = v > 0.f ? v : v * al;
          }
        }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), yr, oo, 0, 0);
      }
    }
  }
}

// Split-K finish: y = epilogue(sum over splits of the raw partial outputs), summed in split
// order (deterministic).  Pixels outside the images were never stored by any split, and none
// of them is read here (n4 covers exactly the B*H*W*Cout outputs).
template <int EPI>
__global__ void wino4g_split_reduce_kernel(const float* __restrict__ part, int S, long long stride, long long n4,
                                           int Cout, const float* __restrict__ sc, const float* __restrict__ sh,
                                           const float* __restrict__ prelu, const float* __restrict__ res,
                                           float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 w[16];
#pragma unroll
  for (int s = 0; s < 16; ++s)
    if (s < S) w[s] = reinterpret_cast<const float4*>(part + s * stride)[i];
  float4 v = w[0];
#pragma unroll
  for (int s = 1; s < 16; ++s)
    if (s < S) {
      v.x += w[s].x;
      v.y += w[s].y;
      v.z += w[s].z;
      v.w += w[s].w;
    }
  for (int s = 16; s < S; ++s) {
    const float4 u = reinterpret_cast<const float4*>(part + s * stride)[i];
    v.x += u.x;
    v.y += u.y;
    v.z += u.z;
    v.w += u.w;
  }
  const int c0 = (int)((i * 4) % Cout);
  float o[4] = {v.x, v.y, v.z, v.w};
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) r = reinterpret_cast<const float4*>(res)[i];
  const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + j;
    float t = o[j] * sc[c] + sh[c];
    if constexpr (EPI == EPI_AFFINE_PRELU) t = t > 0.f ? t : t * prelu[c];
    if constexpr (EPI == EPI_AFFINE_RES) t += rv[j];
    if constexpr (EPI == EPI_AFFINE_RES_PRELU) {
      t += rv[j];
      t = t > 0.f ? t : t * prelu[c];
    }
    o[j] = t;
  }
  reinterpret_cast<float4*>(y)[i] = make_float4(o[0], o[1], o[2], o[3]);
}

// G g G^T of every (cout, cin) filter, in double then rounded once to f32, scattered into
// the fragment order wino4_kernel reads: [xi][Cout/32][Cin/16][q][lane][4] with
// lane = 32*(c/8) + cout%32, q = (c%8)/4, element = c%4 for c = cin%16.
__global__ void wino4_weight_kernel(const float* __restrict__ w, float* __restrict__ u, int Cout, int Cin) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Cout * Cin) return;
  const int o = idx / Cin, i = idx - o * Cin;
  const double G[6][3] = {{0.25, 0.0, 0.0},
                          {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                          {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                          {1.0 / 24, 1.0 / 12, 1.0 / 6},
                          {1.0 / 24, -1.0 / 12, 1.0 / 6},
                          {0.0, 0.0, 1.0}};
  double g[3][3];
#pragma unroll
  for (int y = 0; y < 3; ++y)
#pragma unroll
    for (int x = 0; x < 3; ++x) g[y][x] = w[((long long)(o * 3 + y) * 3 + x) * Cin + i];
  double tg[6][3];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int x = 0; x < 3; ++x) tg[a][x] = G[a][0] * g[0][x] + G[a][1] * g[1][x] + G[a][2] * g[2][x];
  const int NB32 = Cout / 32, KS = Cin / KC;
  const int nb32 = o >> 5, n = o & 31;
  const int s = i / KC, c = i % KC;
  const int ln = 32 * (c >> 3) + n, q = (c & 7) >> 2, e = c & 3;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const double v = tg[a][0] * G[b][0] + tg[a][1] * G[b][1] + tg[a][2] * G[b][2];
      const int xi = 6 * a + b;
      u[((((long long)(xi * NB32 + nb32) * KS + s) * 2 + q) * 64 + ln) * 4 + e] = (float)v;
    }
}

}  // namespace

size_t wino4_weight_floats(int Cout, int Cin) { return (size_t)NXI * Cout * Cin; }

hipError_t launch_wino4_weights(const float* w, float* u, int Cout, int Cin, hipStream_t s) {
  if (Cout % 32 || Cin % KC) return hipErrorInvalidValue;
  const int n = Cout * Cin;
  hipLaunchKernelGGL(wino4_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, u, Cout, Cin);
  return hipGetLastError();
}

// Canvas of a layer: P = H when 4 | H (tiles never straddle images), else P = H + 1 with NC
// images per canvas row chosen so that the canvas width NC*P is a multiple of 4 (14 -> 4 x 15).
void wino4_canvas(Wino4Params& p) {
  auto period = [](int h) { return h % 4 == 0 ? h : h + 1; };
  p.Pr = period(p.H);
  p.Pc = period(p.W);
  p.NC = 1;
  if (p.Pc % 4) {
    p.NC = (p.Pc % 2) ? 4 : 2;
    if (p.NC > p.B) p.NC = p.B;
  }
  const int crow = (p.B + p.NC - 1) / p.NC;  // canvas rows of images
  p.TWc = (p.NC * p.Pc + 3) / 4;
  const int TRc = (crow * p.Pr + 3) / 4;
  p.ntiles = TRc * p.TWc;
}

bool wino4g_supported(int Cin, int Cout, int kh, int kw, int stride, int pad) {
  return kh == 3 && kw == 3 && stride == 1 && pad == 1 && Cin % 32 == 0 && Cin >= 32 && Cout % 32 == 0 && Cout >= 32;
}

size_t wino4g_v_floats(int B, int H, int W, int Cin) {
  Wino4Params p{};
  p.B = B;
  p.H = H;
  p.W = W;
  wino4_canvas(p);
  const size_t mblocks = (p.ntiles + WT - 1) / WT;
  return mblocks * (size_t)(Cin / KC) * CHUNK;
}

hipError_t wino4g_prepare(Wino4Params& p) {
  if (!wino4g_supported(p.Cin, p.Cout, 3, 3, 1, 1) || p.B < 1 || p.H < 1 || p.W < 1 || !p.v ||
      (long long)p.B * p.H * p.W * p.Cin * 4 >= BIGOFF || (long long)p.B * p.H * p.W * p.Cout * 4 >= (1ll << 31) ||
      (long long)NXI * p.Cout * p.Cin * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  wino4_canvas(p);
  p.mblocks = (p.ntiles + WT - 1) / WT;
  if ((size_t)p.mblocks * (p.Cin / KC) * CHUNK > (size_t)p.v_floats) return hipErrorInvalidValue;
  p.nblocks = (p.Cout + 63) / 64;
  p.nbg = std::max(1, std::min(p.mblocks, 32 / p.nblocks));  // tile blocks per XCD group (32 items)
  // split-K when the grid leaves most CUs idle (serving batches): as many splits as fit one
  // round of 256 workgroups, bounded by the K-steps and the partial-output workspace
  const int KST = p.Cin / KC;
  const int nT = p.mblocks * p.nblocks;
  const long long elems = (long long)p.B * p.H * p.W * p.Cout;
  const bool aligned = ((reinterpret_cast<uintptr_t>(p.y) | reinterpret_cast<uintptr_t>(p.res) |
                         reinterpret_cast<uintptr_t>(p.part)) & 15) == 0;
  int S = 1;
  if (p.part && aligned && nT <= 128 && KST > 1) {
    S = std::min(KST, 256 / nT);
    S = (int)std::min<long long>(S, std::min<long long>(p.part_floats, (1ll << 29) - 1) / elems);
    if (S > 1) {
      p.ks_per = (KST + S - 1) / S;
      S = (KST + p.ks_per - 1) / p.ks_per;
    }
  }
  p.ksplit = S > 1 ? S : 1;
  p.part_stride = elems;
  return hipSuccess;
}

hipError_t launch_wino4g_transform(const Wino4Params& p, bool pre, hipStream_t s) {
  if (pre && (!p.pre_scale || !p.pre_shift)) return hipErrorInvalidValue;
  const dim3 tgrid(p.mblocks, p.Cin / 32);
  if (pre)
    hipLaunchKernelGGL(wino4g_itrans_kernel<true>, tgrid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(wino4g_itrans_kernel<false>, tgrid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_wino4g_gemm(const Wino4Params& p, Epi epi, hipStream_t s) {
  const int nT = p.mblocks * p.nblocks;
  const bool split = p.ksplit > 1;
  const dim3 grid(nT * p.ksplit), block(GEMM_THREADS);
#define FR_W4G_CASE(EPI_)                                                                                  \
  if (epi == EPI_) {                                                                                       \
    if (split)                                                                                             \
      hipLaunchKernelGGL((wino4g_gemm_kernel<EPI_, true>), grid, block, 0, s, p);                          \
    else                                                                                                   \
      hipLaunchKernelGGL((wino4g_gemm_kernel<EPI_, false>), grid, block, 0, s, p);                         \
    if (split) {                                                                                           \
      const long long n4 = p.part_stride / 4;                                                              \
      hipLaunchKernelGGL((wino4g_split_reduce_kernel<EPI_>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), \
                         0, s, p.part, p.ksplit, p.part_stride, n4, p.Cout, p.post_scale, p.post_shift,      \
                         p.prelu, p.res, p.y);                                                              \
    }                                                                                                      \
    return hipGetLastError();                                                                              \
  }
  FR_W4G_CASE(EPI_AFFINE_PRELU)      // IR conv1: (pre-BN in pass 1), BN, PReLU; SCRFD conv + BN + ReLU
  FR_W4G_CASE(EPI_AFFINE_RES)        // IR conv2: BN + identity shortcut
  FR_W4G_CASE(EPI_AFFINE)            // SCRFD conv + BN / bias
  FR_W4G_CASE(EPI_AFFINE_RES_PRELU)  // SCRFD BasicBlock conv2 + BN + add + ReLU
#undef FR_W4G_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_wino4g(const Wino4Params& p0, bool pre, Epi epi, hipStream_t s) {
  Wino4Params p = p0;
  hipError_t e = wino4g_prepare(p);
  if (e == hipSuccess) e = launch_wino4g_transform(p, pre, s);
  if (e == hipSuccess) e = launch_wino4g_gemm(p, epi, s);
  return e;
}

}  // namespace frhip
