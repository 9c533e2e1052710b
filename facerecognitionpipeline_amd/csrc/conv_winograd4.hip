// Winograd F(4x4, 3x3) convolution in f32 on gfx950 (v_mfma_f32_16x16x4_f32), one fused,
// persistent kernel per layer.
//
// Replaces the stride-1 3x3 Conv2d of net.BasicBlockIR (res_layer[1] and the stride-1
// res_layer[4], reached through `self.model(batch)`, face_embedder.py:157) and the
// detector's stride-1 3x3 convs, with the pre-BN / post-BN / PReLU / residual epilogues fused.
// Per 4x4 output tile and (cin, cout) pair the algorithm does 36 products instead of 144:
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A     d: 6x6 input patch, g: 3x3 filter
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// (Lavin & Gray 2016, points 0, +-1, +-2, inf).  Filters U = G g G^T are built once per model
// in double (launch_wino4_weights).  Per transform element xi = 6a + b the layer is the GEMM
//   M_xi[tile][cout] = sum_cin V_xi[tile][cin] U_xi[cin][cout],  V = B^T d B.
//
// Work item = 16 tiles x 64 couts x all 36 xi; a workgroup (512 threads) is persistent and
// streams its items' K-steps (16 input channels each) through a 4-deep LDS ring of V:
//   * 4 MFMA waves, one per SIMD: wave w owns couts 16w .. 16w+15 of the item for ALL 36 xi
//     (36 16x16 accumulators, 144 registers).  Per K-step and xi: one ds_read_b128 of V (the B
//     operand), one 1-KiB coalesced load of U in fragment order straight from L2 (the A
//     operand, held in a register ring 12 xi ahead, 9 for the residual epilogues whose
//     registers it needs), 4 MFMAs; xi go in pairs so two accumulation chains interleave.
//     Because U is the A operand, a lane's accumulators hold 4 consecutive couts of one tile
//     for every xi: the output transform A^T M A is lane-local (no LDS exchange, no barrier in
//     the epilogue) and each output pixel is one 16-byte store.
//   * 4 transform waves, one per SIMD: every K-step, transform wave t handles tiles 4t..4t+3 of
//     the item for the step's 16 channels.  A lane holds HALF a patch of two channels: 3
//     columns x 6 rows as 18 8-byte buffer loads from per-item precomputed offsets, issued two
//     K-steps ahead into three rotating register buffers (padding reads 0 through the buffer
//     range check).  It adds the folded pre-activation BN shift (scale folded into U) at
//     in-image pixels, applies B^T down its 3 columns, trades 9 values with its partner lane
//     (v_permlane32_swap: one half keeps patch rows 0-2, the other rows 3-5), applies B^T
//     along its 3 rows and writes them into the ring (18 ds_write_b64).  Each SIMD thus
//     carries a quarter of the transform every step, beside its MFMA wave.
//   * No workgroup barrier per K-step: each wave publishes its progress in an LDS counter
//     (transform wave t: K-steps written; MFMA wave w: K-steps read).  An MFMA wave reads step
//     g once all four transform waves have written it; a transform wave writes step g into
//     slot g % NBUF once all four MFMA waves have read step g - NBUF.  The transform waves may
//     thus run up to NBUF - 1 steps ahead and keep working through an MFMA wave's epilogue.
//     They also leave each item's output geometry in LDS for the epilogue.
// Compared with one 32-output-channel block per workgroup and the transform redone for each
// (round 1), each patch is transformed Cout/64 times instead of Cout/32, and the epilogue
// needs neither LDS staging nor barriers.
//
// Tiles are cut from a "canvas" of the batch (wino4_canvas): images laid out NC per canvas
// row with a period of P rows / columns.  P = H when 4 | H (every tile inside one image);
// otherwise P = H + 1 -- one zero separator row/column between neighbouring images is all a
// 3x3 pad-1 conv needs, so a 4x4 tile may straddle two images and 14x14 images cost 15^2/14^2
// of the products instead of 16^2/14^2.  Patch pixels on a separator or outside the canvas
// load as 0.
//
// Fragment layouts (v_mfma_f32_16x16x4_f32: A[l&15][k=l>>4], B[k=l>>4][l&15], C/D row
// (l>>4)*4 + reg, column l&15).  MFMA m (0..3) of a K-step consumes channel 4k + m, so a lane
// reads the 4 consecutive channels 4k..4k+3 of its tile (V) or of its cout (U) as one float4:
//   V ring slot (one K-step): [36 xi][64 lane = 16 k + tile, as vslot()][4]  (36,864 B)
// U is the MFMA's A operand (rows = couts) and V the B operand (columns = tiles), so the
// accumulator of lane (tile l&15, row group l>>4) holds 4 consecutive couts of one tile.
//   U: [36 xi][Cout/16][Cin/16][64 lane = 16 k + cout][4]
#include <algorithm>
#include <type_traits>
#include <cmath>

#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int NXI = 36;              // transform elements
constexpr int FT = 16;               // 4x4 output tiles per item (MFMA M)
constexpr int FN = 64;               // output channels per item: 4 MFMA waves x 16
constexpr int KC = 16;               // input channels per K-step
constexpr int NBUF = 4;              // LDS ring of transformed K-steps
constexpr int VSTEP = NXI * FT * KC; // floats of one ring slot (9,216)
// xi-slots of U in flight per MFMA wave (36 % URING == 0): 12 where the registers allow (no
// residual in the epilogue: stage-3 conv1 244 -> 239 us, stage-1 263 -> 259), 9 for residual
// epilogues (12 spills ~13 VGPRs there)
template <int EPI>
constexpr int uring_depth() {
  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 9 : 12;
}
constexpr int CPOL_SC1 = 16;         // buffer-store cache policy bit sc1 (write-through to memory)
constexpr int BIGOFF = 0x7F000000;   // row/column offset of padding: any sum with it is past the range
// output-geometry tables of the items in flight: the transform waves' load stream runs at most
// NBUF + 2 K-steps (so items) ahead of the MFMA waves' consumption
constexpr int NGEO = 8;
static_assert(NGEO > NBUF + 2, "geometry table overwritten while an epilogue may still read it");
// output geometry per tile: 4 rows (image-row base, y * W) and 4 columns (image base, x), so the
// epilogue can address the output and the residual in either layout (NHWC or channel-blocked)
constexpr int GEOW = 16;
static_assert((NBUF * VSTEP + NGEO * FT * GEOW + 8) * 4 <= 160 * 1024, "LDS budget");
static_assert(NXI % uring_depth<EPI_AFFINE_RES>() == 0 && NXI % uring_depth<EPI_AFFINE>() == 0,
              "U ring phase must repeat every K-step");

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

// 16-byte slot of fragment lane l = 16 k + i (k: channel quad, i: tile) in a ring plane:
// i XOR c(k), c = 0, 2, 12, 14.  ds_read_b128 serves a wave in four 16-lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) over 64 banks: c(k) keeps bits 3 and 2 of i
// equal-or-opposite as they were, so each group still reads 16 distinct slot columns.
// ds_write_b64 serves 16 contiguous lanes at a time over 32 banks: a transform wave's group is
// 2 tiles x 4 channel quads x 2 channel pairs, and c(k) gives the 4 quads distinct bits 1-2 of
// the slot, so its 32 dwords hit 32 banks (i XOR 4k, the previous map, left 2-way conflicts on
// both sides: SQ_LDS_BANK_CONFLICT ~10% of the kernel's cycles).
__device__ __forceinline__ int vslot(int l) {
  const int k = l >> 4;
  return l ^ ((k & 1) * 2 + (k >> 1) * 12);
}

// Ring hand-off between the two wave roles, one LDS counter per wave instead of a workgroup
// barrier per K-step: transform wave t publishes rdy[t] = the number of K-steps it has written,
// MFMA wave w publishes fre[w] = the number of K-steps it has finished reading.  A consumer
// waits for the minimum of the four counters it depends on.  (With one s_barrier per K-step the
// slowest of the 8 waves gated every step: measured at stage 3, ~14% of every wave's time went
// to waiting at that barrier, and an MFMA wave's epilogue held the transform waves too.)
// Single writer per counter: a plain ds_write after the wave's earlier LDS operations have
// completed (LDS serves a wave's operations in order); readers poll with volatile reads.
typedef __attribute__((address_space(3))) int lds_int;  // LDS pointers: ds_* instructions, not flat_*
template <int N>
__device__ __forceinline__ int lds_min(const int* c) {
  const volatile lds_int* v = (const volatile lds_int*)c;
  int m;
  if constexpr (N == 4)
    m = min(min(v[0], v[1]), min(v[2], v[3]));
  else if constexpr (N == 2)
    m = min(v[0], v[1]);
  else
    m = min(min(min(v[0], v[1]), min(v[2], v[3])), min(v[4], v[5]));
  return __builtin_amdgcn_readfirstlane(m);
}

// Wait until min(c[0..N-1]) >= need; returns the value seen.  The spin is bounded (poll_max
// polls, 2^16 = a few ms by default): a lost hand-off cannot hang the GPU.  An expired wait
// returns the value seen with W4_EXPIRED set: the caller's counter copy then exceeds every later
// `need`, so the wave waits no more, carries on (every global access of the kernel is
// range-checked: wrong data, never a fault) and reports the bit when it leaves the kernel
// (w4_report_handoff).  Folding the flag into the counter copy keeps the hot loop free of a
// store and of a register of its own (a separate flag cost the conv2 kernel 2 spilled VGPRs).
constexpr int W4_EXPIRED = 1 << 30;
template <int N = 4>
__device__ __forceinline__ int lds_wait_min(const int* c, int need, int poll_max) {
  int seen = lds_min<N>(c);
  for (int it = 0; seen < need && it < poll_max; ++it) {
    __builtin_amdgcn_s_sleep(1);
    seen = lds_min<N>(c);
  }
  asm volatile("" ::: "memory");
  return seen < need ? (seen | W4_EXPIRED) : seen;
}
// FR_DEVERR_W4_HANDOFF into the launch's error word (host-pinned, read by the runtime at its sync
// points, which then fail the call with FR_ERR_HIP): a vector store of a constant from every lane
// (idempotent, no atomic needed), system scope so the host sees it once the launch has completed
__device__ __forceinline__ void w4_report_handoff(int seen, int* err) {
  if (__builtin_expect((seen & W4_EXPIRED) != 0, 0) && err)
    __hip_atomic_store(err, FR_DEVERR_W4_HANDOFF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Publish `n` in this wave's counter once its earlier LDS operations have completed.
__device__ __forceinline__ void lds_publish(int* c, int lane, int n) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) *(volatile lds_int*)c = n;
  asm volatile("" ::: "memory");
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

// 1-D input transform B^T d (6 -> 6), 12 ops:
//   t0 = 4 d0 - 5 d2 + d4 = 4 (d0 - d2) + r        r = d4 - d2,  u = d3 - d1
//   t1 = -4 (d1 + d2) + d3 + d4 = p + q            p = d4 - 4 d2, q = d3 - 4 d1
//   t2 = 4 (d1 - d2) - d3 + d4 = p - q
//   t3 = 2 (d3 - d1) + d4 - d2 = r + 2u,  t4 = r - 2u
//   t5 = 4 d1 - 5 d3 + d5 = (d5 - d3) - 4u
__device__ __forceinline__ void bt6(const float (&d)[6], float (&t)[6]) {
  const float r = d[4] - d[2], u = d[3] - d[1];
  const float pp = __builtin_fmaf(-4.f, d[2], d[4]), q = __builtin_fmaf(-4.f, d[1], d[3]);
  t[0] = __builtin_fmaf(4.f, d[0] - d[2], r);
  t[1] = pp + q;
  t[2] = pp - q;
  t[3] = __builtin_fmaf(2.f, u, r);
  t[4] = __builtin_fmaf(-2.f, u, r);
  t[5] = __builtin_fmaf(-4.f, u, d[5] - d[3]);
}

// the same on two channels (packed f32)
__device__ __forceinline__ void bt6v(const f2 (&d)[6], f2 (&t)[6]) {
  const f2 c4 = {4.f, 4.f}, m4 = {-4.f, -4.f}, c2 = {2.f, 2.f}, m2 = {-2.f, -2.f};
  const f2 r = d[4] - d[2], u = d[3] - d[1];
  const f2 pp = __builtin_elementwise_fma(m4, d[2], d[4]), q = __builtin_elementwise_fma(m4, d[1], d[3]);
  t[0] = __builtin_elementwise_fma(c4, d[0] - d[2], r);
  t[1] = pp + q;
  t[2] = pp - q;
  t[3] = __builtin_elementwise_fma(c2, u, r);
  t[4] = __builtin_elementwise_fma(m2, u, r);
  t[5] = __builtin_elementwise_fma(m4, u, d[5] - d[3]);
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

// the same on two couts (packed f32)
__device__ __forceinline__ void at6v(const f2 (&m)[6], f2 (&o)[4]) {
  const f2 c2 = {2.f, 2.f}, c4 = {4.f, 4.f}, c8 = {8.f, 8.f};
  const f2 p12 = m[1] + m[2], m12 = m[1] - m[2];
  const f2 p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = __builtin_elementwise_fma(c2, m34, m12);
  o[2] = __builtin_elementwise_fma(c4, p34, p12);
  o[3] = __builtin_elementwise_fma(c8, m34, m12 + m[5]);
}

// the same on four couts (two packed f32 halves; per element the operations of at6 / at6v)
__device__ __forceinline__ void at6q(const f4 (&m)[6], f4 (&o)[4]) {
  const f4 c2 = {2.f, 2.f, 2.f, 2.f}, c4 = {4.f, 4.f, 4.f, 4.f}, c8 = {8.f, 8.f, 8.f, 8.f};
  const f4 p12 = m[1] + m[2], m12 = m[1] - m[2];
  const f4 p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = __builtin_elementwise_fma(c2, m34, m12);
  o[2] = __builtin_elementwise_fma(c4, p34, p12);
  o[3] = __builtin_elementwise_fma(c8, m34, m12 + m[5]);
}

// item index -> (tile block mb, cout block nb, K split): one XCD's contiguous run of items
// covers GM tile blocks x all cout blocks, so the patches and U blocks it streams are shared
// in its L2
struct Item {
  int mb, nb;  // tile block, cout block
  int split;   // K part (split-K launches)
  int li;      // item index within the launch's item range
};
// global item index gi (0 .. mblocks * nblocks - 1) -> (tile block, cout block)
__device__ __forceinline__ Item item_of(const Wino4Params& p, int gi) {
  const int NB = p.nblocks;
  Item it;
  const int GM = p.nbg;
  const int grp = gi / (GM * NB), rem = gi - grp * GM * NB;
  const int gm = min(GM, p.mblocks - grp * GM);
  it.nb = rem / gm;
  it.mb = grp * GM + (rem - it.nb * gm);
  it.split = 0;
  it.li = 0;
  return it;
}

// A launch covers the items [item0, item0 + nitem) of the layer's item order.
// MODE: 0 = whole items round-robin over the persistent grid; 1 = split-K (every item's K loop
// cut into ksplit parts, raw partial outputs into compact slots [item][part][16 tiles]
// [16 pixels][64 couts], summed in part order by wino4_part_fixup_kernel: small grids).
// (Round 4's stream-K tail and round 4's chained serving layers, both measured slower or neutral,
// are kept outside the library: tools/w4_archive/conv_winograd4_streamk_chain.hip.)
// The kernel body of wino4_kernel (bid, nblk = blockIdx.x, gridDim.x); ring: the workgroup's LDS
// (W4_LDS_FLOATS).
constexpr int W4_LDS_FLOATS = NBUF * VSTEP + std::max(NGEO * FT, 6 * 2 * FT) * GEOW + 8;  // (tall items: 6 x 32 tiles)
constexpr int W4_WIDE = 1, W4_TALL = 2;  // item shapes (wino4_body's VAR)
// RMIX: the residual's layout differs from the output's, in an instance of its own (its offsets are
// computed on their own: more live registers in the epilogue): 1 = residual NHWC, output
// channel-blocked; 2 = residual channel-blocked, output NHWC.  0: p.blk's y and res layouts are the
// same, and the residual is addressed with the output's offsets.
// VAR: the item shape.  0 (the default): 16 tiles x 64 couts, four MFMA waves of 16 couts and four
// transform waves of 4 tiles each.  Whole items without pre-BN only:
//   W4_WIDE (wino4w_kernel): 16 tiles x 96 couts for layers of 65..96 output channels (the
//     detector's 80 / 88 -> 96): six MFMA waves (two each on SIMDs 0 and 1) and two transform waves
//     of 8 tiles each (two passes of 4).  One item per 16 tiles instead of two with most of the
//     second's waves idle, each transforming the same patches.
//   W4_TALL (wino4t_kernel): 32 tiles x 32 couts for layers of at most 32 output channels (the
//     detector's stem conv and head outputs): MFMA wave w takes couts 16 (w & 1) of tile half w >> 1,
//     so all four MFMA waves do useful products (a 64-cout item leaves two of them on clamped
//     weights); four transform waves of 8 tiles (two passes of 4).  A ring slot holds 32 tiles
//     (two 16-tile planes), two slots in the LDS of four.
template <bool PRE, int EPI, int MODE, int RMIX = 0, int VAR = 0>
__device__ __forceinline__ void wino4_body(const Wino4Params& p, float* ring, const int bid, const int nblk) {
  constexpr bool SPLIT = MODE == 1;
  constexpr int NMW = VAR == W4_WIDE ? 6 : 4;             // MFMA waves
  constexpr int NTW = 8 - NMW;                            // transform waves
  constexpr int FTT = VAR == W4_TALL ? 2 * FT : FT;       // tiles per item
  constexpr int FNW = VAR == W4_TALL ? 32 : 16 * NMW;     // output channels per item
  constexpr int NBT = VAR == W4_TALL ? NBUF / 2 : NBUF;   // ring slots
  constexpr int SLOTF = (FTT / FT) * VSTEP;               // floats per ring slot
  constexpr int NGT = VAR == W4_TALL ? 6 : NGEO;          // geometry tables
  static_assert(NGT > NBT + 2 && (NBT * SLOTF + NGT * FTT * GEOW + 8) * 4 <= 160 * 1024, "LDS layout");
  static_assert(VAR == 0 || (!PRE && MODE == 0 && RMIX == 0), "wide / tall items: whole items, no pre-BN");
  __builtin_assume(bid >= 0 && bid < nblk && nblk <= 65535);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout;
  const int KST = Cin / KC;                       // K-steps of the whole reduction
  const int KS = SPLIT ? p.ks_per : KST;          // stream steps per item
  const int nitems = p.nitem * p.ksplit;
  // this workgroup's items are bid, bid + nblk, ... of the XCD-remapped order (item_at(j), j local)
  const int nloc = (nitems - bid + nblk - 1) / nblk;
  const int t_last = nloc - 1;  // last item
  auto item_at = [&](int j) {
    const int t = xcd_remap(bid + j * nblk, nitems);
    const int sp = t / p.nitem, li = t - sp * p.nitem;
    Item it = item_of(p, p.item0 + li);
    it.split = sp;
    it.li = li;
    return it;
  };
  // K-steps item `it` really has (split-K: the last split may be short; its stream is padded
  // with steps whose patches load as zeros, so every item is KS stream steps long)
  auto steps_of = [&](const Item& it) { return SPLIT ? min(KS, KST - it.split * KS) : KST; };
  const int G = nloc * KS;  // K-steps in this workgroup's stream

  int* const geo = reinterpret_cast<int*>(ring + NBT * SLOTF);   // [NGT items][FTT tiles][GEOW]
  int* const rdy = geo + NGT * FTT * GEOW;                        // [NTW] K-steps written, per transform wave
  int* const fre = rdy + NTW;                                     // [NMW] K-steps read, per MFMA wave
  if (tid < 8) rdy[tid] = 0;
  __syncthreads();  // the kernel's only workgroup barrier
  if (G <= 0) return;
  if constexpr (VAR != 0) {
    if (wid >= NMW) {
      // ---- transform waves of wide / tall items: wave t transforms tiles 8t .. 8t+7 of every
      // K-step in two passes of four (q = 0, 1), each pass the lane mapping, loads, transform and
      // ring writes of the four-wave form below (no pre-BN, whole items) into the slot's 16-tile
      // plane of its tiles; the patches of step g + 1 are loaded while step g is transformed
      const int t = wid - NMW;
      const int half = lane >> 5, ii = (lane >> 3) & 3, pr = lane & 7;
      const int ch = 2 * pr;
      const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x, p.B * H * W * Cin * 4);
      const bool xblk = (p.blk & W4_BLK_X) != 0;
      const int xppx = xblk ? KC : Cin;
      const int xstep = xblk ? H * W * KC * 4 : KC * 4;
      const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
      int poff[2][6][3];
      int lj = 0, ls = 0;
      auto enter_item = [&](int j) {
        const Item it = item_at(min(j, t_last));
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int i = 8 * t + 4 * q + ii;
          const int T = it.mb * FTT + i;
          const int tr = T / p.TWc, tc = T - tr * p.TWc;
          const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
          int roff[6], coff[3];
#pragma unroll
          for (int e = 0; e < 6; ++e) {
            int rs;
            const int y = canvas_coord(4 * tr - 1 + e, ir0, p.Pr, H, sep_r, rs);
            roff[e] = y >= 0 && rs * p.NC < p.B && T < p.ntiles ? (rs * p.NC * H * W * Cin + y * W * xppx) * 4 : BIGOFF;
          }
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            int cs;
            const int x = canvas_coord(4 * tc - 1 + 3 * half + e, ic0, p.Pc, W, sep_c, cs);
            coff[e] = x >= 0 && cs < p.NC ? (cs * H * W * Cin + x * xppx + ch) * 4 : BIGOFF;
          }
#pragma unroll
          for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) poff[q][a][b] = (int)((unsigned)roff[a] + (unsigned)coff[b]);
          if (half == 0 && pr == 0 && j <= t_last) {  // the item's output geometry (as below)
            int* gt = geo + ((j % NGT) * FTT + i) * GEOW;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              int rs, cs;
              const int y = canvas_coord(4 * tr + e, ir0, p.Pr, H, sep_r, rs);
              const int x = canvas_coord(4 * tc + e, ic0, p.Pc, W, sep_c, cs);
              const bool rok = y >= 0 && rs * p.NC < p.B && T < p.ntiles, cok = x >= 0 && cs < p.NC;
              gt[e] = rok ? rs * p.NC * H * W * Cout : 0;
              gt[4 + e] = rok ? y * W : -1;
              gt[8 + e] = cok ? cs * H * W * Cout : 0;
              gt[12 + e] = cok ? x : -1;
            }
          }
        }
      };
      struct Patch2 {
        f2 d[2][6][3];
      };
      auto load = [&](Patch2& P) {
        if (ls == 0) enter_item(lj);
        const int soff = __builtin_amdgcn_readfirstlane(min(ls, KST - 1)) * xstep;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) {
              const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, poff[q][a][b], soff, 0);
              P.d[q][a][b] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
            }
        if (++ls == KS) {
          ++lj;
          ls = 0;
        }
      };
      int dst_off[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 8 * t + 4 * q + ii;  // plane i / 16, tile i % 16 of it
        dst_off[q] = (i >> 4) * VSTEP + vslot(16 * (ch >> 2) + (i & 15)) * 4 + (ch & 3) + half * 18 * 256;
      }
      auto store = [&](Patch2& P, int g) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          f2 (&d)[6][3] = P.d[q];
#pragma unroll
          for (int b = 0; b < 3; ++b) {
            f2 c[6], o[6];
#pragma unroll
            for (int a = 0; a < 6; ++a) c[a] = d[a][b];
            bt6v(c, o);
#pragma unroll
            for (int a = 0; a < 6; ++a) d[a][b] = o[a];
          }
#pragma unroll
          for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int b = 0; b < 3; ++b)
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(d[k][b][e]),
                                                                __float_as_uint(d[3 + k][b][e]), false, false);
                d[k][b][e] = __uint_as_float(r[0]);
                d[3 + k][b][e] = __uint_as_float(r[1]);
              }
          float* dst = ring + (g % NBT) * SLOTF + dst_off[q];
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const f2 row[6] = {d[k][0], d[k][1], d[k][2], d[3 + k][0], d[3 + k][1], d[3 + k][2]};
            f2 v[6];
            bt6v(row, v);
#pragma unroll
            for (int b = 0; b < 6; ++b) *reinterpret_cast<f2*>(dst + (6 * k + b) * 256) = v[b];
          }
        }
      };
      int fseen = 0;
      auto put = [&](Patch2& P, int g) {
        if (g - NBT + 1 > fseen) fseen = lds_wait_min<NMW>(fre, g - NBT + 1, p.poll_max);
        store(P, g);
        lds_publish(rdy + t, lane, g + 1);
      };
      Patch2 pa, pb;
      load(pa);
      for (int b = 0;; b += 2) {
        load(pb);  // (past the stream's end it re-reads the clamped last item; never stored)
        __builtin_amdgcn_sched_barrier(0);
        put(pa, b);
        if (b + 1 >= G) break;
        load(pa);
        __builtin_amdgcn_sched_barrier(0);
        put(pb, b + 1);
        if (b + 2 >= G) break;
      }
      w4_report_handoff(fseen, p.err);
      return;
    }
  }
  if (wid >= NMW) {
    // ---- transform waves: every K-step, wave t transforms tiles 4t .. 4t+3 of the item for
    // the step's 16 channels in packed f32, two channels per lane and half a patch per lane:
    // lane (half h, tile 4t + ii, channel pair pr) loads patch columns 3h .. 3h+2 of channels
    // 2pr, 2pr+1 (18 8-byte loads; a wave's load covers 8 runs of 64 contiguous bytes), adds
    // the folded pre-BN shift, applies B^T down its 3 columns, trades 9 values with its partner
    // lane (v_permlane32_swap: half 0 keeps patch rows 0-2, half 1 rows 3-5), applies B^T
    // along its 3 rows and writes them (18 ds_write_b64) into ring slot g % NBUF once the MFMA
    // waves have read that slot's previous step; its patch loads were issued two steps earlier.
    const int t = wid - 4;
    // conv1's transform (pre-BN folded in: 18 more packed FMAs per K-step) is the slower side of
    // the hand-off; at issue priority over its SIMD's MFMA wave it keeps the ring ahead
    // (measured per launch, B = 256: stage-3 conv1 242 -> 232 us, stage-2 229 -> 215; for the
    // conv2 epilogues, whose transform has no pre-BN, priority was neutral to +3%)
    if constexpr (PRE) __builtin_amdgcn_s_setprio(1);
    const int half = lane >> 5, ii = (lane >> 3) & 3, pr = lane & 7;
    const int i = 4 * t + ii, ch = 2 * pr;
    const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x, p.B * H * W * Cin * 4);
    // input layout: NHWC (a pixel's Cin channels contiguous, a K-step's 16 at +16 step floats) or
    // channel-blocked [B][Cin/16][H][W][16] (a pixel's 16 channels of block `step` contiguous, the
    // next pixel 16 floats on: a wave load covers neighbouring pixels' lines)
    const bool xblk = (p.blk & W4_BLK_X) != 0;
    const int xppx = xblk ? KC : Cin;                     // floats from one pixel to the next
    const int xstep = xblk ? H * W * KC * 4 : KC * 4;     // bytes from one K-step to the next
    const __amdgpu_buffer_rsrc_t xr_none = uniform_rsrc(p.x, 0);
    const bool sep_r = p.Pr > H, sep_c = p.Pc > W;
    // the item's patch geometry, recomputed when the load stream enters a new item: byte
    // offset of every patch pixel of the lane's 3 columns (channel ch of step 0; BIGOFF sums
    // for padding)
    int poff[6][3];
    // PRE: in-image masks of the patch rows / the lane's columns (1 or 0).  Separable: a patch
    // pixel of an image past B (partial last canvas row) is never inside the 3x3 window of a
    // stored output (a separator row / column lies between; launch_wino4 forces one below
    // every image row when such a canvas row exists), so it may take the shift like an
    // in-image pixel.
    float rowm[6], colm[3];
    int lj = 0, ls = 0, ks_real = KS, step0 = 0;
    auto enter_item = [&](int j) {
      const Item it = item_at(min(j, t_last));
      ks_real = steps_of(it);
      step0 = SPLIT ? it.split * KS : 0;
      const int T = it.mb * FT + i;
      const int tr = T / p.TWc, tc = T - tr * p.TWc;
      const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
      int roff[6], coff[3];
      bool rin[6], cin[3];
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        int rs;
        const int y = canvas_coord(4 * tr - 1 + e, ir0, p.Pr, H, sep_r, rs);
        rin[e] = y >= 0 && rs * p.NC < p.B && T < p.ntiles;
        roff[e] = rin[e] ? (rs * p.NC * H * W * Cin + y * W * xppx) * 4 : BIGOFF;
      }
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        int cs;
        const int x = canvas_coord(4 * tc - 1 + 3 * half + e, ic0, p.Pc, W, sep_c, cs);
        cin[e] = x >= 0 && cs < p.NC;
        coff[e] = cin[e] ? (cs * H * W * Cin + x * xppx + ch) * 4 : BIGOFF;
      }
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) poff[a][b] = (int)((unsigned)roff[a] + (unsigned)coff[b]);
      if constexpr (PRE) {
#pragma unroll
        for (int e = 0; e < 6; ++e) rowm[e] = rin[e] ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 3; ++e) colm[e] = cin[e] ? 1.f : 0.f;
      }
      // output geometry of the item's tiles, for the MFMA waves' epilogue (not for the
      // stream's overrun past the last item)
      if (half == 0 && pr == 0 && j <= t_last) {
        // rows: [e] image-row base (floats of the images before the row's), [4 + e] y * W (or -1);
        // columns: [8 + e] image base within the row, [12 + e] x (or -1)
        int* gt = geo + ((j % NGEO) * FT + i) * GEOW;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int rs, cs;
          const int y = canvas_coord(4 * tr + e, ir0, p.Pr, H, sep_r, rs);
          const int x = canvas_coord(4 * tc + e, ic0, p.Pc, W, sep_c, cs);
          const bool rok = y >= 0 && rs * p.NC < p.B && T < p.ntiles, cok = x >= 0 && cs < p.NC;
          gt[e] = rok ? rs * p.NC * H * W * Cout : 0;
          gt[4 + e] = rok ? y * W : -1;
          gt[8 + e] = cok ? cs * H * W * Cout : 0;
          gt[12 + e] = cok ? x : -1;
        }
      }
    };
    // a patch buffer: the lane's 6x3 values (2 channels each) and, for PRE, the folded shift
    // t = shift / scale of its channels (tt) with its item's in-image row / column masks (rowm,
    // colm; the masks are copied because the next item's geometry may replace them before this
    // patch is stored).  tt is only multiplied in at store time: using it at load time made the
    // compiler wait for it -- and, loads retiring in order, for the patch loads issued before it --
    // right after issuing them, so each load() stalled for its own patch's round trip (batch 1:
    // two serialized round trips before step 0 reached the ring).
    struct Patch {
      f2 d[6][3];
      f2 tt;
      float rowm[6];
      float colm[3];
    };
    Patch pa, pb, pc;
    // issue the patch loads of the next step of the stream (steps are loaded in order)
    auto load = [&](Patch& P) {
      if (ls == 0) enter_item(lj);
      // split-K padding step: every load is out of range (num_records 0) and reads zeros, and
      // the BN shift is dropped
      // (readfirstlane: the stream counters are wave-uniform, but the compiler loses track of
      // that through the unrolled loop's phis and would wrap every load in a waterfall loop)
      const bool live = !SPLIT || __builtin_amdgcn_readfirstlane(ls < ks_real ? 1 : 0);
      const __amdgpu_buffer_rsrc_t r = live ? xr : xr_none;
      const int step = __builtin_amdgcn_readfirstlane(step0 + min(ls, ks_real - 1));
      const int soff = step * xstep;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][b], soff, 0);
          P.d[a][b] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
        }
      if constexpr (PRE) {
        P.tt = live ? *reinterpret_cast<const f2*>(p.pre_t + step * KC + ch) : f2{0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 6; ++e) P.rowm[e] = rowm[e];
#pragma unroll
        for (int e = 0; e < 3; ++e) P.colm[e] = colm[e];
      }
      if (++ls == KS) {
        ++lj;
        ls = 0;
      }
    };
    // the ring address of (tile i, channels ch, ch+1): A-fragment slot lane 16 k + i
    // (k = ch / 4), elements ch % 4 .. +1, at 16-byte slot vslot(16 k + i); half h writes the
    // transform rows 3h .. 3h+2, i.e. xi from 18 h
    const int dst_off = vslot(16 * (ch >> 2) + i) * 4 + (ch & 3) + half * 18 * 256;
    // transform a loaded patch and write it into ring slot g % NBUF
    auto store = [&](Patch& P, int g) {
      f2 (&d)[6][3] = P.d;
      if constexpr (PRE)
        // BN(x) = scale (x + t) with the scale folded into U: add t at in-image pixels only,
        // the conv's zero padding and the canvas separators stay 0 (BN -> zero-padded Conv2d)
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          const f2 trow = P.tt * P.rowm[a];
#pragma unroll
          for (int b = 0; b < 3; ++b) d[a][b] = __builtin_elementwise_fma(trow, f2{P.colm[b], P.colm[b]}, d[a][b]);
        }
#pragma unroll
      for (int b = 0; b < 3; ++b) {  // the lane's columns: d[.][b] <- (B^T d)[.][b]
        f2 c[6], o[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) c[a] = d[a][b];
        bt6v(c, o);
#pragma unroll
        for (int a = 0; a < 6; ++a) d[a][b] = o[a];
      }
      // partner exchange: swap(upper half of d[k][b], lower half of d[3+k][b]) leaves, in both
      // halves, transform row 3h + k with column b in d[k][b] and column 3 + b in d[3+k][b]
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int b = 0; b < 3; ++b)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(d[k][b][e]),
                                                            __float_as_uint(d[3 + k][b][e]), false, false);
            d[k][b][e] = __uint_as_float(r[0]);
            d[3 + k][b][e] = __uint_as_float(r[1]);
          }
      float* dst = ring + (g % NBUF) * VSTEP + dst_off;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const f2 row[6] = {d[k][0], d[k][1], d[k][2], d[3 + k][0], d[3 + k][1], d[3 + k][2]};
        f2 v[6];
        bt6v(row, v);
#pragma unroll
        for (int b = 0; b < 6; ++b) *reinterpret_cast<f2*>(dst + (6 * k + b) * 256) = v[b];
      }
    };
    // Step g is stored into ring slot g % NBUF once every MFMA wave has finished reading step
    // g - NBUF (fre >= g - NBUF + 1), then published (rdy[t] = g + 1).  Its patch loads were
    // issued two steps earlier (three patch buffers rotate), so a store never waits for its own
    // loads' issue.  Loads run past the stream's end unconditionally (they fetch whatever the
    // clamped geometry names and are never stored): a branch around them would make the
    // compiler's wait-count tracking wait for the freshly issued loads before the store.
    int fseen = 0;
    auto put = [&](Patch& P, int g) {
      if (g - NBUF + 1 > fseen) fseen = lds_wait_min<NMW>(fre, g - NBUF + 1, p.poll_max);
      store(P, g);
      lds_publish(rdy + t, lane, g + 1);
    };
    if (G <= 2) {
      // one or two K-steps (split-K serving launches): no loads past the stream's end.  The
      // general loop below issues two extra patch loads ahead; for a stream this short they
      // only fetch the clamped last item again, and entering that item's geometry waited (a
      // register of its address arithmetic still had a patch load outstanding) for the patches
      // already in flight: a round trip before step 0 could reach the ring.
      load(pa);
      if (G == 2) load(pb);
      put(pa, 0);
      if (G == 2) put(pb, 1);
      w4_report_handoff(fseen, p.err);
      return;
    }
    load(pa);
    load(pb);
    for (int b = 0;; b += 3) {
      load(pc);
      __builtin_amdgcn_sched_barrier(0);  // the loads go out first
      put(pa, b);
      if (b + 1 >= G) break;
      load(pa);
      __builtin_amdgcn_sched_barrier(0);
      put(pb, b + 1);
      if (b + 2 >= G) break;
      load(pb);
      __builtin_amdgcn_sched_barrier(0);
      put(pc, b + 2);
      if (b + 3 >= G) break;
    }
    w4_report_handoff(fseen, p.err);
    return;
  }

  // ---- MFMA waves: wave w owns couts 16w .. 16w+15 of every item (tall items: couts 16 (w & 1)
  // of tile half w >> 1) ---------------------------------------------------------------------
  const int w = VAR == W4_TALL ? (wid & 1) : wid;  // cout block of the item
  const int th = VAR == W4_TALL ? (wid >> 1) : 0;  // 16-tile plane of the item
  const __amdgpu_buffer_rsrc_t ur = uniform_rsrc(p.u, NXI * Cout * Cin * 4);
  const int NB16 = Cout / 16;
  const int lo = lane * 16;
  // U fragment of (item, step s, xi): ((xi * NB16 + nb16) * KST + step) KiB + 16 lane; the
  // xi term is a uniform stride, the rest is the item's base + its clamped step
  const int XS = NB16 * KST * 1024;
  auto ubase = [&](int j) {  // byte offset of (item j, step 0 of its K range, xi 0)
    const Item it = item_at(min(j, t_last));
    return (min(it.nb * (FNW / 16) + w, NB16 - 1) * KST + (SPLIT ? it.split * KS : 0)) * 1024;
  };
  auto ulast = [&](int j) {  // last real K-step of item j (split-K: the short last split)
    return SPLIT ? steps_of(item_at(min(j, t_last))) - 1 : KST - 1;
  };
  // the stream: item j (local), steps [0, KS)
  int j = 0;
  constexpr int URING = uring_depth<EPI>();
  f4 uring[URING];
  int ub = ubase(j), ul = ulast(j);
#pragma unroll
  for (int r = 0; r < URING; ++r) uring[r] = ld4(ur, lo, r * XS + ub);
  const float* vrd = ring + th * VSTEP + vslot(lane) * 4;
  // B fragments (V) of the next xi pair, carried across K-steps: step g + 1's first pair is read
  // during step g's last MFMAs, once the transform waves have published it
  int rseen = lds_wait_min<NTW>(rdy, 1, p.poll_max);  // step 0 is in the ring
  f4 a0n = *reinterpret_cast<const f4*>(vrd), a1n = *reinterpret_cast<const f4*>(vrd + 256);
  int g = 0;
  // Whole-item launches (MODE 0) split each item's epilogue in two.  Part A, at the end of item
  // j: the output transform, the BN parameters and the residual loads.  Part B, one output pixel
  // per xi pair of item j + 1's FIRST K-step (pixel i at pair i + 2): BN, PReLU, residual add and
  // the 16-byte store.  So the residual loads' latency and the stores' write-back overlap MFMAs,
  // and the next item's U refills no longer queue behind a burst of 16 stores (vmcnt counts loads
  // and stores in issue order).  The pending pixel state (outputs, residual, offsets) replaces
  // accumulators that are not live yet at the start of a K-step, so it costs no registers at the
  // peak.  Before the first item nothing is pending (offsets past the range: stores dropped);
  // the last item's part B runs after the loop.
  constexpr bool DEFER = !SPLIT;
  constexpr bool DRES = DEFER && (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU);
  const __amdgpu_buffer_rsrc_t yr_d = uniform_rsrc(p.y, p.B * H * W * Cout * 4);
  f4 pv[16], pres[16], psc = {1.f, 1.f, 1.f, 1.f}, psh = {0.f, 0.f, 0.f, 0.f}, pal = psh, pcl = psh;
  int po[16];
  if constexpr (DEFER) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pv[i] = pres[i] = f4{0.f, 0.f, 0.f, 0.f};
      po[i] = BIGOFF;
    }
  }
  // PReLU t > 0 ? t : a t as med3(t, a t, c): c = +inf for a slope a <= 1 (= max(t, a t)),
  // -inf for a > 1 (= min(t, a t)); med3 returns one of its operands, so the value is the
  // reference's exactly (up to the sign of a zero), in a packed multiply and a med3 per value
  // instead of a multiply, a compare and a select
  auto prelu_q = [](f4 v, f4 al, f4 cl) {
    const f4 av = v * al;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __builtin_amdgcn_fmed3f(v[r], av[r], cl[r]);
    return v;
  };
  auto finish = [&](int i) {  // part B of pending pixel i
    f4 v = __builtin_elementwise_fma(pv[i], psc, psh);
    if constexpr (EPI == EPI_AFFINE_PRELU) v = prelu_q(v, pal, pcl);
    if constexpr (DRES) {
      v += pres[i];
      if constexpr (EPI == EPI_AFFINE_RES_PRELU) v = prelu_q(v, pal, pcl);
    }
    const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);
  };
  // One item of the stream: its K-steps, then its epilogue.
  auto segment = [&]() {
    const Item it = item_at(j);
    const int s0 = 0, s1 = KS;
    const bool live = it.nb * FNW + w * 16 < Cout;  // Cout % FNW != 0: idle wave of the last block
    const int ub_next = ubase(j + 1);               // the next item's step 0; its first step (prefetched
                                                    // during this item's last one)
    f4 acc[NXI];
#pragma unroll
    for (int x = 0; x < NXI; ++x) acc[x] = f4{0.f, 0.f, 0.f, 0.f};
    auto kstep = [&](int s, auto first_step) {
      // ring slot g % NBUF holds step g (published before this wave read its first pair)
      const float* vb = vrd + (g % NBT) * SLOTF;
      const float* vn = vrd + ((g + 1) % NBT) * SLOTF;
      // U refills: xi + URING of this step, or xi + URING - 36 of the next step (or item)
      const int cur = ub + min(s, ul) * 1024;
      const int nxt = s + 1 < s1 ? ub + min(s + 1, ul) * 1024 : ub_next;
      // xi in pairs: the two accumulation chains interleave (a 16x16x4 MFMA's result is not
      // ready for the next one on the same accumulator at issue rate).  A fragments one pair
      // ahead (the LDS reads of pair x + 2 are in flight during pair x's MFMAs); an idle
      // quarter (!live) computes on a clamped U block and is never stored.
#pragma unroll
      for (int x = 0; x < NXI; x += 2) {
        const f4 a0 = a0n, a1 = a1n;
        // the last pair reads step g + 1's first fragments: wait until it is published (the
        // counter seen last time usually already covers it: no poll)
        if (x + 2 == NXI && g + 1 < G && rseen < g + 2) rseen = lds_wait_min<NTW>(rdy, g + 2, p.poll_max);
        const float* nb = x + 2 < NXI ? vb + (x + 2) * 256 : vn;
        a0n = *reinterpret_cast<const f4*>(nb);
        a1n = *reinterpret_cast<const f4*>(nb + 256);
        const f4 u0 = uring[x % URING], u1 = uring[(x + 1) % URING];
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
          uring[y % URING] = y + URING < NXI ? ld4(ur, lo, (y + URING) * XS + cur)
                                             : ld4(ur, lo, (y + URING - NXI) * XS + nxt);
        }
        // pin the slot's order: LDS reads of the next pair, the 8 MFMAs, the 2 U refills
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        // the previous item's pending output pixel x / 2 - 2 (after this pair's refills, so the
        // refills of earlier pairs never wait for its store)
        if constexpr (DEFER && decltype(first_step)::value)
          if (x >= 4) finish(x / 2 - 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      ++g;
      // every fragment of step g - 1 has been read (they fed this step's MFMAs): free its slot
      lds_publish(fre + wid, lane, g);
    };
    // the item's first K-step is peeled off the loop: it follows the previous item's epilogue
    // in straight-line code, so the wait for its U fragments counts exactly the epilogue's
    // stores in between (a merged loop header made the compiler wait for every outstanding
    // load and store, vmcnt(0), at every K-step)
    kstep(s0, std::true_type{});
    for (int s = s0 + 1; s < s1; ++s) kstep(s, std::false_type{});
    ub = ub_next;
    ul = ulast(j + 1);
    // an idle quarter (!live, Cout % 64 != 0) runs the epilogue too, with every store dropped
    // (no branch: a merge here costs the next K-step a full wait for stores)
    // ---- epilogue (lane-local): U is the A operand, so lane (tile n, row group rg) holds
    // couts 4rg .. 4rg+3 of tile n for every xi; Y = A^T M A per (tile, cout), BN (+PReLU |
    // +residual), one 16-byte store of the 4 couts per output pixel
    const int n = lane & 15, rg = lane >> 4;
    const int cout0 = min(it.nb * FNW + w * 16, Cout - 16) + 4 * rg;  // (clamped for an idle wave)
    const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.res, DRES ? p.B * H * W * Cout * 4 : 0);
    // byte offsets of tile n's 16 outputs = a row part + a column part (8 multiplies, not 16).
    // Padding rows / columns and an idle quarter get BIGOFF, so every sum with them lies past the
    // buffer's range (unsigned) and the store / residual load is dropped by the range check,
    // which also drops the pixels of absent images in a partial last canvas row (>= B*H*W).
    const int* gt = geo + ((j % NGT) * FTT + th * FT + n) * GEOW;
    // byte offsets of the tile's 16 pixels (4 couts each) in a tensor of the output's shape, NHWC
    // (ppx = Cout floats per pixel, couts at cout0) or channel-blocked (ppx = 16, cout0's block)
    auto row_col_offsets = [&](bool blk, int (&ro)[4], int (&co)[4]) {
      const int ppx = blk ? 16 : Cout;
      const int cb = blk ? (cout0 >> 4) * H * W * 16 + (cout0 & 15) : cout0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ro[e] = gt[4 + e] >= 0 && live ? (gt[e] + gt[4 + e] * ppx + cb) * 4 : BIGOFF;
        co[e] = gt[12 + e] >= 0 ? (gt[8 + e] + gt[12 + e] * ppx) * 4 : BIGOFF;
      }
    };
    auto tile_offsets = [&](bool blk, int (&oo)[4][4]) {
      int ro[4], co[4];
      row_col_offsets(blk, ro, co);
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) oo[y][x] = (int)((unsigned)ro[y] + (unsigned)co[x]);
    };
    const bool yblk = RMIX ? RMIX == 1 : (p.blk & W4_BLK_Y) != 0, rblk = RMIX ? RMIX == 2 : (p.blk & W4_BLK_RES) != 0;
    int oo[4][4];
    tile_offsets(yblk, oo);
    if constexpr (DEFER) {
      // part A: rows of A^T M A on all 4 couts (each frees 8 accumulator registers), the residual
      // of output rows 0-1 in flight during the column pass, then rows 2-3
      auto transform_to_pv = [&]() {
        f4 z[6][4];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          const f4 m6[6] = {acc[6 * a], acc[6 * a + 1], acc[6 * a + 2], acc[6 * a + 3], acc[6 * a + 4], acc[6 * a + 5]};
          at6q(m6, z[a]);
        }
        if constexpr (DRES && RMIX) {
          int rro[4], rco[4];
          row_col_offsets(rblk, rro, rco);
#pragma unroll
          for (int i = 0; i < 8; ++i) pres[i] = ld4(rr, (int)((unsigned)rro[i >> 2] + (unsigned)rco[i & 3]));
        } else if constexpr (DRES) {
#pragma unroll
          for (int i = 0; i < 8; ++i) pres[i] = ld4(rr, oo[i >> 2][i & 3]);
        }
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const f4 c6[6] = {z[0][x], z[1][x], z[2][x], z[3][x], z[4][x], z[5][x]};
          f4 o[4];
          at6q(c6, o);
#pragma unroll
          for (int y = 0; y < 4; ++y) pv[4 * y + x] = o[y];
        }
      };
      auto set_pending = [&]() {
        if constexpr (DRES && RMIX) {
          int rro[4], rco[4];
          row_col_offsets(rblk, rro, rco);
#pragma unroll
          for (int i = 8; i < 16; ++i) pres[i] = ld4(rr, (int)((unsigned)rro[i >> 2] + (unsigned)rco[i & 3]));
        } else if constexpr (DRES) {
#pragma unroll
          for (int i = 8; i < 16; ++i) pres[i] = ld4(rr, oo[i >> 2][i & 3]);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) po[i] = oo[i >> 2][i & 3];
        psc = *reinterpret_cast<const f4*>(p.post_scale + cout0);
        psh = *reinterpret_cast<const f4*>(p.post_shift + cout0);
        if constexpr (EPI == EPI_AFFINE_PRELU || EPI == EPI_AFFINE_RES_PRELU) {
          pal = *reinterpret_cast<const f4*>(p.prelu + cout0);
#pragma unroll
          for (int r = 0; r < 4; ++r) pcl[r] = pal[r] <= 1.f ? __builtin_inff() : -__builtin_inff();
        }
      };
      transform_to_pv();
      set_pending();
      return;
    }
    // MODE 1 (split-K): raw partial outputs (the same output transform, no epilogue) into compact
    // slot [16 tiles][16 pixels][64 couts] of split it.split of launch item it.li, summed in split
    // order and finished by wino4_part_fixup_kernel.  Write-through (sc1): the fixup on other XCDs
    // reads the slots right after this launch, and a launch that leaves its slots dirty in L2 pays
    // for their write-back at the kernel boundary (serving batch 1: embed + match 1.925 -> 1.851
    // ms, same box)
    if constexpr (SPLIT) {
      f4 z[6][4];
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const f4 m6[6] = {acc[6 * a], acc[6 * a + 1], acc[6 * a + 2], acc[6 * a + 3], acc[6 * a + 4], acc[6 * a + 5]};
        at6q(m6, z[a]);
      }
      const int slot = it.li * p.ksplit + it.split;
      const __amdgpu_buffer_rsrc_t sr = uniform_rsrc(p.part, (int)min(p.part_floats * 4, 0x7fffffffll));
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const f4 c6[6] = {z[0][x], z[1][x], z[2][x], z[3][x], z[4][x], z[5][x]};
        f4 o[4];
        at6q(c6, o);
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const u32x4 bits = {__float_as_uint(o[y].x), __float_as_uint(o[y].y), __float_as_uint(o[y].z),
                              __float_as_uint(o[y].w)};
          const int off = ((((slot * FT + n) * 16 + y * 4 + x) * FN) + w * 16 + 4 * rg) * 4;
          __builtin_amdgcn_raw_buffer_store_b128(bits, sr, off, 0, CPOL_SC1);
        }
      }
    }
  };
  for (; j < nloc; ++j) segment();
  if constexpr (DEFER)
#pragma unroll
    for (int i = 0; i < 16; ++i) finish(i);  // the last item's part B
  w4_report_handoff(rseen, p.err);
}

template <bool PRE, int EPI, int MODE, int RMIX = 0>
__global__ __launch_bounds__(512, 1) void wino4_kernel(Wino4Params p) {
  __shared__ __attribute__((aligned(16))) float ring[W4_LDS_FLOATS];
  wino4_body<PRE, EPI, MODE, RMIX>(p, ring, blockIdx.x, gridDim.x);
}

// Wide items (96 couts, six MFMA waves): whole-item launches of layers of 65..96 output channels
template <int EPI>
__global__ __launch_bounds__(512, 1) void wino4w_kernel(Wino4Params p) {
  __shared__ __attribute__((aligned(16))) float ring[W4_LDS_FLOATS];
  wino4_body<false, EPI, 0, 0, W4_WIDE>(p, ring, blockIdx.x, gridDim.x);
}

// Tall items (32 tiles x 32 couts): whole-item launches of layers of at most 32 output channels
template <int EPI>
__global__ __launch_bounds__(512, 1) void wino4t_kernel(Wino4Params p) {
  __shared__ __attribute__((aligned(16))) float ring[W4_LDS_FLOATS];
  wino4_body<false, EPI, 0, 0, W4_TALL>(p, ring, blockIdx.x, gridDim.x);
}

// Split-K finish of one output element group: y = epilogue(sum of an item's raw partial outputs,
// in part order: deterministic) at the item's in-image pixels.  idx = (tile n, pixel, cout quad)
// of launch item li, whose parts are in slots li * S .. li * S + S - 1.
template <int EPI>
__device__ __forceinline__ void w4_fixup_elem(const Wino4Params& p, int li, int idx) {
  const int gi = p.item0 + li, slot0 = li * p.ksplit, S = p.ksplit;
  const Item it = item_of(p, gi);
  const int n = idx >> 8, px = (idx >> 4) & 15, cq = idx & 15;
  const int cout0 = it.nb * FN + 4 * cq;
  const int T = it.mb * FT + n;
  if (n >= FT || cout0 >= p.Cout || T >= p.ntiles) return;
  const int H = p.H, W = p.W;
  const int tr = T / p.TWc, tc = T - tr * p.TWc;
  const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;
  int rs, cs;
  const int y = canvas_coord(4 * tr + (px >> 2), ir0, p.Pr, H, p.Pr > H, rs);
  const int x = canvas_coord(4 * tc + (px & 3), ic0, p.Pc, W, p.Pc > W, cs);
  if (y < 0 || rs * p.NC >= p.B || x < 0 || cs >= p.NC) return;
  const long long pix = (long long)(rs * p.NC * H + y) * W + (long long)cs * H * W + x;
  if (pix >= (long long)p.B * H * W) return;
  const float4* slab = reinterpret_cast<const float4*>(p.part);
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  // sixteen slot loads in flight at a time (every part of a split-K item: S <= 16 K-steps of
  // 16 channels per part at the serving sizes), summed in part order (deterministic): a loop of
  // one load and one add per part waited out every load's latency in turn (batch 1: 7.3 us per
  // fixup launch, 94 launches per forward; eight at a time: ~5 us)
  for (int s0 = 0; s0 < S; s0 += 16) {
    float4 a[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const long long q = ((((long long)slot0 + s0 + u) * FT + n) * 16 + px) * (FN / 4) + cq;
      a[u] = s0 + u < S ? slab[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (s0 + u < S) {
        v[0] += a[u].x;
        v[1] += a[u].y;
        v[2] += a[u].z;
        v[3] += a[u].w;
      }
  }
  // float offset of (pix, cout0) in NHWC or in the channel-blocked layout [B][Cout/16][H][W][16]
  auto at = [&](bool blk) {
    if (!blk) return pix * p.Cout + cout0;
    const long long hw = (long long)H * W, img = pix / hw;
    return img * hw * p.Cout + (long long)(cout0 >> 4) * hw * 16 + (pix - img * hw) * 16 + (cout0 & 15);
  };
  const long long yo = at((p.blk & W4_BLK_Y) != 0), ro = at((p.blk & W4_BLK_RES) != 0);
  float rv[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rv[r] = p.res[ro + r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t = v[r] * p.post_scale[cout0 + r] + p.post_shift[cout0 + r];
    if constexpr (EPI == EPI_AFFINE_PRELU) t = t > 0.f ? t : t * p.prelu[cout0 + r];
    if constexpr (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) {
      t += rv[r];
      if constexpr (EPI == EPI_AFFINE_RES_PRELU) t = t > 0.f ? t : t * p.prelu[cout0 + r];
    }
    v[r] = t;
  }
  // write-through like the slots: the next layer's split-K launch reads this output from every XCD
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(p.y, p.B * H * W * p.Cout * 4);
  const u32x4 bits = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(bits, yr, (int)(yo * 4), 0, CPOL_SC1);
}

// Split-K finish launch: grid (FT * 16 * FN / 4 / blockDim, items), blockIdx.y = launch item.
template <int EPI>
__global__ void wino4_part_fixup_kernel(Wino4Params p, int KST, int P) {
  w4_fixup_elem<EPI>(p, blockIdx.y, blockIdx.x * blockDim.x + threadIdx.x);
}

// G g G^T of every (cout, cin) filter, in double then rounded once to f32, scattered into the
// A-fragment (U) order wino4_kernel reads: [xi][Cout/16][Cin/16][lane = 16 k + cout%16][m] with
// cin % 16 = 4k + m.
__global__ void wino4_weight_kernel(const float* __restrict__ w, const float* __restrict__ pre_scale,
                                    float* __restrict__ u, int Cout, int Cin) {
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
    for (int x = 0; x < 3; ++x)
      g[y][x] = (double)w[((long long)(o * 3 + y) * 3 + x) * Cin + i] * (pre_scale ? (double)pre_scale[i] : 1.0);
  double tg[6][3];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int x = 0; x < 3; ++x) tg[a][x] = G[a][0] * g[0][x] + G[a][1] * g[1][x] + G[a][2] * g[2][x];
  const int NB16 = Cout / 16, KS = Cin / KC;
  const int nb16 = o >> 4, n = o & 15;
  const int s = i / KC, c = i % KC;
  const int ln = 16 * (c >> 2) + n, m = c & 3;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const double v = tg[a][0] * G[b][0] + tg[a][1] * G[b][1] + tg[a][2] * G[b][2];
      const int xi = 6 * a + b;
      u[(((long long)(xi * NB16 + nb16) * KS + s) * 64 + ln) * 4 + m] = (float)v;
    }
}

}  // namespace

size_t wino4_weight_floats(int Cout, int Cin) { return (size_t)NXI * Cout * Cin; }

hipError_t launch_wino4_weights(const float* w, const float* pre_scale, float* u, int Cout, int Cin, hipStream_t s) {
  if (Cout % 16 || Cin % KC) return hipErrorInvalidValue;
  const int n = Cout * Cin;
  hipLaunchKernelGGL(wino4_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, pre_scale, u, Cout, Cin);
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

bool wino4_supported(int Cin, int Cout, int kh, int kw, int stride, int pad) {
  return kh == 3 && kw == 3 && stride == 1 && pad == 1 && Cin % 16 == 0 && Cin >= 16 && Cout % 16 == 0 && Cout >= 16;
}

namespace {
// validation + canvas + item blocks of a layer (launch_wino4)
bool w4_setup(Wino4Params& p, bool pre) {
  p.poll_max = p.poll_max == 0 ? WINO4_POLL_DEFAULT : std::max(p.poll_max, 0);  // < 0: no polls (tests)
  if (!wino4_supported(p.Cin, p.Cout, 3, 3, 1, 1) || p.B < 1 || p.H < 1 || p.W < 1 ||
      (pre && !p.pre_t) || (long long)p.B * p.H * p.W * p.Cin * 4 >= BIGOFF ||
      (long long)p.B * p.H * p.W * p.Cout * 4 >= (1ll << 31) || (long long)NXI * p.Cout * p.Cin * 4 >= (1ll << 31))
    return false;
  wino4_canvas(p);
  if (pre && p.NC > 1 && p.B % p.NC && p.Pr == p.H) {
    // a partial last canvas row directly below full ones: give every image row a separator
    // row so the absent images' pixels stay outside every stored output's window (PRE masks)
    p.Pr = p.H + 1;
    p.ntiles = ((((p.B + p.NC - 1) / p.NC) * p.Pr + 3) / 4) * p.TWc;
  }
  p.mblocks = (p.ntiles + FT - 1) / FT;
  p.nblocks = (p.Cout + FN - 1) / FN;
  // tile blocks per XCD item group: 32 items for up to 4 cout blocks; at Cout = 512 (8 cout
  // blocks) 8 tile blocks x 8 cout blocks, so an XCD round streams half of the layer's U (37.7 MB)
  // instead of all of it, for patches read twice (stage 4: 238 -> 232 us, PMC-modelled traffic
  // 677 -> 453 MB per launch)
  p.nbg = std::max(1, std::min(p.mblocks, std::max(32 / p.nblocks, 8)));
  if (p.nbg_override > 0) p.nbg = std::max(1, std::min(p.mblocks, p.nbg_override));
  return true;
}

constexpr long long SLOT = (long long)FT * 16 * FN;  // floats of one compact partial slot

bool w4_aligned(const Wino4Params& p) {
  return ((reinterpret_cast<uintptr_t>(p.y) | reinterpret_cast<uintptr_t>(p.res) | reinterpret_cast<uintptr_t>(p.part)) &
          15) == 0;
}

int w4_cus() {
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus > 0 ? cus : 256;
}

// K parts for a split-K launch of n items: as many as fit one round of workgroups, bounded by
// the K-steps and the slot workspace; ks_per steps each
int w4_split_of(const Wino4Params& p, int n, int cus, int& ks_per) {
  const int KST = p.Cin / KC;
  int S = (int)std::min<long long>(std::min(KST, cus / n), p.part_floats / (SLOT * n));
  // a grid of one-K-step splits over more than half the chip loses to half the grid with two
  // steps each (half the slots for the fixup to sum): IR-101 batch 4, 2.37 -> 2.18 ms per
  // embed + match; batch 1 (64 workgroups at stage 3) and batch 8 (two-step splits over the
  // whole chip; halving them again cost +2.6%) keep theirs
  if (S * n > cus / 2 && (KST + S - 1) / S < 2) S = std::max(1, std::min(S, (cus / 2) / n));
  if (p.max_split > 0) S = std::min(S, p.max_split);
  ks_per = KST;
  if (S > 1) {
    ks_per = (KST + S - 1) / S;
    S = (KST + ks_per - 1) / ks_per;
  }
  return std::max(S, 1);
}
}  // namespace

hipError_t launch_wino4(const Wino4Params& p0, bool pre, Epi epi, hipStream_t s) {
  Wino4Params p = p0;
  if (!w4_setup(p, pre)) return hipErrorInvalidValue;
  const int KST = p.Cin / KC;
  const int nT = p.mblocks * p.nblocks;
  const bool aligned = w4_aligned(p);
  const int cus = w4_cus();
  const bool can_split = p.part && !p.no_split && aligned && KST > 1;
  auto split_of = [&](int n, int& ks_per) { return w4_split_of(p, n, cus, ks_per); };
  // Whole-item launch of n items from item0 (MODE 0), or split-K launch (MODE 1) + fixup.  (A
  // stream-K tail for the part-empty last round of whole items -- IR-101 B = 256: stage 3 3.52
  // rounds run as 4 -- was built in round 4 and measured neutral; two concurrent lanes fill that
  // round instead: tools/w4_archive/)
  Wino4Params pw = p;
  auto whole = [&](int item0, int n) {
    pw = p;
    pw.item0 = item0;
    pw.nitem = n;
    pw.ksplit = 1;
    pw.ks_per = KST;
  };
  auto splitk = [&](int item0, int n, int S, int ks_per) {
    pw = p;
    pw.item0 = item0;
    pw.nitem = n;
    pw.ksplit = S;
    pw.ks_per = ks_per;
  };
#define FR_W4_LAUNCH(PRE_, EPI_, MODE_)                                                                     \
  {                                                                                                         \
    const int nit = pw.nitem * pw.ksplit;                                                                   \
    hipLaunchKernelGGL((wino4_kernel<PRE_, EPI_, MODE_>), dim3(std::min(nit, cus)), dim3(512), 0, s, pw);   \
    if (MODE_ == 1) /* 64-thread blocks: a serving grid's few items still spread over the CUs */          \
      hipLaunchKernelGGL((wino4_part_fixup_kernel<EPI_>), dim3(FT * 16 * FN / 4 / 64, pw.nitem),     \
                         dim3(64), 0, s, pw, KST, cus);                                                     \
  }
  // a residual whose layout differs from y's (p.blk: the seams between NHWC and channel-blocked
  // activations): whole-item launches run instances of their own (RMIX); a split-K
  // launch's fixup addresses the residual on its own anyway, so split-K is the usual one
  const bool rmix = (((p.blk & W4_BLK_RES) != 0) != ((p.blk & W4_BLK_Y) != 0)) &&
                    (epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_PRELU);
  if (rmix) {
    if (pre || epi != EPI_AFFINE_RES) return hipErrorInvalidValue;
    int ks_per = KST;
    const int S = can_split && nT <= cus / 2 ? split_of(nT, ks_per) : 1;
    if (S > 1) {
      splitk(0, nT, S, ks_per);
      FR_W4_LAUNCH(false, EPI_AFFINE_RES, 1)
      return hipGetLastError();
    }
    whole(0, nT);
    const dim3 grid(std::min(nT, cus));
    if (p.blk & W4_BLK_Y)
      hipLaunchKernelGGL((wino4_kernel<false, EPI_AFFINE_RES, 0, 1>), grid, dim3(512), 0, s, pw);
    else
      hipLaunchKernelGGL((wino4_kernel<false, EPI_AFFINE_RES, 0, 2>), grid, dim3(512), 0, s, pw);
    return hipGetLastError();
  }
  // Wide items: a whole-item launch of a layer of 65..96 couts (the detector's 80-channel towers
  // and heads) as one 96-cout item per 16 tiles on wino4w_kernel, not a 64-cout item plus one with
  // three of its four MFMA waves idle (each with its own input transform).  A wide item costs
  // about two 64-cout items' time (SIMDs 0 and 1 run two MFMA waves each), so it only wins when the
  // 64-cout items take more than one round of workgroups (detector head at stride 32, 100 items:
  // 23.5 -> 32.9 us per tower conv as 50 wide items)
  // Tall items likewise: a layer of at most 32 couts as 32-tile x 32-cout items on wino4t_kernel
  // (a 64-cout item leaves two of its four MFMA waves on clamped weights), half the items at
  // about a 64-cout item's time each.
  const bool shape_epi = epi == EPI_AFFINE || epi == EPI_AFFINE_PRELU || epi == EPI_AFFINE_RES_PRELU;
  const bool wide = p.Cout > FN && p.Cout <= 96, tall = p.Cout <= 32;
  if (p.shapes && !pre && shape_epi && (wide || tall) && (nT > cus || p.shapes == 2)) {
    if (tall) p.mblocks = (p.ntiles + 2 * FT - 1) / (2 * FT);
    p.nblocks = 1;
    p.nbg = std::max(1, std::min(p.mblocks, p.nbg_override > 0 ? p.nbg_override : 32));
    whole(0, p.mblocks);
    const dim3 grid(std::min(p.mblocks, cus));
#define FR_W4_SHAPED(EPI_)                                                  \
  if (wide)                                                                 \
    hipLaunchKernelGGL((wino4w_kernel<EPI_>), grid, dim3(512), 0, s, pw);   \
  else                                                                      \
    hipLaunchKernelGGL((wino4t_kernel<EPI_>), grid, dim3(512), 0, s, pw);
    if (epi == EPI_AFFINE) {
      FR_W4_SHAPED(EPI_AFFINE)
    } else if (epi == EPI_AFFINE_PRELU) {
      FR_W4_SHAPED(EPI_AFFINE_PRELU)
    } else {
      FR_W4_SHAPED(EPI_AFFINE_RES_PRELU)
    }
#undef FR_W4_SHAPED
    return hipGetLastError();
  }
#define FR_W4_CASE(PRE_, EPI_)                                                                              \
  if (pre == PRE_ && epi == EPI_) {                                                                         \
    int ks_per = KST;                                                                                       \
    if (can_split && nT <= cus / 2) {                                                                       \
      /* small grid (serving batches): every item's K loop split */                                         \
      const int S = split_of(nT, ks_per);                                                                   \
      if (S > 1) {                                                                                          \
        splitk(0, nT, S, ks_per);                                                                           \
        FR_W4_LAUNCH(PRE_, EPI_, 1)                                                                         \
      } else {                                                                                              \
        whole(0, nT);                                                                                       \
        FR_W4_LAUNCH(PRE_, EPI_, 0)                                                                         \
      }                                                                                                     \
    } else {                                                                                                \
      /* whole items.  (Running a part-empty last round as a split-K launch of its own was      */          \
      /* measured neutral: stage 2, 6 rounds + 32 items, 244.6 -> 245.8 us; the short launch and  */          \
      /* its fixup cost about the round they save.)                                               */          \
      whole(0, nT);                                                                                         \
      FR_W4_LAUNCH(PRE_, EPI_, 0)                                                                           \
    }                                                                                                       \
    return hipGetLastError();                                                                               \
  }
  FR_W4_CASE(true, EPI_AFFINE_PRELU)       // IR conv1: pre-BN (in the transform), BN, PReLU
  FR_W4_CASE(false, EPI_AFFINE_RES)        // IR conv2: BN + identity shortcut
  FR_W4_CASE(false, EPI_AFFINE_PRELU)      // SCRFD conv + BN + ReLU (zero slopes)
  FR_W4_CASE(false, EPI_AFFINE)            // SCRFD conv + BN / bias
  FR_W4_CASE(false, EPI_AFFINE_RES_PRELU)  // SCRFD BasicBlock conv2 + BN + add + ReLU
#undef FR_W4_CASE
#undef FR_W4_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace frhip
