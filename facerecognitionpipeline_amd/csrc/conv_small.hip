// Serving-batch 3x3 convs (stride 1 or 2, pad 1, optional fused 1x1 stride-s shortcut) of the IR
// body, NHWC f32 on v_mfma_f32_16x16x4_f32: one workgroup per 16 output pixels x 16 output
// channels, the whole K reduction inside the workgroup.
//
// Why: a batch-1 forward is latency-bound.  The F(4x4) kernel needs split-K
// to occupy the chip at batch 1 (4 items at stage 3), i.e. a second launch per layer (the fixup)
// and a 64-KiB partial slot per split, and its filters are 4x larger than the direct ones (36 vs
// 9 values per (cin, cout)), all of which stream from HBM once per forward.  Here a layer is ONE
// launch: M = n*Ho*Wo pixels x Cout in 16x16 tiles (IR-101 stage 3 at batch 1: 13 x 16 = 208
// workgroups), each reducing all 9*Cin (+ Cin2) products of its tile:
//   * 4 waves split the K chunks (16 channels of one tap) round-robin, each keeping CH = 12 chunks
//     of fragments in flight (a register ring: one 16-byte load of weights and one of input per
//     lane and chunk), two accumulators per wave (consecutive chunks alternate: a 16x16x4 f32
//     MFMA's result is not ready for the next one at issue rate); the 4 waves' sums are added in
//     a fixed order through LDS (deterministic) and wave 0 applies the epilogue.  (8 waves with
//     18 chunks in flight each: no faster at stage 3, 2x slower at stage 1 where 190 VGPRs left
//     one workgroup per CU; `tools/convs_bench.py`.)
//   * XCD-aware order: the workgroups of one 16-channel output block (which read the same
//     weights) sit on one XCD, so each weight is fetched from HBM once per layer, not once per XCD.
//   * filters in fragment order (launch_convs_weights): a wave's weight load is one contiguous
//     KiB, not 16 rows x 64 B (16 filter rows 9 Cin * 4 B apart); measured on this GPU
//     (tools/l2_stride_bench.hip, 208 workgroups x 4 waves x 36 loads, 12 in flight): 2.5 vs 5.2 us.
//   * activations between two such layers channel-blocked (p.blk): [B][C/16][H][W][16], so a
//     wave's input load (16 consecutive pixels x 16 channels) is one contiguous KiB too, and so is
//     its output store; NHWC where the producer or a consumer is another kernel.
//   * outputs stored write-through (sc1): the next launch reads them from other XCDs anyway, and
//     what a launch leaves dirty in L2 is written back at the kernel boundary.
//   * pre-BN (conv1): the previous conv2's launch writes BN(y) beside y (ConvParams::y2, the same
//     fma the per-tap form does, so bitwise the same operand) and conv1 runs without PRE on it;
//     where that is not set up (PRE), the per-channel scale / shift are staged in LDS and applied
//     to in-image taps only when a fragment is consumed (zero padding stays zero).
//   * fragments: weights are the MFMA's A operand (16 couts x 4 channels, lane (cout, quad q)),
//     input its B operand (16 pixels x 4 channels); MFMA e of a chunk consumes channel 4q + e of
//     both, so a lane reads 4 consecutive channels per 16-byte load; the accumulator of lane
//     (pixel l & 15, row group l >> 4) holds couts 4 (l >> 4) .. +3 of one pixel: one 16-byte store.
#include <algorithm>

#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NWV = 4;   // waves per workgroup (the K chunks split round-robin)
constexpr int CH = 12;  // chunks in flight per wave
constexpr int SCMAX = 4;   // fused-shortcut chunks per wave (Cin2 <= 16 * NWV * SCMAX)
constexpr int BIGOFF = 0x7F000000;
constexpr int MAXC = 512;  // pre-BN channels staged in LDS
constexpr int CPOL_SC1 = 16;  // buffer-store cache policy bit sc1 (write-through)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* ptr, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, (int)std::min(bytes, 0x7fffffffll),
                                           0x00020000);
}
__device__ __forceinline__ u32x4 bits4(f4 v) {
  return u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
}
__device__ __forceinline__ f4 ld4(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

template <bool PRE, int EPI>
__global__ __launch_bounds__(64 * NWV) void convs_kernel(ConvParams p) {
  __shared__ __attribute__((aligned(16))) float pst[PRE ? 2 * MAXC : 4];
  __shared__ __attribute__((aligned(16))) f4 red[NWV - 1][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Cin = p.Cin, Cin2 = p.Cin2, Cout = p.Cout, H = p.H, W = p.W, Ho = p.Ho, Wo = p.Wo, S = p.stride;
  const int NCB = Cout / 16, NPB = (p.M + 15) / 16;
  // XCD-aware tile order: blocks g = x + 8 s (x = the XCD the hardware deals block g to) take
  // the cout blocks cb = x (mod 8), all their pixel blocks in turn (NCB % 8 == 0), else plain order
  int cb, pb;
  {
    const int g = blockIdx.x;
    if (NCB % 8 == 0) {
      const int x = g & 7, s = g >> 3;
      cb = x + 8 * (s / NPB);
      pb = s - (s / NPB) * NPB;
    } else {
      cb = g / NPB;
      pb = g - cb * NPB;
    }
  }
  const int q = lane >> 4;
  // this lane's B-operand pixel and A-operand cout
  const int m = pb * 16 + (lane & 15);
  const bool mval = m < p.M;
  const int mm = mval ? m : 0;
  const int b = mm / (Ho * Wo), r0 = mm - b * (Ho * Wo), oy = r0 / Wo, ox = r0 - oy * Wo;
  const int KR = 9 * Cin + Cin2;  // weight row length
  const __amdgpu_buffer_rsrc_t xr = rsrc(p.x, (long long)p.B * H * W * Cin * 4);
  const __amdgpu_buffer_rsrc_t x2r = rsrc(p.x2 ? p.x2 : p.x, p.x2 ? (long long)p.B * H * W * Cin2 * 4 : 0);
  const __amdgpu_buffer_rsrc_t wr = rsrc(p.w, (long long)Cout * KR * 4);
  const int CC = Cin >> 4;           // 16-channel chunks per tap
  // activation layouts: bytes per pixel and per 16-channel chunk (NHWC or channel-blocked)
  const bool xbk = p.blk & CONVS_BLK_X, x2bk = p.blk & CONVS_BLK_X2, rbk = p.blk & CONVS_BLK_RES,
             ybk = p.blk & CONVS_BLK_Y;
  const int xpx = xbk ? 64 : Cin * 4, xcc = xbk ? H * W * 64 : 64;
  const int wl = (cb * (KR >> 4) * 64 + lane) * 16;  // this lane's 16 B of chunk 0 of block cb
  // This wave's conv chunks: (tap, channel chunk cc) for cc = w, w + NWV, ... < CC, taps in
  // order, walked incrementally with wave-uniform (scalar) state and no branches: per chunk a few
  // scalar and ~10 vector ops (the first version's divisions, branches and per-chunk buffer
  // descriptor selects were ~100 scalar instructions per chunk; the CU's one scalar unit, shared by
  // its 4 waves, then took longer than the MFMAs and the loads).  Past the last chunk the offsets
  // are out of range: zeros.  The fused shortcut's chunks (x2) are loaded once up front.
  const int ncc = w < CC ? (CC - w + NWV - 1) / NWV : 0;  // this wave's chunks per tap
  const int nI = 9 * ncc;
  int it_i = 0, it_tap = 0, it_k = 0;
  const int oys = oy * S - 1, oxs = ox * S - 1;
  const int xbase = b * H * W * Cin * 4 + 4 * q * 4;
  auto next_frag = [&](int& woff, int& xoff, int& meta) {
    const int ky = (it_tap * 11) >> 5, kx = it_tap - 3 * ky;  // it_tap / 3 for it_tap < 9
    const int c0 = (w + NWV * it_k) * 16;
    const int iy = oys + ky, ix = oxs + kx;
    const bool live = it_i < nI;
    const bool in = live && mval && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    woff = live ? wl + (it_tap * CC + (c0 >> 4)) * 1024 : BIGOFF;
    xoff = in ? xbase + (iy * W + ix) * xpx + (c0 >> 4) * xcc : BIGOFF;
    meta = (c0 + 4 * q) | (in ? 1 << 16 : 0);
    ++it_i;
    const bool wrap = ++it_k == ncc;
    it_k = wrap ? 0 : it_k;
    it_tap += wrap ? 1 : 0;
  };
  // the fused shortcut: chunks cc = w, w + NWV, ... of Cin2 (at most SCMAX per wave)
  f4 swa[SCMAX], sxa[SCMAX];
#pragma unroll
  for (int k = 0; k < SCMAX; ++k) {
    const int c0 = (w + NWV * k) * 16;
    const bool live = c0 < Cin2;
    swa[k] = ld4(wr, live ? wl + (9 * CC + (c0 >> 4)) * 1024 : BIGOFF);
    sxa[k] = ld4(x2r, live && mval ? b * H * W * Cin2 * 4 + (oy * S * W + ox * S) * (x2bk ? 64 : Cin2 * 4) +
                                         (c0 >> 4) * (x2bk ? H * W * 64 : 64) + 16 * q
                                   : BIGOFF);
  }
  f4 wa[CH], xa[CH];
  int mt[CH];
#pragma unroll
  for (int d = 0; d < CH; ++d) {
    int wo, xo, me;
    next_frag(wo, xo, me);
    wa[d] = ld4(wr, wo);
    xa[d] = ld4(xr, xo);
    mt[d] = me;
  }
  // the epilogue's operands, loaded now so their latency overlaps the K loop (wave 0 uses them)
  const int c4 = cb * 16 + 4 * q;
  // output element (floats) of this lane's 4 couts: b, pixel r0 of Ho x Wo, block cb, 4 q
  const int yoff = b * Ho * Wo * Cout + r0 * (ybk ? 16 : Cout) + cb * (ybk ? Ho * Wo * 16 : 16) + 4 * q;
  f4 e_sc = {0.f, 0.f, 0.f, 0.f}, e_sh = e_sc, e_al = e_sc, e_res = e_sc, e_s2 = e_sc, e_t2 = e_sc;
  if (w == 0) {
    if (p.y2) {
      e_s2 = *reinterpret_cast<const f4*>(p.y2_scale + c4);
      e_t2 = *reinterpret_cast<const f4*>(p.y2_shift + c4);
    }
    e_sc = *reinterpret_cast<const f4*>(p.post_scale + c4);
    e_sh = *reinterpret_cast<const f4*>(p.post_shift + c4);
    if constexpr (EPI == EPI_AFFINE_PRELU) e_al = *reinterpret_cast<const f4*>(p.prelu + c4);
    if constexpr (EPI == EPI_AFFINE_RES)
      if (mval)
        e_res = *reinterpret_cast<const f4*>(p.res + b * Ho * Wo * Cout + r0 * (rbk ? 16 : Cout) +
                                             cb * (rbk ? Ho * Wo * 16 : 16) + 4 * q);
    if constexpr (EPI == EPI_AFFINE_RES_SUB)  // res[b, S oy, S ox] (MaxPool2d(1, 2) of the block input)
      if (mval)
        e_res = *reinterpret_cast<const f4*>(p.res + b * p.res_H * p.res_W * Cout +
                                             (oy * S * p.res_W + ox * S) * (rbk ? 16 : Cout) +
                                             cb * (rbk ? p.res_H * p.res_W * 16 : 16) + 4 * q);
  }
  // pre-BN scale / shift into LDS while the first fragments are in flight
  if constexpr (PRE) {
    for (int c = tid; c < Cin; c += 64 * NWV) {
      pst[c] = p.pre_scale[c];
      pst[MAXC + c] = p.pre_shift[c];
    }
    __syncthreads();
  }
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  for (int i0 = 0; i0 < nI; i0 += CH) {
#pragma unroll
    for (int d = 0; d < CH; ++d) {
      const f4 a = wa[d];
      f4 v = xa[d];
      if constexpr (PRE) {
        // BN(x) at in-image taps (the conv's zero padding stays 0)
        const int me = mt[d];
        const int c = me & 0xffff;
        const f4 sc = *reinterpret_cast<const f4*>(pst + c), sh = *reinterpret_cast<const f4*>(pst + MAXC + c);
        const f4 t = __builtin_elementwise_fma(v, sc, sh);
        v = (me >> 16) ? t : f4{0.f, 0.f, 0.f, 0.f};
      }
      f4& ac = acc[d & 1];
      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, v.x, ac, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, v.y, ac, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, v.z, ac, 0, 0, 0);
      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, v.w, ac, 0, 0, 0);
      // refill the slot with the wave's chunk i0 + d + CH (out of range: zeros, never read)
      int wo, xo, me;
      next_frag(wo, xo, me);
      wa[d] = ld4(wr, wo);
      xa[d] = ld4(xr, xo);
      mt[d] = me;
    }
  }
#pragma unroll
  for (int k = 0; k < SCMAX; ++k) {
    f4& ac = acc[k & 1];
    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(swa[k].x, sxa[k].x, ac, 0, 0, 0);
    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(swa[k].y, sxa[k].y, ac, 0, 0, 0);
    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(swa[k].z, sxa[k].z, ac, 0, 0, 0);
    ac = __builtin_amdgcn_mfma_f32_16x16x4f32(swa[k].w, sxa[k].w, ac, 0, 0, 0);
  }
  f4 sum = acc[0] + acc[1];
  if (w > 0) red[w - 1][lane] = sum;
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int k = 0; k < NWV - 1; ++k) sum += red[k][lane];
  // epilogue: lane holds couts c4 .. c4 + 3 of pixel m
  if (!mval) return;
  f4 v = __builtin_elementwise_fma(sum, e_sc, e_sh);
  if constexpr (EPI == EPI_AFFINE_PRELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] > 0.f ? v[k] : v[k] * e_al[k];
  }
  if constexpr (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_SUB) v += e_res;
  const long long ybytes = (long long)p.M * Cout * 4;
  __builtin_amdgcn_raw_buffer_store_b128(bits4(v), rsrc(p.y, ybytes), yoff * 4, 0, CPOL_SC1);
  if (p.y2)
    __builtin_amdgcn_raw_buffer_store_b128(bits4(__builtin_elementwise_fma(v, e_s2, e_t2)), rsrc(p.y2, ybytes), yoff * 4,
                                           0, CPOL_SC1);
}

__global__ __launch_bounds__(256) void convs_weights_kernel(const float* __restrict__ w, float* __restrict__ wf,
                                                          int Cout, int KR) {
  const int NK = KR >> 4;
  const long long i = blockIdx.x * 256ll + threadIdx.x;  // one 16-byte fragment per thread
  if (i >= (long long)(Cout >> 4) * NK * 64) return;
  const int l = (int)(i & 63);
  const long long t = i >> 6;
  const int kc = (int)(t % NK), cb = (int)(t / NK);
  *reinterpret_cast<f4*>(wf + i * 4) =
      *reinterpret_cast<const f4*>(w + (long long)(cb * 16 + (l & 15)) * KR + kc * 16 + 4 * (l >> 4));
}

}  // namespace

hipError_t launch_convs_weights(const float* w, float* wf, int Cout, int KR, hipStream_t s) {
  if (!w || !wf || Cout <= 0 || KR <= 0 || Cout % 16 || KR % 16) return hipErrorInvalidValue;
  const long long n = (long long)Cout * KR / 4;
  hipLaunchKernelGGL(convs_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, wf, Cout, KR);
  return hipGetLastError();
}

bool convs_supported(const ConvParams& p, bool pre, Epi epi) {
  const bool epi_ok = epi == EPI_AFFINE_PRELU ||
                      (!pre && (epi == EPI_AFFINE || epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_SUB));
  return epi_ok && p.KH == 3 && p.KW == 3 && p.pad == 1 && (p.stride == 1 || p.stride == 2) && p.Cin % 16 == 0 &&
         p.Cout % 16 == 0 && p.Cin2 % 16 == 0 && p.Cin2 <= 16 * NWV * SCMAX && (p.Cin2 == 0 || p.x2) && (!pre || p.Cin <= MAXC) && p.M >= 1 &&
         (long long)p.B * p.H * p.W * std::max(p.Cin, p.Cin2) * 4 < BIGOFF &&
         (long long)p.Cout * (9 * p.Cin + p.Cin2) * 4 < BIGOFF;
}

hipError_t launch_convs(const ConvParams& p, bool pre, Epi epi, hipStream_t s) {
  if (!convs_supported(p, pre, epi) || !p.x || !p.w || !p.y || !p.post_scale || !p.post_shift ||
      (epi == EPI_AFFINE_PRELU && !p.prelu) || ((epi == EPI_AFFINE_RES || epi == EPI_AFFINE_RES_SUB) && !p.res) ||
      (p.y2 && (!p.y2_scale || !p.y2_shift)))
    return hipErrorInvalidValue;
  const int grid = ((p.M + 15) / 16) * (p.Cout / 16);
  if (pre)
    hipLaunchKernelGGL((convs_kernel<true, EPI_AFFINE_PRELU>), dim3(grid), dim3(64 * NWV), 0, s, p);
  else if (epi == EPI_AFFINE_PRELU)
    hipLaunchKernelGGL((convs_kernel<false, EPI_AFFINE_PRELU>), dim3(grid), dim3(64 * NWV), 0, s, p);
  else if (epi == EPI_AFFINE)
    hipLaunchKernelGGL((convs_kernel<false, EPI_AFFINE>), dim3(grid), dim3(64 * NWV), 0, s, p);
  else if (epi == EPI_AFFINE_RES)
    hipLaunchKernelGGL((convs_kernel<false, EPI_AFFINE_RES>), dim3(grid), dim3(64 * NWV), 0, s, p);
  else
    hipLaunchKernelGGL((convs_kernel<false, EPI_AFFINE_RES_SUB>), dim3(grid), dim3(64 * NWV), 0, s, p);
  return hipGetLastError();
}

}  // namespace frhip
