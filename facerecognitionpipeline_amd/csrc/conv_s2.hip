// Stride-2 3x3 conv of the first stage-1 block, Conv2d(64, 64, 3, stride 2, pad 1) + BN + the
// MaxPool2d(1, 2) shortcut (net.BasicBlockIR res_layer[4] + shortcut_layer of an AdaFace unit whose
// width does not change, reached through `self.model(batch)`, face_embedder.py:157), NHWC f32, on
// v_mfma_f32_16x16x4_f32, as a band kernel.
//
// Why a kernel of its own: on the implicit-GEMM kernel this layer (N = 64 output channels, input
// streamed from HBM at stride 2) ran at 58% of the fp32 MFMA peak -- each 32-channel K-step
// re-gathers its 128 output pixels' taps through L1/L2 and there are only 64 columns to reuse
// them over.  Here a workgroup owns a BAND of two output rows of one image (112 pixels x 64
// couts): the five input rows the band's 3x3 windows touch are staged once per 32-channel half in
// LDS (5 x 113 pixels x 32 channels, pixel pitch 36 floats: 16-byte aligned, and a stride-2 gather
// of 16 pixels touches every bank at most twice), and all 9 taps read them from there.
//   * 4 waves, wave w owns couts 16w .. 16w+15 for all 112 pixels (7 blocks of 16): the weights
//     are the MFMA's A operand (16 couts x 4 channels per lane fragment, one 16-byte L2 load per
//     tap and 16 channels), the staged input its B operand (16 pixels x 4 channels: one
//     ds_read_b128 per pixel block, tap and 16 channels).  A lane's accumulator then holds 4
//     consecutive couts of one output pixel: one 16-byte store per pixel.
//   * MFMA e (0..3) of a 16-channel chunk consumes channels 4q + e (q = lane / 16) of both
//     operands, so each lane reads 4 consecutive channels with one 16-byte access.
//   * persistent, 2 workgroups per CU (79.5 KB of LDS each); the next half's input is fetched into
//     registers while this half's MFMAs run.
// Numerics: exact f32 products, f32 accumulation (MFMA = fmaf chain); only the order of the K
// sum differs from the direct kernel / the CPU reference.
#include <algorithm>

#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 64;          // input = output channels
constexpr int HALF = 32;       // channels staged per pass
constexpr int PITCH = 36;      // LDS floats per staged pixel (32 channels + 4: aligned, 2-way gathers)
constexpr int ROWPX = 113;     // staged pixels per row (input columns -1 .. 111)
constexpr int BROWS = 5;       // input rows of a band of 2 output rows
constexpr int NBLK = 7;        // 16-pixel blocks of a band (2 x 56 output pixels)
constexpr int BIGOFF = 0x7F000000;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* ptr, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f4 ld4(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}

#ifndef S2_WLEAD
#define S2_WLEAD 4
#endif
constexpr int WLEAD = S2_WLEAD;  // weight fragments in flight ahead of their step
constexpr int NSTG = (BROWS * ROWPX * (HALF / 4) + 255) / 256;  // staged float4 per thread and half

// Persistent: workgroup g takes bands g, g + gridDim.x, ... (band = 2 output rows of one image).
// Per band and 32-channel half: the NEXT half's (or band's) input is fetched into registers, one
// float4 per MFMA step, while this half's MFMAs run, and written to LDS between two barriers when
// they are done.  Buffer loads retire in issue order (one vmcnt), so each step's weight fragment
// is issued two steps ahead and BEFORE that step's staging load.  256 threads.
__global__ __launch_bounds__(256, 2) void s2c64_kernel(S2Params p) {
  __shared__ __attribute__((aligned(16))) float band[BROWS * ROWPX * PITCH];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Hi = p.H, Wi = p.W, Ho = p.Ho, Wo = p.Wo;
  const int nb2 = (Ho + 1) / 2, nbands = p.B * nb2;
  const int cols = 2 * Wo + 1;  // staged input columns -1 .. 2 Wo - 1
  const __amdgpu_buffer_rsrc_t xr = rsrc(p.x, (long long)p.B * Hi * Wi * C * 4);
  const __amdgpu_buffer_rsrc_t wr = rsrc(p.w, (long long)C * 9 * C * 4);
  const __amdgpu_buffer_rsrc_t rr = rsrc(p.res, (long long)p.B * Hi * Wi * C * 4);
  const __amdgpu_buffer_rsrc_t yr = rsrc(p.y, (long long)p.B * Ho * Wo * C * 4);

  // the lane's output pixel of each block: band pixel p = 16 blk + (lane & 15) = (row oyl, col ox)
  // -> staged pixel of tap (0, 0): row 2 oyl, column 2 ox (staged column = input column + 1)
  const int q = lane >> 4;
  int pbase[NBLK];
#pragma unroll
  for (int k = 0; k < NBLK; ++k) {
    const int pp = 16 * k + (lane & 15);
    const bool valid = pp < 2 * Wo;  // (a band pixel past 2 Wo gathers pixel 0's taps; never stored)
    const int oyl = valid && pp >= Wo ? 1 : 0, ox = valid ? pp - oyl * Wo : 0;
    pbase[k] = ((2 * oyl) * ROWPX + 2 * ox) * PITCH + 4 * q;
  }
  // weight fragment of (tap, 16-channel chunk): cout 16 w + (lane & 15), channels chunk + 4 q .. +3
  const int wrow = ((16 * w + (lane & 15)) * 9) * C * 4 + 16 * q;

  // staging of input rows 2 oy0 - 1 .. 2 oy0 + 3, columns -1 .. 2 Wo - 1, channels 32 h .. +31
  // (zero outside the image -- the conv's padding -- through out-of-range buffer offsets)
  // per staged float4 u of this thread, band-independent and packed so that the per-band
  // address math stays 18 registers:  bits 0..17 byte offset of (row r, staged column cx, c4)
  // relative to the band's row -1 / column -1,  bits 18..20 r,  bit 21 valid (inside the staged
  // window and not the left padding column)
  int pk[NSTG];
#pragma unroll
  for (int u = 0; u < NSTG; ++u) {
    const int i = tid + 256 * u;
    const int c4 = i & 7, px = i >> 3;
    const int r = px / cols, cx = px - r * cols;
    const bool v = i < BROWS * cols * 8 && cx >= 1;
    pk[u] = ((r * Wi + cx) * C + 4 * c4) * 4 | r << 18 | (v ? 1 << 21 : 0);
  }
  f4 stg[NSTG];
  // (bi >= nbands: no band left; the load is issued anyway, out of range -- a branch around it
  // would make the compiler's vmcnt bookkeeping assume the shorter queue and wait on the staging)
  auto fetch1 = [&](int u, int bi, int h) {
    int k = pk[u];
    asm volatile("" : "+v"(k));  // decode per use: keeps LICM from hoisting 18 x 3 decoded values
    const int b = bi / nb2, iy0 = 4 * (bi - b * nb2) - 1;
    const int r = (k >> 18) & 7, iy = iy0 + r;
    const bool in = (k & (1 << 21)) && (unsigned)iy < (unsigned)Hi && bi < nbands;
    const int base = ((b * Hi + iy0) * Wi - 1) * C * 4 + HALF * h * 4;
    stg[u] = ld4(xr, in ? base + (k & 0x3FFFF) : BIGOFF);
  };
  auto commit = [&]() {
#pragma unroll
    for (int u = 0; u < NSTG; ++u) {
      const int i = tid + 256 * u;
      if (i < BROWS * cols * 8) {
        const int c4 = i & 7, px = i >> 3, r = (pk[u] >> 18) & 7;
        *reinterpret_cast<f4*>(band + (px + r * (ROWPX - cols)) * PITCH + 4 * c4) = stg[u];
      }
    }
  };
  static_assert(NSTG == 18, "one staged float4 per (tap, 16-channel chunk) step");

  // weight fragment of step s (0..35 = half, tap, 16-channel chunk); the same for every band, so
  // one ring runs across halves and bands, WLEAD steps ahead
  auto wload = [&](int s) {
    const int h = s / 18, t = s - 18 * h;
    return ld4(wr, wrow + ((t >> 1) * C + HALF * h + 16 * (t & 1)) * 4);
  };
  f4 wf[36];
#pragma unroll
  for (int s = 0; s < WLEAD; ++s) wf[s] = wload(s);

  int bi = blockIdx.x;
#pragma unroll
  for (int u = 0; u < NSTG; ++u) fetch1(u, bi, 0);
  for (; bi < nbands; bi += gridDim.x) {
    const int b = bi / nb2, oy0 = 2 * (bi - b * nb2);
    f4 acc[NBLK];
#pragma unroll
    for (int k = 0; k < NBLK; ++k) acc[k] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // every wave is done with the staged half it read last
      commit();
      __syncthreads();
      // the next half (or the next band's first half) to stage
      const int nbi = h == 0 ? bi : bi + (int)gridDim.x, nh = h ^ 1;
      auto toff = [](int t) {
        const int tap = t >> 1, c16 = t & 1, ky = tap / 3, kx = tap - 3 * ky;
        return (ky * ROWPX + kx) * PITCH + 16 * c16;
      };
      f4 bv[NBLK];
#pragma unroll
      for (int k = 0; k < NBLK; ++k) bv[k] = *reinterpret_cast<const f4*>(band + pbase[k] + toff(0));
#pragma unroll
      for (int t = 0; t < 18; ++t) {
        // issue order per step: the weights of step s + WLEAD, then one float4 of the next
        // staging; waiting for step s's weights then covers only staging loads issued at least
        // WLEAD steps earlier
        const int s = 18 * h + t;
        wf[(s + WLEAD) % 36] = wload((s + WLEAD) % 36);
        fetch1(t, nbi, nh);
        // channel e of every block before channel e + 1: consecutive MFMAs never chain on one
        // accumulator (a 16x16x4 f32 result is not ready for the next MFMA at issue rate).  A
        // block's fragment of step t + 1 is read from LDS right after its last MFMA of step t,
        // so the read's latency hides behind the step's remaining MFMAs, not at the step's start.
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
          for (int k = 0; k < NBLK; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[s][e], bv[k][e], acc[k], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < NBLK; ++k) {
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[s][3], bv[k][3], acc[k], 0, 0, 0);
          if (t + 1 < 18) bv[k] = *reinterpret_cast<const f4*>(band + pbase[k] + toff(t + 1));
        }
      }
    }
    // epilogue: lane holds couts 16 w + 4 q .. +3 of band pixel 16 blk + (lane & 15)
    const int co = 16 * w + 4 * q;
    const f4 sc = *reinterpret_cast<const f4*>(p.post_scale + co);
    const f4 sh = *reinterpret_cast<const f4*>(p.post_shift + co);
#pragma unroll
    for (int k = 0; k < NBLK; ++k) {
      const int pp = 16 * k + (lane & 15);
      const int oyl = pp >= Wo ? 1 : 0, ox = pp - oyl * Wo, oy = oy0 + oyl;
      const bool in = pp < 2 * Wo && oy < Ho;
      // y = BN(conv) + x[b, 2 oy, 2 ox] (MaxPool2d(1, 2) of the block input)
      const int ro = in ? (((b * Hi + 2 * oy) * Wi + 2 * ox) * C + co) * 4 : BIGOFF;
      const int yo = in ? (((b * Ho + oy) * Wo + ox) * C + co) * 4 : BIGOFF;
      f4 v = acc[k] * sc + sh;
      v += ld4(rr, ro);
      const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
      __builtin_amdgcn_raw_buffer_store_b128(bits, yr, yo, 0, 0);
    }
  }
}

}  // namespace

bool s2c64_supported(int Cin, int Cout, int kh, int kw, int stride, int pad, int H, int W) {
  return Cin == C && Cout == C && kh == 3 && kw == 3 && stride == 2 && pad == 1 && H % 2 == 0 && W % 2 == 0 &&
         W / 2 <= 56 && W / 2 >= 8;
}

hipError_t launch_s2c64(const S2Params& p0, hipStream_t s) {
  S2Params p = p0;
  if (!s2c64_supported(C, C, 3, 3, 2, 1, p.H, p.W) || p.B < 1 || !p.x || !p.w || !p.y || !p.res ||
      !p.post_scale || !p.post_shift || (long long)p.B * p.H * p.W * C * 4 >= BIGOFF)
    return hipErrorInvalidValue;
  p.Ho = p.H / 2;
  p.Wo = p.W / 2;
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (cus <= 0) cus = 256;
  const int nbands = p.B * ((p.Ho + 1) / 2);
  hipLaunchKernelGGL(s2c64_kernel, dim3(std::min(nbands, 2 * cus)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace frhip
