// Winograd F(2x2, 3x3) convolution in f32 on gfx950 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the stride-1 3x3 Conv2d of net.BasicBlockIR (res_layer[1] and the
// stride-1 res_layer[4]; reached through `self.model(batch)`, face_embedder.py:157)
// with the same fused pre-BN / post-BN / PReLU / residual epilogues as the direct
// implicit-GEMM kernel (conv_mfma_impl.h).  The arithmetic stays f32 throughout;
// the algorithm trades 36 multiplies per 2x2 output tile and (cin, cout) pair for 16
// (Lavin & Gray 2016), so the MFMA work of a layer drops 2.25x:
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A     d: 4x4 input patch, g: 3x3 filter
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   G   = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
//
// Per transform element xi = 4a + b (16 of them) the layer is one GEMM
//   M_xi[tile][cout] = sum_cin V_xi[tile][cin] * U_xi[cin][cout]
// and one workgroup owns WT = 32 tiles x BN = 32*NBW output channels for all 16.
//
//   * 8 waves; wave w owns xi = 2w, 2w+1 and the whole 32 x BN tile of both, so its
//     accumulators are 2 x NBW 32x32 MFMA blocks (32*NBW VGPRs) and no operand it reads
//     is read by any other wave.
//   * K-step = 16 input channels.  Thread (tile, channel group cg of 4, patch column j)
//     loads its patch column as 4 x 16-B buffer loads (OOB offset -> 0 = zero padding;
//     the pre-BN affine is applied only to in-image taps), mixes rows in registers and
//     columns across its lane quad (DPP quad_perm), and writes 4 x float4 of V to LDS
//     V[xi][tile][ch] (rows of 20 floats: the ds_read_b128 fragment reads are
//     conflict-free; planes 648 floats apart: so are the ds_write_b128).  The transform is
//     shared by all 16 GEMMs, which is why the 16 live in one workgroup.
//   * U (transformed filters, built once per model by wino_weight_kernel) never
//     touches LDS: it is pre-permuted in HBM into MFMA-fragment order, so each wave
//     fetches its own B fragments with fully coalesced 1 KiB buffer loads.
//   * Software pipeline, one barrier per K-step: during step s the wave issues the
//     loads of patch s+2 and U(s+1), runs the MFMAs of s, and in their shadow
//     transforms patch s+1 (loaded a whole step earlier) into the other LDS buffer.
//     The step body is branch-free (steps past the end load through OOB offsets), so
//     sched_group_barrier can interleave loads, transform VALU and LDS writes with the
//     MFMAs.
//   * Epilogue: residuals are prefetched, accumulators go through LDS (M[xi][tile][cout],
//     one 32-column half at a time), each thread inverse-transforms (tile, cout) pairs
//     and applies BN (+PReLU | + residual) at the <= 4 in-image pixels of the tile.
//
// Lane map of 32x32x2 MFMA: A operand lane (m = l%32, h = l/32) = A[m][k=h], B operand
// lane (n = l%32, h) = B[k=h][n].  We permute the 16 channels of a K-step so that MFMA
// j (0..7) multiplies channel 8h + j: lane (m, h) reads V[xi][m][8h .. 8h+7] with two
// ds_read_b128 and the matching 8 U values with two 16-B loads.
#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int WT = 32;             // 2x2 output tiles per workgroup (MFMA M)
constexpr int WKC = 16;            // input channels per K-step
constexpr int VROW = 20;           // LDS floats per (xi, tile) row: 16 channels + 4 pad
constexpr int VPLANE = WT * VROW + 8;  // one xi plane; 648 = 8 mod 32: conflict-free b128 writes
constexpr int VBUF = 16 * VPLANE;  // one K-step of V (40 KiB)
constexpr int MROW = 33;           // epilogue staging row: 32 couts + 1
constexpr int MPLANE = WT * MROW;
constexpr int OOB = 0x80000000;    // buffer offset past any range: loads return 0
static_assert(16 * MPLANE <= 2 * VBUF, "epilogue staging must fit the V buffers");

__device__ __forceinline__ int wino_xcd_remap(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Buffer descriptor from provably wave-uniform inputs (readfirstlane), so the compiler
// keeps it in SGPRs instead of wrapping every buffer op in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* ptr, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(ptr);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), (short)0, n,
                                           0x00020000);
}

template <int NBW, bool PRE, int EPI>
__global__ __launch_bounds__(512, 1) void wino_kernel(WinoParams p) {
  constexpr int BN = 32 * NBW;
  constexpr bool RES = EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU;
  __shared__ __attribute__((aligned(16))) float lds[2 * VBUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int t = wino_xcd_remap(blockIdx.x, p.mblocks * p.nblocks);
  const int mb = t % p.mblocks, nb = t / p.mblocks;
  const int H = p.H, W = p.W, Cin = p.Cin;
  const int per_img = p.TH * p.TW;
  const int KS = Cin / WKC;
  const int NB32 = p.Cout / 32;

  // ---- transform role: thread (tile, channel group of 4, patch column j) ------------
  // lane = j + 4*cg + 16*tile_in_wave: a quad holds the 4 columns of one (tile, cg), so
  // the column half of the transform is a DPP quad exchange.
  const int tj = tid & 3, tcg = (tid >> 2) & 3, tl = tid >> 4;
  const int T = mb * WT + tl;
  int base = 0;
  unsigned mask = 0;  // bit i: patch pixel (row i, column tj) is inside the image
  if (T < p.ntiles) {
    const int n = T / per_img;
    const int r = T - n * per_img;
    const int ty = r / p.TW, tx = r - ty * p.TW;
    const int y0 = 2 * ty - 1, x = 2 * tx - 1 + tj;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((unsigned)(y0 + i) < (unsigned)H && (unsigned)x < (unsigned)W) mask |= 1u << i;
    base = (((n * H + y0) * W + x) * Cin + 4 * tcg) * 4;  // only used at in-image taps
  }
  const int rowb = W * Cin * 4;
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x, p.B * H * W * Cin * 4);
  const __amdgpu_buffer_rsrc_t ur = uniform_rsrc(p.u, 16 * p.Cout * Cin * 4);
  auto f4 = [](u32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
  };

  // per-lane offsets fixed for the whole K loop (OOB for out-of-image pixels); the K-step
  // enters as a scalar soffset.  Prefetches past the last step re-load the last step
  // (clamped), so no lane ever needs a per-step range select.
  int voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) voff[i] = ((mask >> i) & 1u) ? base + i * rowb : OOB;
  const __amdgpu_buffer_rsrc_t pr = uniform_rsrc(p.pre_scale, PRE ? Cin * 4 : 0);
  const __amdgpu_buffer_rsrc_t qr = uniform_rsrc(p.pre_shift, PRE ? Cin * 4 : 0);
  auto load_in = [&](float4 (&d)[4], float4 (&ps)[2], int s) {
    const int so = min(s, KS - 1) * WKC * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = f4(__builtin_amdgcn_raw_buffer_load_b128(xr, voff[i], so, 0));
    if constexpr (PRE) {
      ps[0] = f4(__builtin_amdgcn_raw_buffer_load_b128(pr, 16 * tcg, so, 0));
      ps[1] = f4(__builtin_amdgcn_raw_buffer_load_b128(qr, 16 * tcg, so, 0));
    }
  };
  // V = B^T d B for this thread's column: rows mixed in registers (B^T d), columns
  // mixed across the quad: V[.][j] = sa*(r[.][j] + c*r[.][partner]), partner = (2,2,1,1)[j],
  // c = (-1, 1, -1, -1)[j], sa = -1 for j = 3 only.  sa is folded into the filters (U of
  // the b = 3 transform elements is stored negated), so each element is one fma whose
  // DPP operand the compiler folds into v_fmac_f32_dpp.
  const float cq = tj == 1 ? 1.f : -1.f;
  auto store_v = [&](const float4 (&d)[4], const float4 (&ps)[2], int buf) {
    float4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = d[i];
      if constexpr (PRE) {
        const bool ok = (mask >> i) & 1u;
        v[i].x = ok ? v[i].x * ps[0].x + ps[1].x : 0.f;
        v[i].y = ok ? v[i].y * ps[0].y + ps[1].y : 0.f;
        v[i].z = ok ? v[i].z * ps[0].z + ps[1].z : 0.f;
        v[i].w = ok ? v[i].w * ps[0].w + ps[1].w : 0.f;
      }
    }
    float4 r[4];
    r[0] = v[0] - v[2];
    r[1] = v[1] + v[2];
    r[2] = v[2] - v[1];
    r[3] = v[1] - v[3];
    float* dst = lds + buf * VBUF + tj * VPLANE + tl * VROW + 4 * tcg;
    auto mix = [&](float x) {
      const float o = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x5A, 0xF, 0xF, true));
      return __builtin_fmaf(o, cq, x);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float4*>(dst + 4 * i * VPLANE) = make_float4(mix(r[i].x), mix(r[i].y), mix(r[i].z), mix(r[i].w));
  };

  // ---- GEMM role: wave wid owns xi = 2*wid + xl ----------------------------------------
  // U fragment (xi, 32-col block, K-step s, half q): 64 lanes x float4, contiguous 1 KiB.
  typedef float4 ufrag[2][NBW][2];
  int ubase[2][NBW];
#pragma unroll
  for (int xl = 0; xl < 2; ++xl)
#pragma unroll
    for (int b = 0; b < NBW; ++b) ubase[xl][b] = (((2 * wid + xl) * NB32 + nb * NBW + b) * KS * 2 * 64 + lane) * 16;
  auto load_u = [&](ufrag& u, int s) {
    const int so = min(s, KS - 1) * 2 * 64 * 16;
#pragma unroll
    for (int xl = 0; xl < 2; ++xl)
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          u[xl][b][q] = f4(__builtin_amdgcn_raw_buffer_load_b128(ur, ubase[xl][b] + q * 64 * 16, so, 0));
  };

  floatx16 acc[2][NBW];
#pragma unroll
  for (int xl = 0; xl < 2; ++xl)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[xl][b][e] = 0.f;

  // One K-step s.  On entry: V(s) in LDS buffer `buf`, patch s+1 in `dc` (loaded a step
  // ago), U(s) in `uc`.  Issues the loads of patch s+2 (into `dn`, free since V(s) was
  // written) and U(s+1), runs the MFMAs of s and, in their shadow, transforms patch s+1
  // into the other LDS buffer; one barrier.
  auto step = [&](int s, const ufrag& uc, ufrag& un, const float4 (&dc)[4], const float4 (&pc)[2],
                  float4 (&dn)[4], float4 (&pn)[2], int buf) {
    // U(s+1) first: vmcnt retires in issue order, so the wait for U at the top of the next
    // step must not also wait for this step's patch loads (which may come from HBM)
    load_u(un, s + 1);
    load_in(dn, pn, s + 2);
    const float* vb = lds + buf * VBUF + (lane & 31) * VROW + 8 * (lane >> 5);
    float4 a[2][2];
#pragma unroll
    for (int xl = 0; xl < 2; ++xl) {
      const float* vx = vb + (2 * wid + xl) * VPLANE;
      a[xl][0] = *reinterpret_cast<const float4*>(vx);
      a[xl][1] = *reinterpret_cast<const float4*>(vx + 4);
    }
#pragma unroll
    for (int xl = 0; xl < 2; ++xl)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          acc[xl][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[xl][j >> 2][j & 3], uc[xl][b][j >> 2][j & 3],
                                                            acc[xl][b], 0, 0, 0);
    store_v(dc, pc, buf ^ 1);
    // 4 fragment reads up front; then per MFMA: a share of the loads, of the transform
    // VALU and (in the second half) of its 16 LDS writes
    constexpr int NMFMA = 16 * NBW;
    constexpr int NVMEM = 4 + 4 * NBW + (PRE ? 2 : 0);
    constexpr int VM_PER = (NVMEM + NMFMA - 1) / NMFMA;
    constexpr int VALU_PER = PRE ? 8 : 4;
    constexpr int DSW_FROM = NMFMA / 2;
    constexpr int DSW_PER = (4 + (NMFMA - DSW_FROM) - 1) / (NMFMA - DSW_FROM);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int i = 0; i < NMFMA; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, VM_PER, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, VALU_PER, 0);
      if (i >= DSW_FROM) __builtin_amdgcn_sched_group_barrier(0x200, DSW_PER, 0);
    }
    __syncthreads();
    // nothing crosses a step boundary: VALU of the next step hoisted above the barrier
    // would wait on loads issued in this one
    __builtin_amdgcn_sched_barrier(0);
  };

  float4 dA[4], dB[4], pA[2], pB[2];
  ufrag uA, uB;
  load_in(dA, pA, 0);
  load_u(uA, 0);
  load_in(dB, pB, 1);
  store_v(dA, pA, 0);
  __syncthreads();
  for (int s = 0; s < KS; s += 2) {  // KS is even (Cin % 32 == 0)
    step(s, uA, uB, dB, pB, dA, pA, 0);
    step(s + 1, uB, uA, dA, pA, dB, pB, 1);
  }

  // ---- epilogue: inverse transform + BN (+PReLU | +residual) -------------------------
  const int ec = tid & 31;  // cout within a 32-column half
  // per tile slot q: top-left output pixel and the in-image mask of its 4 pixels; the
  // residuals are loaded before the staging barrier so their latency overlaps it
  int pix[2], okm[2];
  float rv[NBW][2][4];
  const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.res, RES ? p.B * H * W * p.Cout * 4 : 0);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int Tq = mb * WT + (tid >> 5) + 16 * q;
    const int n = Tq / per_img;
    const int r = Tq - n * per_img;
    const int ty = r / p.TW, tx = r - ty * p.TW;
    const int ok = Tq < p.ntiles ? 1 : 0;
    const int oky1 = ok & (2 * ty + 1 < H ? 1 : 0), okx1 = ok & (2 * tx + 1 < W ? 1 : 0);
    okm[q] = ok | (okx1 << 1) | (oky1 << 2) | ((oky1 & okx1) << 3);
    pix[q] = (n * H + 2 * ty) * W + 2 * tx;
#pragma unroll
    for (int b = 0; b < NBW; ++b) {
      const int cout = nb * BN + b * 32 + ec;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rv[b][q][e] = 0.f;
        if constexpr (RES) {
          const int o = (pix[q] + (e >> 1) * W + (e & 1)) * p.Cout + cout;
          rv[b][q][e] =
              __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rr, ((okm[q] >> e) & 1) ? o * 4 : OOB, 0, 0));
        }
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    if (b > 0) __syncthreads();
#pragma unroll
    for (int xl = 0; xl < 2; ++xl) {
      float* dst = lds + (2 * wid + xl) * MPLANE + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * MROW] = acc[xl][b][r];
    }
    __syncthreads();
    const int cout = nb * BN + b * 32 + ec;
    const float sc = p.post_scale[cout], sh = p.post_shift[cout];
    float al = 0.f;
    if constexpr (EPI == EPI_AFFINE_PRELU || EPI == EPI_AFFINE_RES_PRELU) al = p.prelu[cout];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int tile = (tid >> 5) + 16 * q;
      float m[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) m[e] = lds[e * MPLANE + tile * MROW + ec];
      float t0[4], t1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t0[j] = m[j] + m[4 + j] + m[8 + j];
        t1[j] = m[4 + j] - m[8 + j] - m[12 + j];
      }
      float yv[4];
      yv[0] = t0[0] + t0[1] + t0[2];
      yv[1] = t0[1] - t0[2] - t0[3];
      yv[2] = t1[0] + t1[1] + t1[2];
      yv[3] = t1[1] - t1[2] - t1[3];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (!((okm[q] >> e) & 1)) continue;
        const int o = (pix[q] + (e >> 1) * W + (e & 1)) * p.Cout + cout;
        float v = yv[e] * sc + sh;
        if constexpr (EPI == EPI_AFFINE_PRELU) v = v > 0.f ? v : v * al;
        if constexpr (EPI == EPI_AFFINE_RES) v += rv[b][q][e];
        if constexpr (EPI == EPI_AFFINE_RES_PRELU) {
          v += rv[b][q][e];
          v = v > 0.f ? v : v * al;
        }
        p.y[o] = v;
      }
    }
  }
}

// G g G^T of every (cout, cin) filter, in double then rounded once to f32, scattered
// into the fragment order wino_kernel reads: [xi][Cout/32][Cin/16][q][lane][4] with
// lane = 32*(c/8) + cout%32, q = (c%8)/4, element = c%4 for c = cin%16.
__global__ void wino_weight_kernel(const float* __restrict__ w, float* __restrict__ u, int Cout, int Cin) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Cout * Cin) return;
  const int o = idx / Cin, i = idx - o * Cin;
  double g[3][3];
#pragma unroll
  for (int y = 0; y < 3; ++y)
#pragma unroll
    for (int x = 0; x < 3; ++x) g[y][x] = w[((long long)(o * 3 + y) * 3 + x) * Cin + i];
  double tg[4][3];
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    tg[0][x] = g[0][x];
    tg[1][x] = 0.5 * (g[0][x] + g[1][x] + g[2][x]);
    tg[2][x] = 0.5 * (g[0][x] - g[1][x] + g[2][x]);
    tg[3][x] = g[2][x];
  }
  const int NB32 = Cout / 32, KS = Cin / 16;
  const int nb32 = o >> 5, n = o & 31;
  const int s = i >> 4, c = i & 15;
  const int ln = 32 * (c >> 3) + n, q = (c & 7) >> 2, e = c & 3;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    double ua[4];
    ua[0] = tg[a][0];
    ua[1] = 0.5 * (tg[a][0] + tg[a][1] + tg[a][2]);
    ua[2] = 0.5 * (tg[a][0] - tg[a][1] + tg[a][2]);
    ua[3] = tg[a][2];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int xi = 4 * a + b;
      // b = 3 stored negated: wino_kernel's input transform produces -V for that column
      u[((((long long)(xi * NB32 + nb32) * KS + s) * 2 + q) * 64 + ln) * 4 + e] = (float)(b == 3 ? -ua[b] : ua[b]);
    }
  }
}

}  // namespace

bool wino_supported(int Cin, int Cout, int kh, int kw, int stride, int pad) {
  return kh == 3 && kw == 3 && stride == 1 && pad == 1 && Cin % 32 == 0 && Cin >= 32 && Cout % 32 == 0 &&
         Cout >= 32;
}

hipError_t launch_wino_weights(const float* w, float* u, int Cout, int Cin, hipStream_t s) {
  if (Cout % 32 || Cin % 32) return hipErrorInvalidValue;
  const int n = Cout * Cin;
  hipLaunchKernelGGL(wino_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, w, u, Cout, Cin);
  return hipGetLastError();
}

hipError_t launch_wino(const WinoParams& p0, bool pre, Epi epi, hipStream_t s) {
  WinoParams p = p0;
  if (!wino_supported(p.Cin, p.Cout, 3, 3, 1, 1) || p.B < 1 || p.H < 1 || p.W < 1 ||
      (long long)p.B * p.H * p.W * p.Cin * 4 >= (1ll << 31) ||
      (long long)p.B * p.H * p.W * p.Cout * 4 >= (1ll << 31) || (long long)16 * p.Cout * p.Cin * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  p.TH = (p.H + 1) / 2;
  p.TW = (p.W + 1) / 2;
  p.ntiles = p.B * p.TH * p.TW;
  p.mblocks = (p.ntiles + WT - 1) / WT;
  const int nbw = (p.Cout % 64 == 0) ? 2 : 1;
  p.nblocks = p.Cout / (32 * nbw);
  const dim3 grid(p.mblocks * p.nblocks), block(512);
#define FR_WINO_CASE(NBW_, PRE_, EPI_)                                         \
  if (nbw == NBW_ && pre == PRE_ && epi == EPI_) {                             \
    hipLaunchKernelGGL((wino_kernel<NBW_, PRE_, EPI_>), grid, block, 0, s, p); \
    return hipGetLastError();                                                  \
  }
  FR_WINO_CASE(2, true, EPI_AFFINE_PRELU)
  FR_WINO_CASE(2, false, EPI_AFFINE_RES)
  FR_WINO_CASE(1, true, EPI_AFFINE_PRELU)
  FR_WINO_CASE(1, false, EPI_AFFINE_RES)
#undef FR_WINO_CASE
  return hipErrorInvalidValue;
}

size_t wino_weight_floats(int Cout, int Cin) { return (size_t)16 * Cout * Cin; }

}  // namespace frhip
