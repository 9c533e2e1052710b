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
//   * K-step = 16 input channels.  Thread (tile = tid/16, ch = tid%16) loads the 4x4
//     patch of its tile at its channel (buffer loads: OOB offset -> 0 = zero padding;
//     the pre-BN affine is applied only to in-image taps), transforms it with 32 adds
//     and writes the 16 V values to LDS V[xi][tile][ch] (rows of 20 floats: the
//     ds_read_b128 fragment reads are conflict-free).  The transform is shared by all
//     16 GEMMs, which is why the 16 live in one workgroup.
//   * U (transformed filters, built once per model by wino_weight_kernel) never
//     touches LDS: it is pre-permuted in HBM into MFMA-fragment order, so each wave
//     fetches its own B fragments with fully coalesced 1 KiB global loads.
//   * Register double buffering: the next step's patch and U fragments are in flight
//     while the current step's 32*NBW MFMAs run; one barrier per K-step.
//   * Epilogue: accumulators go through LDS (M[xi][tile][cout], one 32-column half at
//     a time), each thread inverse-transforms (tile, cout) pairs and applies
//     BN (+PReLU | + residual) at the <= 4 in-image pixels of the tile.
//
// Lane map of 32x32x2 MFMA: A operand lane (m = l%32, h = l/32) = A[m][k=h], B operand
// lane (n = l%32, h) = B[k=h][n].  We permute the 16 channels of a K-step so that MFMA
// j (0..7) multiplies channel 8h + j: lane (m, h) reads V[xi][m][8h .. 8h+7] with two
// ds_read_b128 and the matching 8 U values with two 16-B global loads.
#include "frhip_kernels.h"

namespace frhip {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int WT = 32;             // 2x2 output tiles per workgroup (MFMA M)
constexpr int WKC = 16;            // input channels per K-step
constexpr int VROW = 20;           // LDS floats per (xi, tile) row: 16 channels + 4 pad
constexpr int VPLANE = WT * VROW;  // one xi plane
constexpr int VBUF = 16 * VPLANE;  // one K-step of V (40 KiB)
constexpr int MROW = 33;           // epilogue staging row: 32 couts + 1
constexpr int MPLANE = WT * MROW;
static_assert(16 * MPLANE <= 2 * VBUF, "epilogue staging must fit the V buffers");

__device__ __forceinline__ int wino_xcd_remap(int bid, int n) {
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int NBW, bool PRE, int EPI>
__global__ __launch_bounds__(512, 1) void wino_kernel(WinoParams p) {
  constexpr int BN = 32 * NBW;
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

  // ---- transform role: one (tile, channel) per thread --------------------------------
  const int tl = tid >> 4, tc = tid & 15;
  const int T = mb * WT + tl;
  int base = 0;
  unsigned mask = 0;
  if (T < p.ntiles) {
    const int n = T / per_img;
    const int r = T - n * per_img;
    const int ty = r / p.TW, tx = r - ty * p.TW;
    const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((unsigned)(y0 + i) < (unsigned)H && (unsigned)(x0 + j) < (unsigned)W) mask |= 1u << (4 * i + j);
    base = (((n * H + y0) * W + x0) * Cin + tc) * 4;  // only used at in-image taps
  }
  const int rowb = W * Cin * 4, colb = Cin * 4;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.B * H * W * Cin * 4, 0x00020000);
  constexpr int OOB = 0x80000000;

  float d[16];
  float psc = 1.f, psh = 0.f;
  auto load_in = [&](int s) {
    const int off = base + s * WKC * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = (mask >> (4 * i + j)) & 1u;
        d[4 * i + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, ok ? off + i * rowb + j * colb : OOB, 0, 0));
      }
    if constexpr (PRE) {
      psc = p.pre_scale[s * WKC + tc];
      psh = p.pre_shift[s * WKC + tc];
    }
  };
  auto store_v = [&](int buf) {
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      v[e] = d[e];
      if constexpr (PRE) v[e] = ((mask >> e) & 1u) ? v[e] * psc + psh : 0.f;
    }
    float m[16];
    // B^T d (rows), then (.) B (columns)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      m[0 + j] = v[0 + j] - v[8 + j];
      m[4 + j] = v[4 + j] + v[8 + j];
      m[8 + j] = v[8 + j] - v[4 + j];
      m[12 + j] = v[4 + j] - v[12 + j];
    }
    float* dst = lds + buf * VBUF + tl * VROW + tc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dst[(4 * i + 0) * VPLANE] = m[4 * i + 0] - m[4 * i + 2];
      dst[(4 * i + 1) * VPLANE] = m[4 * i + 1] + m[4 * i + 2];
      dst[(4 * i + 2) * VPLANE] = m[4 * i + 2] - m[4 * i + 1];
      dst[(4 * i + 3) * VPLANE] = m[4 * i + 1] - m[4 * i + 3];
    }
  };

  // ---- GEMM role: wave wid owns xi = 2*wid + xl ----------------------------------------
  // U fragment (xi, 32-col block nb32, K-step s, half q): 64 lanes x float4, contiguous.
  const float4* ub = reinterpret_cast<const float4*>(p.u);
  auto u_index = [&](int xl, int b, int s, int q) {
    const int xi = 2 * wid + xl;
    return (((xi * NB32 + nb * NBW + b) * KS + s) * 2 + q) * 64 + lane;
  };
  float4 u0[2][NBW][2], u1[2][NBW][2];
  auto load_u = [&](float4 (&u)[2][NBW][2], int s) {
#pragma unroll
    for (int xl = 0; xl < 2; ++xl)
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int q = 0; q < 2; ++q) u[xl][b][q] = ub[u_index(xl, b, s, q)];
  };

  floatx16 acc[2][NBW];
#pragma unroll
  for (int xl = 0; xl < 2; ++xl)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[xl][b][e] = 0.f;

  auto mma = [&](const float4 (&u)[2][NBW][2], int buf) {
    const float* vb = lds + buf * VBUF + (lane & 31) * VROW + 8 * (lane >> 5);
    float4 a[2][2];
#pragma unroll
    for (int xl = 0; xl < 2; ++xl) {
      const float* vx = vb + (2 * wid + xl) * VPLANE;
      a[xl][0] = *reinterpret_cast<const float4*>(vx);
      a[xl][1] = *reinterpret_cast<const float4*>(vx + 4);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int xl = 0; xl < 2; ++xl)
#pragma unroll
        for (int b = 0; b < NBW; ++b)
          acc[xl][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[xl][j >> 2][j & 3], u[xl][b][j >> 2][j & 3],
                                                            acc[xl][b], 0, 0, 0);
  };

  // one K-step: prefetch s+1 (patch + U into `un`), MFMAs of s from LDS `buf` with `uc`,
  // transform s+1 into the other buffer, barrier
  auto step = [&](int s, const float4 (&uc)[2][NBW][2], float4 (&un)[2][NBW][2], int buf) {
    const bool live = s + 1 < KS;
    if (live) {
      load_in(s + 1);
      load_u(un, s + 1);
    }
    mma(uc, buf);
    if (live) store_v(buf ^ 1);
    __syncthreads();
  };

  load_in(0);
  load_u(u0, 0);
  store_v(0);
  __syncthreads();
  for (int s = 0; s < KS; s += 2) {  // KS is even (Cin % 32 == 0)
    step(s, u0, u1, 0);
    step(s + 1, u1, u0, 1);
  }

  // ---- epilogue: inverse transform + BN (+PReLU | +residual) -------------------------
  const int ec = tid & 31;  // cout within the 32-column half
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
    if constexpr (EPI == EPI_AFFINE_PRELU) al = p.prelu[cout];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int tile = (tid >> 5) + 16 * q;
      const int Tq = mb * WT + tile;
      if (Tq >= p.ntiles) continue;
      float m[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) m[e] = lds[e * MPLANE + tile * MROW + ec];
      float t0[4], t1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t0[j] = m[j] + m[4 + j] + m[8 + j];
        t1[j] = m[4 + j] - m[8 + j] - m[12 + j];
      }
      float yv[2][2];
      yv[0][0] = t0[0] + t0[1] + t0[2];
      yv[0][1] = t0[1] - t0[2] - t0[3];
      yv[1][0] = t1[0] + t1[1] + t1[2];
      yv[1][1] = t1[1] - t1[2] - t1[3];
      const int n = Tq / per_img;
      const int r = Tq - n * per_img;
      const int ty = r / p.TW, tx = r - ty * p.TW;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int oy = 2 * ty + i, ox = 2 * tx + j;
          if (oy >= H || ox >= W) continue;
          const long long o = ((long long)(n * H + oy) * W + ox) * p.Cout + cout;
          float v = yv[i][j] * sc + sh;
          if constexpr (EPI == EPI_AFFINE_PRELU) v = v > 0.f ? v : v * al;
          if constexpr (EPI == EPI_AFFINE_RES) v += p.res[o];
          if constexpr (EPI == EPI_AFFINE_RES_PRELU) {
            v += p.res[o];
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
      u[((((long long)(xi * NB32 + nb32) * KS + s) * 2 + q) * 64 + ln) * 4 + e] = (float)ua[b];
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
      (long long)p.B * p.H * p.W * p.Cin * 4 >= (1ll << 31) || (long long)p.B * p.H * p.W * p.Cout >= (1ll << 31))
    return hipErrorInvalidValue;
  p.TH = (p.H + 1) / 2;
  p.TW = (p.W + 1) / 2;
  p.ntiles = p.B * p.TH * p.TW;
  p.mblocks = (p.ntiles + WT - 1) / WT;
  const int nbw = (p.Cout % 64 == 0) ? 2 : 1;
  p.nblocks = p.Cout / (32 * nbw);
  const dim3 grid(p.mblocks * p.nblocks), block(512);
#define FR_WINO_CASE(NBW_, PRE_, EPI_)                                                  \
  if (nbw == NBW_ && pre == PRE_ && epi == EPI_) {                                      \
    hipLaunchKernelGGL((wino_kernel<NBW_, PRE_, EPI_>), grid, block, 0, s, p);          \
    return hipGetLastError();                                                           \
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
