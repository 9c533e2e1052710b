#!/usr/bin/env python3
"""Where the F(4x4) GEMM kernel's time goes: textual variants of the shipping
csrc/conv_winograd4.hip (tools only, never shipped), each linked with tools/w4g_bench.cpp.

usage: w4g_variants.py build [names...]   (here, hipcc cross-compiles)
       w4g_variants.py run [names...]     (on the GPU box)
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "facerecognitionpipeline_amd", "csrc")
SRC = os.path.join(CSRC, "conv_winograd4.hip")
BENCH = os.path.join(REPO, "tools", "w4g_bench.cpp")
OUT = os.path.join(REPO, "tools", "wv")
SHAPES = [(256, 14, 256, 256, 2), (256, 14, 256, 256, 1), (256, 28, 128, 128, 2), (256, 56, 64, 64, 2),
          (256, 7, 512, 512, 2)]

EPI_START = "    // an idle quarter (!live, Cout % 64 != 0) runs the epilogue too"
EPI_END = "\n  }\n}\n\n// G g G^T"
MFMA8 = "".join(f"        acc[x{o}] = __builtin_amdgcn_mfma_f32_16x16x4f32(u{e}.{c}, a{e}.{c}, acc[x{o}], 0, 0, 0);\n"
                for c in "xyzw" for e, o in ((0, ""), (1, " + 1")))
ULOAD = """          uring[y % URING] = y + URING < NXI ? ld4(ur, lo, (y + URING) * XS + cur)
                                             : ld4(ur, lo, (y + URING - NXI) * XS + nxt);"""


def nouload(s):
    assert ULOAD in s
    return s.replace(ULOAD, "")


TRANS_PUT = "      store(P, g);\n"


def waitonly(s):
    """the transform waves wait for their patch loads (one sum of the patch written to the ring),
    but run none of the transform's arithmetic: separates the patch-load latency from the
    transform code's cost"""
    assert TRANS_PUT in s
    return s.replace(TRANS_PUT, """      {
        f2 sm = P.d[0][0];
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) sm += P.d[a][b];
        *reinterpret_cast<f2*>(ring + (g % NBUF) * VSTEP + dst_off) = sm;
      }
""")


GEO_EDITS = [
    ("        roff[e] = rin[e] ? (rs * p.NC * H + y) * W * Cin * 4 : BIGOFF;",
     "        roff[e] = rin[e] ? vmul24(vmad24(vmul24(rs, p.NC), H, y), W * Cin * 4) : BIGOFF;"),
    ("        coff[e] = cin[e] ? ((cs * H * W + x) * Cin + ch) * 4 : BIGOFF;",
     "        coff[e] = cin[e] ? vmad24(vmad24(cs, H * W, x), Cin, ch) * 4 : BIGOFF;"),
    ("          gt[e] = (y >= 0 && rs * p.NC < p.B && T < p.ntiles) ? (rs * p.NC * H + y) * W : -1;",
     "          gt[e] = (y >= 0 && rs * p.NC < p.B && T < p.ntiles) ? vmul24(vmad24(vmul24(rs, p.NC), H, y), W) : -1;"),
    ("          gt[4 + e] = (x >= 0 && cs < p.NC) ? cs * H * W + x : -1;",
     "          gt[4 + e] = (x >= 0 && cs < p.NC) ? vmad24(cs, H * W, x) : -1;"),
]
GEO_HELPERS = """
__device__ __forceinline__ int vmad24(int a, int b, int c) {
  int r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ int vmul24(int a, int b) {
  int r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
"""


def nomad(s):
    """item geometry with explicit 24-bit mul / mad instructions (no v_mad_u64_u32, whose unused
    high addend register can carry an outstanding load and cost a vmcnt wait at item entry)"""
    a = "__device__ __forceinline__ int canvas_coord("
    assert a in s
    s = s.replace(a, GEO_HELPERS + a, 1)
    for x, y in GEO_EDITS:
        assert x in s, x
        s = s.replace(x, y)
    return s


def notrans(s):
    """the transform waves keep loading and publishing, but transform and write nothing"""
    assert TRANS_PUT in s
    return s.replace(TRANS_PUT, "")


def noepi(s):
    a = s.index(EPI_START)
    b = s.index(EPI_END, a)
    dummy = ("    float sum = 0.f;\n#pragma unroll\n    for (int x = 0; x < NXI; ++x) sum += acc[x][0] + acc[x][3];\n"
             "    if (sum == 12345.f) p.y[tid] = 1.f;")
    return s[:a] + dummy + s[b:]


STORE = "__builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[y][x], 0, 0);"
GEO_LINE = "      const int ir0 = (4 * tr) / p.Pr, ic0 = (4 * tc) / p.Pc;\n      int roff[6], coff[3];"
WARM = """
      // warm L2 with this item's residual rows (one pixel = 64 couts = two 128-B lines per lane)
      if constexpr (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU)
        if (!SPLIT && j <= t_last) {
          const int px = half * 8 + pr, yy = px >> 2, xx = px & 3;
          int rs2, cs2;
          const int y2 = canvas_coord(4 * tr + yy, ir0, p.Pr, H, sep_r, rs2);
          const int x2 = canvas_coord(4 * tc + xx, ic0, p.Pc, W, sep_c, cs2);
          if (y2 >= 0 && rs2 * p.NC < p.B && T < p.ntiles && x2 >= 0 && cs2 < p.NC) {
            const int pix = (rs2 * p.NC * H + y2) * W + cs2 * H * W + x2;
            const int off = (pix * Cout + it.nb * 64) * 4;
            sink += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, off, 0, 0)) +
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, off + 128, 0, 0));
          }
        }
"""


def reswarm(s):
    assert GEO_LINE in s
    s = s.replace(GEO_LINE, GEO_LINE.replace("\n      int roff", WARM + "      int roff"), 1)
    a = "    float rowm[6], colm[3];\n"
    assert a in s
    s = s.replace(a, a + "    float sink = 0.f;\n    const __amdgpu_buffer_rsrc_t rw = uniform_rsrc(p.res, p.res ? p.B * H * W * Cout * 4 : 0);\n", 1)
    a = "    lds_barrier();  // barrier G: the MFMA waves close their last K-step with it\n    return;"
    assert a in s
    return s.replace(a, "    lds_barrier();  // barrier G: the MFMA waves close their last K-step with it\n"
                        "    if (sink == 1234.5f) ring[tid] = sink;\n    return;")


ENTER = "      const Item it = item_at(min(j, t_last));\n      ks_real = steps_of(it);\n      step0 = SPLIT ? it.split * KS : 0;\n"


def noenter(s):
    # geometry of the first item only (outputs wrong): what enter_item costs per item
    assert ENTER in s
    return s.replace(ENTER, ENTER + "      if (j > (SK ? t_first : 0)) return;\n", 1)


GEOW = "        if (g < 8 && j <= t_last) geo[((j & 3) * FT + i) * 8 + g] = g < 4 ? rv : cv;"


def samegeo(s):
    # every item's epilogue writes (and reads its residual at) the first item's pixels: what the
    # output stores to fresh addresses cost
    assert GEOW in s
    s = s.replace(GEOW, "        if (g < 8 && j <= t_last && j == 0) for (int q = 0; q < 4; ++q) geo[(q * FT + i) * 8 + g] = g < 4 ? rv : cv;")
    return s


KBAR = "      lds_publish(fre + w, lane, g);"


def nobar(s):
    # MFMA waves alone and without the per-K-step barrier (the transform waves, idle, wait at
    # their first one until the MFMA waves exit): what the barrier costs the MFMA stream
    s = VARIANTS["mfmaonly"](s)
    assert KBAR in s
    return s.replace(KBAR, "      asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");")


BT6V = """  const f2 c4 = {4.f, 4.f}, m4 = {-4.f, -4.f}, c2 = {2.f, 2.f}, m2 = {-2.f, -2.f};
  const f2 r = d[4] - d[2], u = d[3] - d[1];
  const f2 pp = __builtin_elementwise_fma(m4, d[2], d[4]), q = __builtin_elementwise_fma(m4, d[1], d[3]);
  t[0] = __builtin_elementwise_fma(c4, d[0] - d[2], r);
  t[1] = pp + q;
  t[2] = pp - q;
  t[3] = __builtin_elementwise_fma(c2, u, r);
  t[4] = __builtin_elementwise_fma(m2, u, r);
  t[5] = __builtin_elementwise_fma(m4, u, d[5] - d[3]);"""
BT6S = """  float a[6], b[6], ta[6], tb[6];
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    a[e] = d[e].x;
    b[e] = d[e].y;
  }
  bt6(a, ta);
  bt6(b, tb);
#pragma unroll
  for (int e = 0; e < 6; ++e) t[e] = f2{ta[e], tb[e]};"""
PREFMA = "d[a][b] = __builtin_elementwise_fma(P.trow[a], f2{P.colm[b], P.colm[b]}, d[a][b]);"
PRES = "d[a][b] = f2{__builtin_fmaf(P.trow[a].x, P.colm[b], d[a][b].x), __builtin_fmaf(P.trow[a].y, P.colm[b], d[a][b].y)};"


def scalartr(s):
    # the input transform's math in scalar f32 (same 8-byte loads and lane layout)
    assert BT6V in s and PREFMA in s
    return s.replace(BT6V, BT6S).replace(PREFMA, PRES)


AT6V = """  const f2 c2 = {2.f, 2.f}, c4 = {4.f, 4.f}, c8 = {8.f, 8.f};
  const f2 p12 = m[1] + m[2], m12 = m[1] - m[2];
  const f2 p34 = m[3] + m[4], m34 = m[3] - m[4];
  o[0] = m[0] + p12 + p34;
  o[1] = __builtin_elementwise_fma(c2, m34, m12);
  o[2] = __builtin_elementwise_fma(c4, p34, p12);
  o[3] = __builtin_elementwise_fma(c8, m34, m12 + m[5]);"""
AT6S = """#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float p12 = m[1][e] + m[2][e], m12 = m[1][e] - m[2][e];
    const float p34 = m[3][e] + m[4][e], m34 = m[3][e] - m[4][e];
    o[0][e] = m[0][e] + p12 + p34;
    o[1][e] = __builtin_fmaf(2.f, m34, m12);
    o[2][e] = __builtin_fmaf(4.f, p34, p12);
    o[3][e] = __builtin_fmaf(8.f, m34, m12 + m[5][e]);
  }"""


def scalarepi(s):
    # the epilogue's output transform in scalar f32 (same arithmetic per element)
    assert AT6V in s
    return s.replace(AT6V, AT6S)


def res12(s):
    # 12-deep U ring for the residual epilogues too, with the residual loaded one output row ahead
    for a, b in (("  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 9 : 12;", "  return 12;"),
                 ("      if (!SK && q == 1) load_res(0);", ""),
                 ("    if constexpr (!SK) load_res(2);", ""),
                 ("      if constexpr (SK && RES) {", "      if constexpr (RES) {")):
        assert a in s, a
        s = s.replace(a, b)
    return s


STAMP_HDR = """
// ---- stamps variant: per-wave cycle accounting (s_memtime), written once per wave by lane 0 ----
__device__ unsigned long long w4dbg[1024 * 8 * 4];
#define W4_WAIT(c_, n_, pm_)                                        \\
  ({                                                                \\
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();    \\
    const int r_ = lds_wait_min4(c_, n_, pm_);                      \\
    bar_cyc += __builtin_amdgcn_s_memtime() - t0_;                  \\
    r_;                                                             \\
  })
#define W4_PUT()                                                                        \\
  if (lane == 0) {                                                                      \\
    unsigned long long* d_ = w4dbg + ((size_t)bid * 8 + wid) * 4;                \\
    d_[0] = __builtin_amdgcn_s_memtime() - t_start;                                     \\
    d_[1] = bar_cyc;                                                                    \\
    d_[2] = epi_cyc;                                                                    \\
    d_[3] = (unsigned long long)G;                                                      \\
  }
"""
STAMP_HOST = """
#include <cstdio>
extern "C" void w4g_after_run() {
  static unsigned long long h[1024 * 8 * 4];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(frhip::w4dbg), sizeof(h)) != hipSuccess) return;
  double tot[2] = {0, 0}, bar[2] = {0, 0}, epi[2] = {0, 0}, st[2] = {0, 0};
  unsigned long long tmax[2] = {0, 0};
  int n[2] = {0, 0};
  for (int b = 0; b < 1024; ++b)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long* d = h + ((size_t)b * 8 + w) * 4;
      if (!d[0]) continue;
      const int k = w < 4 ? 0 : 1;
      tot[k] += d[0]; bar[k] += d[1]; epi[k] += d[2]; st[k] += d[3]; ++n[k];
      if (d[0] > tmax[k]) tmax[k] = d[0];
    }
  for (int k = 0; k < 2; ++k)
    if (n[k])
      printf("  %s waves: %d, avg total %.0f cyc (max %llu), hand-off wait %.0f (%.1f%%), epilogue %.0f (%.1f%%), "
             "K-steps %.1f -> %.0f cyc/K-step, %.0f outside waits+epilogue per K-step\\n",
             k ? "transform" : "MFMA", n[k], tot[k] / n[k], tmax[k], bar[k] / n[k], 100 * bar[k] / tot[k],
             epi[k] / n[k], 100 * epi[k] / tot[k], st[k] / n[k], tot[k] / st[k], (tot[k] - bar[k] - epi[k]) / st[k]);
}
"""


def stamps(s):
    # s_memtime accounting per wave: total, time waiting on the ring counters (the per-K-step
    # barrier before the counter hand-off), MFMA-wave epilogue
    s = s.replace("= lds_wait_min4(", "= W4_WAIT(")
    a = "__device__ __forceinline__ int canvas_coord("
    assert a in s
    s = s.replace(a, STAMP_HDR + a, 1)
    a = "  const int tid = threadIdx.x, lane = tid & 63;\n"
    assert a in s
    s = s.replace(a, a + "  unsigned long long bar_cyc = 0, epi_cyc = 0;\n"
                         "  const unsigned long long t_start = __builtin_amdgcn_s_memtime();\n", 1)
    a = "      if (b + 3 >= G) break;\n    }\n    w4_report_handoff(fseen, p.err);\n    return;"
    assert a in s
    s = s.replace(a, "      if (b + 3 >= G) break;\n    }\n    W4_PUT();\n    w4_report_handoff(fseen, p.err);\n    return;")
    assert EPI_START in s
    s = s.replace(EPI_START, "    const unsigned long long t_e0 = __builtin_amdgcn_s_memtime();\n" + EPI_START, 1)
    # part A of the deferred epilogue (whole items); part B runs inside the next item's MFMAs
    a = "      transform_to_pv();\n      set_pending();\n      return;"
    assert a in s
    s = s.replace(a, "      transform_to_pv();\n      set_pending();\n      epi_cyc += __builtin_amdgcn_s_memtime() - t_e0;\n      return;")
    a = "  w4_report_handoff(rseen, p.err);\n}\n"
    assert s.count(a) == 1
    s = s.replace(a, "  W4_PUT();\n  w4_report_handoff(rseen, p.err);\n}\n")
    return s + STAMP_HOST


MFMA_START = "  // ---- MFMA waves: wave w owns couts 16w .. 16w+15 of every item"
TR_START = "    const int t = wid - 4;\n"


def prio_mfma(s):
    # MFMA waves at s_setprio 1: they win issue arbitration on their SIMD
    assert MFMA_START in s
    return s.replace(MFMA_START, "  __builtin_amdgcn_s_setprio(1);\n" + MFMA_START, 1)


def prio_tr(s):
    # transform waves (the younger half, waves 4-7) at s_setprio 1
    assert TR_START in s
    return s.replace(TR_START, TR_START + "    __builtin_amdgcn_s_setprio(1);\n", 1)


LD4_DEF = "__device__ __forceinline__ f4 ld4(__amdgpu_buffer_rsrc_t r, int off, int soff = 0) {"


def upolicy(aux):
    # U fragment loads with a cache-policy aux field (sc0 = 1, nt = 2, sc1 = 16): L1 bypass
    def f(s):
        assert LD4_DEF in s
        extra = ("template <int AUX>\n__device__ __forceinline__ f4 ld4p(__amdgpu_buffer_rsrc_t r, int off, int soff = 0) {\n"
                 "  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, AUX);\n"
                 "  return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};\n}\n\n")
        s = s.replace(LD4_DEF, extra + LD4_DEF, 1)
        n = s.count("ld4(ur, ")
        assert n >= 3, n
        return s.replace("ld4(ur, ", f"ld4p<{aux}>(ur, ")
    return f


def early_res(s):
    # residual rows 0-1 issued before the output transform, rows 2-3 before couts 2-3 (scalar
    # output transform: fewer live registers)
    s = scalarepi(s)
    for a, b in (("      if (!SK && q == 1) load_res(0);", "      if (!SK && q == 0) load_res(0);\n      if (!SK && q == 1) load_res(2);"),
                 ("    if constexpr (!SK) load_res(2);", "")):
        assert a in s, a
        s = s.replace(a, b)
    return s


NBG = "  p.nbg = std::max(1, std::min(p.mblocks, std::max(32 / p.nblocks, 8)));"


GRID = "dim3(MODE_ == 2 ? cus : std::min(nit, cus))"


def grid(n):
    # whole-item launches (MODE 0) on a persistent grid of n workgroups instead of one per CU: two
    # concurrent lanes on disjoint parts of the chip instead of queueing behind each other
    def f(s):
        assert GRID in s
        return s.replace(GRID, f"dim3(MODE_ == 2 ? cus : std::min(nit, MODE_ == 0 ? {n} : cus))")
    return f


def nbg(minimum):
    # at least `minimum` tile blocks per XCD item group (Cout = 512: 4 -> 8, U streamed per XCD
    # round halves, patches read twice)
    def f(s):
        assert NBG in s
        return s.replace(NBG, f"  p.nbg = std::max(1, std::min(p.mblocks, std::max(32 / p.nblocks, {minimum})));")
    return f


def halftrans(s):
    """transform + LDS writes on even K-steps only (wrong results): the gain an item with twice
    the couts per transformed patch could reach"""
    assert TRANS_PUT in s
    return s.replace(TRANS_PUT, "      if ((g & 1) == 0) store(P, g);\n")


def halfpatch(s):
    """halftrans + patch loads of odd K-steps skipped"""
    a = "          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][b], soff, 0);"
    assert a in s
    s = s.replace(a, "          const u32x2 v = (ls & 1) ? u32x2{0u, 0u} : __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][b], soff, 0);")
    return halftrans(s)


def halfu(s):
    """U refills of odd xi skipped (wrong results): the gain of twice the tiles per U fragment"""
    a = "          uring[y % URING] = y + URING < NXI ?"
    assert a in s
    return s.replace(a, "          if (e == 0) uring[y % URING] = y + URING < NXI ?")


LOOP3 = """    Patch pa, pb, pc;"""
LOOPBODY3 = """    load(pa);
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
    }"""
LOOPBODY4 = """    load(pa);
    load(pb);
    load(pc);
    for (int b = 0;; b += 4) {
      load(pd);
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
      load(pc);
      __builtin_amdgcn_sched_barrier(0);
      put(pd, b + 3);
      if (b + 4 >= G) break;
    }"""


def pf3(s):
    """patch loads three K-steps ahead (four rotating buffers) instead of two"""
    assert LOOP3 in s and LOOPBODY3 in s
    return s.replace(LOOP3, "    Patch pa, pb, pc, pd;").replace(LOOPBODY3, LOOPBODY4)


PLOAD = """#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][b], soff, 0);
          P.d[a][b] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
        }"""
PLOAD12 = """#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, poff[a][0], soff, 0);
        P.d[a][0] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
        P.d[a][1] = f2{__uint_as_float(v.z), __uint_as_float(v.w)};
        const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][2], soff, 0);
        P.d[a][2] = f2{__uint_as_float(w.x), __uint_as_float(w.y)};
      }"""


def load12(s):
    """12 patch loads per lane and step (6 of them 16-byte) instead of 18 8-byte ones, same bytes
    give or take (wrong data): does the load instruction count or the bytes cost?"""
    assert PLOAD in s
    return s.replace(PLOAD, PLOAD12)


PLOAD_PAIR = """#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          u32x2 v = {0u, 0u};
          if (odd == 0) {
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, poff[a][b], soff, 0);
            v = u32x2{q.x ^ q.z, q.y ^ q.w};
          }
          P.d[a][b] = f2{__uint_as_float(v.x), __uint_as_float(v.y)};
        }"""


def pair128(s):
    """patch loads of two K-steps at once: 16-byte loads on even steps, none on odd (wrong data):
    the bound for loading a pixel's whole 128-B line of 32 channels once per two steps"""
    assert PLOAD in s
    s = s.replace(PLOAD, PLOAD_PAIR)
    a = "      const int soff = step * KC * 4;"
    assert a in s
    return s.replace(a, a + "\n      const int odd = __builtin_amdgcn_readfirstlane(ls & 1);")


REFILL = """#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int y = x + e;
          uring[y % URING] = y + URING < NXI ? ld4(ur, lo, (y + URING) * XS + cur)
                                             : ld4(ur, lo, (y + URING - NXI) * XS + nxt);
        }"""


def nofirstrefill(s):
    """no U refills in an item's first K-step (wrong results): the cost of those refills waiting
    behind the previous epilogue's stores in vmcnt order (plus 1/KS of the U traffic)"""
    for a in (REFILL, "    auto kstep = [&](int s) {", "    kstep(s0);\n", "for (int s = s0 + 1; s < s1; ++s) kstep(s);"):
        assert a in s, a
    s = s.replace(REFILL, "        if constexpr (!decltype(FIRST)::value)\n" + REFILL)
    s = s.replace("    auto kstep = [&](int s) {", "    auto kstep = [&](int s, auto FIRST) {")
    s = s.replace("    kstep(s0);\n", "    kstep(s0, std::true_type{});\n")
    s = s.replace("for (int s = s0 + 1; s < s1; ++s) kstep(s);", "for (int s = s0 + 1; s < s1; ++s) kstep(s, std::false_type{});")
    return "#include <type_traits>\n" + s


def noscale(s):
    """epilogue BN scale / shift / PReLU slopes as constants instead of per-item global loads
    (wrong results): the cost of those loads' latency, exposed in the MFMA waves' epilogue"""
    for a, b in (("      sc = *reinterpret_cast<const f4*>(p.post_scale + cout0);", "      sc = f4{1.01f, 0.99f, 1.02f, 0.98f};"),
                 ("      sh = *reinterpret_cast<const f4*>(p.post_shift + cout0);", "      sh = f4{0.01f, -0.01f, 0.02f, -0.02f};"),
                 ("      al = *reinterpret_cast<const f4*>(p.prelu + cout0);", "      al = f4{0.25f, 0.2f, 0.3f, 0.1f};")):
        assert a in s, a
        s = s.replace(a, b)
    return s


def aprio(s):
    """transform waves at issue priority only while the ring holds <= 1 transformed step ahead of
    the slowest MFMA wave (else priority 0), for every epilogue"""
    a = "    if constexpr (PRE) __builtin_amdgcn_s_setprio(1);\n"
    b = "      store(P, g);\n"
    assert a in s and b in s
    s = s.replace(a, "")
    return s.replace(b, "      {\n        const int ahead = g - lds_min4(fre);\n"
                        "        if (ahead <= 1) __builtin_amdgcn_s_setprio(1); else __builtin_amdgcn_s_setprio(0);\n"
                        "      }\n" + b)


def aprio2(s):
    """aprio with the threshold at 2 steps ahead"""
    return aprio(s).replace("if (ahead <= 1)", "if (ahead <= 2)")


CBLK_EDITS = [
    ("        roff[e] = rin[e] ? (rs * p.NC * H + y) * W * Cin * 4 : BIGOFF;",
     "        roff[e] = rin[e] ? (rs * p.NC * H * W * Cin + y * W * KC) * 4 : BIGOFF;"),
    ("        coff[e] = cin[e] ? ((cs * H * W + x) * Cin + ch) * 4 : BIGOFF;",
     "        coff[e] = cin[e] ? (cs * H * W * Cin + x * KC + ch) * 4 : BIGOFF;"),
    ("      const int soff = step * KC * 4;", "      const int soff = step * H * W * KC * 4;"),
    ("          gt[e] = (y >= 0 && rs * p.NC < p.B && T < p.ntiles) ? (rs * p.NC * H + y) * W : -1;",
     "          gt[e] = (y >= 0 && rs * p.NC < p.B && T < p.ntiles) ? rs * p.NC * H * W * Cout + y * W * 16 : -1;"),
    ("          gt[4 + e] = (x >= 0 && cs < p.NC) ? cs * H * W + x : -1;",
     "          gt[4 + e] = (x >= 0 && cs < p.NC) ? cs * H * W * Cout + x * 16 : -1;"),
    ("        ro[e] = orow >= 0 && live ? (orow * Cout + cout0) * 4 : BIGOFF;",
     "        ro[e] = orow >= 0 && live ? (orow + (cout0 >> 4) * H * W * 16 + (cout0 & 15)) * 4 : BIGOFF;"),
    ("        co[e] = ocol >= 0 ? ocol * Cout * 4 : BIGOFF;", "        co[e] = ocol >= 0 ? ocol * 4 : BIGOFF;"),
]


def cblk(s):
    """channel-blocked activations [n][C/16][H][W][16] for the patch loads, the output stores and
    the residual loads (timing only here: the bench's data stays as it is)"""
    for x, y in CBLK_EDITS:
        assert x in s, x
        s = s.replace(x, y)
    return s


NOPRE_A = "  FR_W4_CASE(true, EPI_AFFINE_PRELU)       // IR conv1: pre-BN (in the transform), BN, PReLU\n"
NOPRE_B = "hipError_t launch_wino4(const Wino4Params& p0, bool pre, Epi epi, hipStream_t s) {\n"


def nopre(s):
    """conv1 without the pre-BN in the transform (as if the previous conv2's epilogue had applied it
    to a second copy of its output): timing only"""
    assert NOPRE_A in s and NOPRE_B in s
    return s.replace(NOPRE_A, "").replace(NOPRE_B, NOPRE_B + "  if (pre && epi == EPI_AFFINE_PRELU) pre = false;\n")


Y2_STORE = "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);\n"


def y2store(s):
    """conv2 epilogues also write BN_next(y) = y * s + t (here the post-BN pair again) into a second
    tensor of y's shape (the residual buffer: timing only): what the next conv1's pre-BN costs here"""
    assert Y2_STORE in s
    return s.replace(Y2_STORE, Y2_STORE + """    if constexpr (DRES) {
      const f4 v2 = __builtin_elementwise_fma(v, psc, psh);
      const u32x4 b2 = {__float_as_uint(v2.x), __float_as_uint(v2.y), __float_as_uint(v2.z), __float_as_uint(v2.w)};
      __builtin_amdgcn_raw_buffer_store_b128(b2, y2r_d, po[i], 0, 0);
    }
""").replace("  const __amdgpu_buffer_rsrc_t yr_d = uniform_rsrc(p.y, p.B * H * W * Cout * 4);\n",
             "  const __amdgpu_buffer_rsrc_t yr_d = uniform_rsrc(p.y, p.B * H * W * Cout * 4);\n"
             "  const __amdgpu_buffer_rsrc_t y2r_d = uniform_rsrc(p.res, p.res ? p.B * H * W * Cout * 4 : 0);\n")


FINISH = """  auto finish = [&](int i) {  // part B of pending pixel i
    f4 v = __builtin_elementwise_fma(pv[i], psc, psh);
    if constexpr (EPI == EPI_AFFINE_PRELU) v = prelu_q(v, pal, pcl);
    if constexpr (DRES) {
      v += pres[i];
      if constexpr (EPI == EPI_AFFINE_RES_PRELU) v = prelu_q(v, pal, pcl);
    }
    const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);
  };
"""
PAIRSTORE = """  // part B in pixel pairs (x, x + 1) of a tile row: lanes of tiles n, n ^ 1 (lane ^ 1, same couts)
  // swap one value each (DPP quad_perm [1,0,3,2]) so that each store instruction writes whole
  // 128-B lines of the channel-blocked output (pixels 2k, 2k + 1 of one tile)
  f4 pend = {0.f, 0.f, 0.f, 0.f};
  int pend_off = BIGOFF;
  auto epi_px = [&](int i) {
    f4 v = __builtin_elementwise_fma(pv[i], psc, psh);
    if constexpr (EPI == EPI_AFFINE_PRELU) v = prelu_q(v, pal, pcl);
    if constexpr (DRES) {
      v += pres[i];
      if constexpr (EPI == EPI_AFFINE_RES_PRELU) v = prelu_q(v, pal, pcl);
    }
    return v;
  };
  auto swp = [](float f) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(f), 0xB1, 0xF, 0xF, false));
  };
  auto st = [&](f4 v, int off) {
    const u32x4 bits = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, off, 0, 0);
  };
  auto finish = [&](int i) {
    if ((i & 1) == 0) {
      const bool odd = (threadIdx.x & 1) != 0;
      const f4 v0 = epi_px(i), v1 = epi_px(i + 1);
      const f4 t = odd ? v0 : v1;
      const f4 sw = {swp(t.x), swp(t.y), swp(t.z), swp(t.w)};
      const int so = __builtin_amdgcn_update_dpp(0, odd ? po[i] : po[i + 1], 0xB1, 0xF, 0xF, false);
      st(odd ? sw : v0, odd ? so : po[i]);
      pend = odd ? v1 : sw;
      pend_off = odd ? po[i + 1] : so;
    } else {
      st(pend, pend_off);
    }
  };
"""


def pairstore(s):
    assert FINISH in s
    return s.replace(FINISH, PAIRSTORE)


VARIANTS = {
    "pairstore": pairstore,
    "nopre": nopre,
    "y2store": y2store,
    "cblk_nopre_y2": lambda s: y2store(nopre(cblk(s))),
    "cblk": cblk,
    "cblk_noload": lambda s: VARIANTS["noload"](cblk(s)),
    "uring18pre": lambda s: s.replace("  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 9 : 12;",
                                      "  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 9 : 18;"),
    "uring6res": lambda s: s.replace("  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 9 : 12;",
                                     "  return (EPI == EPI_AFFINE_RES || EPI == EPI_AFFINE_RES_PRELU) ? 6 : 12;"),
    "grid128": grid(128),
    "grid192": grid(192),
    "nbg8": nbg(8),
    "nbg16": nbg(16),
    "nbuf3": lambda s: s.replace("constexpr int NBUF = 4; ", "constexpr int NBUF = 3; "),
    "early_res": early_res,
    "u_sc1": upolicy(16),
    "u_nt": upolicy(2),
    "u_sc01": upolicy(17),
    "u_sc0": upolicy(1),
    "prio_mfma": prio_mfma,
    "prio_tr": prio_tr,
    "stamps_prio_mfma": lambda s: stamps(prio_mfma(s)),
    "stamps_prio_tr": lambda s: stamps(prio_tr(s)),
    "stamps": stamps,
    "scalarepi": scalarepi,
    "scalarall": lambda s: scalarepi(scalartr(s)),
    "stamps_scalarall": lambda s: stamps(scalarepi(scalartr(s))),
    "scalartr_prio_tr": lambda s: prio_tr(scalartr(s)),
    "stamps_scalartr": lambda s: stamps(scalartr(s)),
    "res12": res12,
    "uring12": lambda s: s.replace("constexpr int URING = 9; ", "constexpr int URING = 12;"),
    "noenter": noenter,
    "scalartr": scalartr,
    "nobar": lambda s: nobar(s),
    "samegeo": samegeo,
    "st_nt": lambda s: s.replace(STORE, STORE.replace(", 0, 0);", ", 0, 2);")),
    "st_sc1": lambda s: s.replace(STORE, STORE.replace(", 0, 0);", ", 0, 16);")),
    "st_sc01": lambda s: s.replace(STORE, STORE.replace(", 0, 0);", ", 0, 17);")),
    "reswarm": reswarm,
    "base": lambda s: s,
    "aprio": aprio,
    "aprio2": aprio2,
    "noscale": noscale,
    "nofirstrefill": nofirstrefill,
    "nonpersist": lambda s: s.replace("dim3(MODE_ == 2 ? cus : std::min(nit, cus))", "dim3(MODE_ == 2 ? cus : (MODE_ == 0 ? nit : std::min(nit, cus)))"),
    "pair128": pair128,
    "load12": load12,
    "u18split": lambda s: s.replace("  constexpr int URING = uring_depth<EPI>();", "  constexpr int URING = MODE == 1 ? 18 : uring_depth<EPI>();"),
    "pf3": pf3,
    "halftrans": halftrans,
    "halfpatch": halfpatch,
    "halfu": halfu,
    "noepi": noepi,
    "notrans": notrans,
    "waitonly": waitonly,
    "partb_sc1": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 16);"),
    "partb_sc0": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 1);"),
    "partb_sc01": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 17);"),
    "partb_nostore": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    if (v.x == 12345.678f && p.B < 0) __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);"),
    "partb_small": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i] & 0xfff0, 0, 0);"),
    "partb_nt": lambda s: s.replace("    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 0);", "    __builtin_amdgcn_raw_buffer_store_b128(bits, yr_d, po[i], 0, 2);"),
    # deferred epilogue pieces removed (wrong results, timing only)
    "nopartb": lambda s: s.replace("          if (x >= 4) finish(x / 2 - 2);", "          if (x >= 4 && p.B < 0) finish(x / 2 - 2);"),
    "nores2": lambda s: s.replace("pres[i] = ld4(rr, oo[i >> 2][i & 3]);", "pres[i] = f4{0.f, 0.f, 0.f, 0.f};"),
    "stamps_nopartb": lambda s: stamps(s.replace("          if (x >= 4) finish(x / 2 - 2);", "          if (x >= 4 && p.B < 0) finish(x / 2 - 2);")),
    "noprio": lambda s: s.replace("    if constexpr (PRE) __builtin_amdgcn_s_setprio(1);\n", ""),
    "nomad": nomad,
    "nofixup": lambda s: s.replace("    if (MODE_ == 1) /* 64-thread blocks", "    if (false) /* 64-thread blocks"),
    "noload": lambda s: s.replace("""          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, poff[a][b], soff, XPOL);""",
                                  """          const u32x2 v = {(unsigned)(poff[a][b] + soff), 0u};"""),
    "nomfma": lambda s: (s.replace(MFMA8, "        acc[x][0] += a0.x * u0.x + a1.w * u1.w;\n") if MFMA8 in s else s + "#error MFMA8"),
    "nouload": nouload,
    "mfmaonly": lambda s: nouload(notrans(noepi(s))),
    "nores": lambda s: s.replace("rv[y][x] = ld4(rr, oo[y][x]);", "rv[y][x] = f4{0.f, 0.f, 0.f, 0.f};"),
    "nostore": lambda s: s.replace("__builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[y][x], 0, 0);",
                                   "if (bits.x == 0x7fc00001u) __builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[y][x], 0, 0);"),
    "smallstore": lambda s: s.replace("__builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[y][x], 0, 0);",
                                      "__builtin_amdgcn_raw_buffer_store_b128(bits, yr, oo[y][x] & 0xfff0, 0, 0);"),
    "smallres": lambda s: s.replace("rv[y][x] = ld4(rr, oo[y][x]);", "rv[y][x] = ld4(rr, oo[y][x] & 0xfff0);"),
    "nomfma_noload": lambda s: VARIANTS["noload"](VARIANTS["nomfma"](s)),
    "nomfma_notrans": lambda s: notrans(VARIANTS["nomfma"](s)),
    "nomfma_noepi": lambda s: noepi(VARIANTS["nomfma"](s)),
    "skeleton": lambda s: nouload(notrans(noepi(VARIANTS["nomfma"](s)))),
}


def build(name):
    s = open(SRC).read()
    v = VARIANTS[name](s)
    assert name == "base" or v != s, name
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, f"w4g_{name}.hip")
    open(src, "w").write(v)
    exe = os.path.join(OUT, f"w4g_{name}")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-slp-vectorize", "-I" + CSRC,
                    "-I" + os.path.join(REPO, "include"), "-x", "hip", src, "-x", "hip", BENCH, "-o", exe], check=True)
    return exe


def main():
    cmd, names = sys.argv[1], sys.argv[2:] or list(VARIANTS)
    if cmd == "build":
        with ThreadPoolExecutor(8) as ex:
            print(list(ex.map(build, names)))
    else:
        for n in names:
            # base: the default schedule (whole items + tail split-K), whole items only, stream-K
            for tag, sk, ns in ((("", 0, 0), ("/whole", 0, 1), ("/sk", 2, 0)) if n == "base" else (("", 0, 0),)):
                for shp in SHAPES:
                    r = subprocess.run(["timeout", "-k", "5", "60", os.path.join(OUT, f"w4g_{n}")] +
                                       [str(x) for x in shp] + ["20", str(sk), str(ns)], capture_output=True, text=True)
                    print(f"{n + tag:12s} {r.stdout.strip()} {r.stderr.strip()[-200:]}", flush=True)
                    if r.returncode:
                        return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
