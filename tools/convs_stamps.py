#!/usr/bin/env python3
"""Where a serving conv launch's time goes (tools only, never shipped): a libfrhip.so variant
whose convs_kernel logs s_memrealtime stamps (100 MHz) per workgroup into a device array, then
one batch-1 forward and per-stage medians.  Per workgroup (wave 0): entry, first fragment's
MFMAs done (its loads' round trip), K loop done, the LDS reduction's barrier passed, output
stored (waited); the launch's span from the first workgroup's entry to the last one's store,
and the gap from the previous launch's last store to this launch's first entry.

    python tools/convs_stamps.py build [spread]     (here: tools/wv/lib_cs_stamps[_spread].so)
    python tools/convs_stamps.py run [n] [so] [arch]   (GPU box)

"spread" also launches grids of <= 256 workgroups with 96 KiB of dynamic LDS each, so that no CU
holds two of them (A/B of the hardware's workgroup placement).
"""
import os
import subprocess
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "wv", "lib_cs_stamps.so")
CAP = 65536


SPREAD = [("  const int grid = ((p.M + 15) / 16) * (p.Cout / 16);\n",
           "  const int grid = ((p.M + 15) / 16) * (p.Cout / 16);\n  const size_t lds = grid <= 256 ? 98304 : 0;\n"),
          (", 0, s, p);", ", lds, s, p);")]


def build(spread=False):
    edits = [
        ('#include "frhip_kernels.h"\n',
         '#include "frhip_kernels.h"\n\n__device__ unsigned long long cs_log[65536 * 4];\n'
         '__device__ unsigned int cs_ctr;\n'
         'extern "C" __attribute__((visibility("default"))) int cs_read(void* dst, size_t bytes, unsigned* n) {\n'
         '  (void)hipMemcpyFromSymbol(n, HIP_SYMBOL(cs_ctr), 4, 0, hipMemcpyDeviceToHost);\n'
         '  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(cs_log), bytes, 0, hipMemcpyDeviceToHost);\n}\n'
         'extern "C" __attribute__((visibility("default"))) int cs_reset() {\n'
         '  unsigned z = 0;\n'
         '  return (int)hipMemcpyToSymbol(HIP_SYMBOL(cs_ctr), &z, 4, 0, hipMemcpyHostToDevice);\n}\n'),
        ("  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);\n",
         "  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);\n"
         "  const unsigned long long T0 = __builtin_amdgcn_s_memrealtime();\n"
         "  unsigned long long T2 = T0, T3 = T0, T4 = T0;\n"),
        ("      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, v.w, ac, 0, 0, 0);\n",
         "      ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, v.w, ac, 0, 0, 0);\n"
         "      if (i0 == 0 && d == 0) T2 = __builtin_amdgcn_s_memrealtime();\n"),
        ("  f4 sum = acc[0] + acc[1];\n",
         "  T3 = __builtin_amdgcn_s_memrealtime();\n  f4 sum = acc[0] + acc[1];\n"),
        ("  if (w != 0) return;\n",
         "  if (w != 0) return;\n  T4 = __builtin_amdgcn_s_memrealtime();\n"),
        ("  if (!mval) return;\n", ""),
        ("  __builtin_amdgcn_raw_buffer_store_b128(bits4(v), rsrc(p.y, ybytes), yoff * 4, 0, CPOL_SC1);\n  if (p.y2)\n",
         "  if (mval) __builtin_amdgcn_raw_buffer_store_b128(bits4(v), rsrc(p.y, ybytes), yoff * 4, 0, CPOL_SC1);\n  if (p.y2 && mval)\n"),
        ("                                           0, CPOL_SC1);\n}",
         "                                           0, CPOL_SC1);\n"
         "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
         "  if (lane == 0) {\n"
         "    const unsigned long long T5 = __builtin_amdgcn_s_memrealtime();\n"
         "    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));\n"
         "    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));\n"
         "    const unsigned i = atomicAdd(&cs_ctr, 1u);\n"
         "    if (i < 65536) {\n"
         "      cs_log[4 * i] = T0;\n"
         "      cs_log[4 * i + 1] = (T2 - T0) | ((T3 - T0) << 32);\n"
         "      cs_log[4 * i + 2] = (T4 - T0) | ((T5 - T0) << 32);\n"
         "      cs_log[4 * i + 3] = blockIdx.x | ((unsigned long long)gridDim.x << 16) | ((unsigned long long)hw << 32) |\n"
         "                          ((unsigned long long)(xcc & 15) << 60);\n"
         "    }\n"
         "  }\n}"),
    ]
    if spread:
        edits += SPREAD
    args = [sys.executable, os.path.join(REPO, "tools", "lib_variant.py"), "cs_stamps" + ("_spread" if spread else ""),
            "conv_small.hip"]
    for a, b in edits:
        args += [a, b]
    subprocess.run(args, check=True)


def build_spread_only():
    args = [sys.executable, os.path.join(REPO, "tools", "lib_variant.py"), "cs_spread", "conv_small.hip"]
    for a, b in SPREAD:
        args += [a, b]
    subprocess.run(args, check=True)


def run(n, so=SO, arch="ir_101"):
    import ctypes

    import numpy as np
    import torch

    sys.path.insert(0, REPO)
    from facerecognitionpipeline_amd import _lib
    _lib.LIB_PATH = so
    from facerecognitionpipeline_amd import weights as W
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder

    emb = FaceEmbedder(architecture=arch, model_path="synthetic", max_batch=64, graph_batch=0)
    crops = torch.from_numpy(W.synthetic_crops(n)).cuda()
    for _ in range(10):
        emb.embed_tensor(crops)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(so)
    assert lib.cs_reset() == 0
    emb.embed_tensor(crops)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (CAP * 4))()
    cnt = ctypes.c_uint(0)
    assert lib.cs_read(buf, ctypes.c_size_t(CAP * 32), ctypes.byref(cnt)) == 0
    k = min(cnt.value, CAP)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(CAP, 4)[:k].astype(np.int64)
    t0 = a[:, 0]
    d2, d3 = a[:, 1] & 0xFFFFFFFF, a[:, 1] >> 32
    d4, d5 = a[:, 2] & 0xFFFFFFFF, a[:, 2] >> 32
    grid = (a[:, 3] >> 16) & 0xFFFF
    hw = (a[:, 3] >> 32) & 0x0FFFFFFF
    xcc = (a[:, 3] >> 60) & 15
    order = np.argsort(t0)
    launches, cur, cur_end = [], [], -1
    for i in order:
        if cur and (t0[i] > cur_end or grid[i] != grid[cur[0]]):
            launches.append(cur)
            cur, cur_end = [], -1
        cur.append(i)
        cur_end = max(cur_end, t0[i] + d5[i])
    if cur:
        launches.append(cur)
    print(f"{arch} batch {n}: {len(launches)} serving conv launches, {k} workgroup records (10 ns ticks shown as us)")
    by = defaultdict(list)
    prev_end = None
    for L in launches:
        L = np.array(L)
        s0 = t0[L].min()
        end = (t0[L] + d5[L]).max()
        gap = (s0 - prev_end) / 100.0 if prev_end is not None else float("nan")
        prev_end = end
        row = [len(L), (t0[L].max() - s0) / 100.0, np.median(d2[L]) / 100.0, np.median(d3[L]) / 100.0,
               np.median(d4[L]) / 100.0, np.median(d5[L]) / 100.0, d5[L].max() / 100.0, (end - s0) / 100.0, gap]
        # CUs holding two or more of the launch's workgroups at once
        cu = (xcc[L] << 16) | ((hw[L] >> 8) & 0xFF) | (((hw[L] >> 13) & 7) << 8)
        _, c = np.unique(cu, return_counts=True)
        row.append(float((c > 1).sum()))
        by[int(grid[L[0]])].append(row)
    cols = ["wgs", "entry skew", "1st data", "K loop end", "reduced", "stored", "max stored", "span",
            "gap before", "CUs x2+"]
    print("grid  launches  " + "  ".join(f"{c:>10s}" for c in cols))
    for g, rows in sorted(by.items(), key=lambda kv: -len(kv[1])):
        r = np.median(np.array(rows), 0)
        print(f"{g:4d}  {len(rows):8d}  " + "  ".join(f"{x:10.2f}" for x in r))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(len(sys.argv) > 2 and sys.argv[2] == "spread")
        if len(sys.argv) > 2 and sys.argv[2] == "spread":
            build_spread_only()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 1, sys.argv[3] if len(sys.argv) > 3 else SO,
            sys.argv[4] if len(sys.argv) > 4 else "ir_101")
