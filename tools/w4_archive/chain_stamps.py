#!/usr/bin/env python3
"""Where a chained F(4x4) layer's time goes (tools only, never shipped): a libfrhip.so variant
whose wino4_chain_kernel writes s_memrealtime stamps (100 MHz) per (layer, workgroup) of its
longest chain (IR-101 stage 3) into a device array, then a batch-1 forward and per-phase medians.

    python tools/chain_stamps.py build          (here: tools/wv/lib_ch_stamps.so)
    python tools/chain_stamps.py run [n]        (GPU box)
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "tools", "wv", "lib_ch_stamps.so")
NL, NW, NS = 64, 256, 16
PHASES = ["wait prev layer", "body: ring step 0 ready", "body: K loop", "body: epilogue + drain",
          "item arrivals", "reduce + drain"]


def build():
    src = "conv_winograd4.hip"
    edits = [
        ('#include "frhip_kernels.h"\n',
         '#include "frhip_kernels.h"\n\n__device__ unsigned int w4chain_dbg[64 * 256 * 16];\n'
         '__shared__ int w4dbg_on;\n'
         'extern "C" __attribute__((visibility("default"))) int w4chain_dbg_read(void* dst, size_t bytes) {\n'
         '  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(w4chain_dbg), bytes, 0, hipMemcpyDeviceToHost);\n}\n'),
        ("  int rseen = lds_wait_min4(rdy, 1, p.poll_max);  // step 0 is in the ring\n",
         "  int rseen = lds_wait_min4(rdy, 1, p.poll_max);  // step 0 is in the ring\n"
         "  if constexpr (CH) if (lane == 0 && w == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 2] = "
         "__builtin_amdgcn_s_memrealtime();\n"),
        ("    for (int s = s0 + 1; s < s1; ++s) kstep(s, std::false_type{});\n",
         "    for (int s = s0 + 1; s < s1; ++s) kstep(s, std::false_type{});\n"
         "    if constexpr (CH) if (lane == 0 && w == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 3] = "
         "__builtin_amdgcn_s_memrealtime();\n"),
        ("    if (bid >= nwg) continue;\n",
         "    if (bid >= nwg) continue;\n"
         "    if (tid == 0) w4dbg_on = nl > 30 ? l : -1;\n"
         "#define STAMP(k) if (tid == 0 && nl > 30) w4chain_dbg[(l * 256 + bid) * 16 + (k)] = __builtin_amdgcn_s_memrealtime();\n"
         "    STAMP(0)\n"),
        ("      if (tid == 0) ok = w4_poll_ge(sync + l, links[l - 1].nwg, poll_max) && ok;\n      __syncthreads();\n",
         "      if (tid == 0) ok = w4_poll_ge(sync + l, links[l - 1].nwg, poll_max) && ok;\n      __syncthreads();\n"
         "    }\n    {\n      STAMP(1)\n"),
        ("    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // this wave's partial-slot stores\n    __syncthreads();\n",
         "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // this wave's partial-slot stores\n    __syncthreads();\n"
         "    STAMP(4)\n"),
        ("      ok = w4_poll_ge(sync + L.cbase + li, S, poll_max) && ok;\n    }\n    __syncthreads();\n",
         "      ok = w4_poll_ge(sync + L.cbase + li, S, poll_max) && ok;\n    }\n    __syncthreads();\n    STAMP(5)\n"),
        ("    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // this wave's output stores\n    __syncthreads();\n",
         "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // this wave's output stores\n    __syncthreads();\n"
         "    STAMP(6)\n"),
        # transform wave 4: start, after its first two patch loads are issued, after step 0 is in the ring
        ("    const int t = wid - 4;\n",
         "    const int t = wid - 4;\n"
         "    if constexpr (CH) if (lane == 0 && t == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 7] = "
         "__builtin_amdgcn_s_memrealtime();\n"),
        ("    load(pa);\n    load(pb);\n    for (int b = 0;; b += 3) {\n",
         "    load(pa);\n    load(pb);\n"
         "    if constexpr (CH) if (lane == 0 && t == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 8] = "
         "__builtin_amdgcn_s_memrealtime();\n"
         "    for (int b = 0;; b += 3) {\n"),
        ("      put(pa, b);\n",
         "      put(pa, b);\n"
         "      if constexpr (CH) if (b == 0 && lane == 0 && t == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 9] = "
         "__builtin_amdgcn_s_memrealtime();\n"),
        ("  const int w = wid;\n",
         "  const int w = wid;\n"
         "  if constexpr (CH) if (lane == 0 && w == 0 && w4dbg_on >= 0) w4chain_dbg[(w4dbg_on * 256 + bid) * 16 + 10] = "
         "__builtin_amdgcn_s_memrealtime();\n"),
    ]
    args = [sys.executable, os.path.join(REPO, "tools", "lib_variant.py"), "ch_stamps", src]
    for a, b in edits:
        args += [a, b]
    subprocess.run(args, check=True)


def run(n):
    import ctypes

    import numpy as np
    import torch

    sys.path.insert(0, REPO)
    from facerecognitionpipeline_amd import _lib
    _lib.LIB_PATH = SO
    from facerecognitionpipeline_amd import weights as W
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder

    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=64, graph_batch=0)
    crops = torch.from_numpy(W.synthetic_crops(n)).cuda()
    for _ in range(10):
        emb.embed_tensor(crops)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(SO)
    buf = (ctypes.c_uint * (NL * NW * NS))()
    rc = lib.w4chain_dbg_read(buf, ctypes.c_size_t(NL * NW * NS * 4))
    assert rc == 0, rc
    a = np.frombuffer(buf, dtype=np.uint32).reshape(NL, NW, NS).astype(np.int64)
    used = [(l, w) for l in range(NL) for w in range(NW) if a[l, w, 0] and a[l, w, 6]]
    layers = sorted({l for l, _ in used})
    print(f"batch {n}: stage-3 chain, {len(layers)} layers; per layer: median over its workgroups (us)")
    layers = [l for l in layers if l < max(layers)]  # the last layer (next stage's conv1) differs
    print("layer  wgs  " + "  ".join(f"{p[:14]:>14s}" for p in PHASES) + "   total  (start skew)")
    tot = np.zeros(len(PHASES))
    for l in layers:
        ws = [w for ll, w in used if ll == l]
        s = a[l, ws]
        d = np.stack([s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2], s[:, 4] - s[:, 3],
                      s[:, 5] - s[:, 4], s[:, 6] - s[:, 5]], 1) / 100.0  # 10 ns ticks -> us
        med = np.median(d, 0)
        tot += med
        skew = (s[:, 0].max() - s[:, 0].min()) / 100.0
        if l < 6 or l % 10 == 0:
            print(f"{l:5d} {len(ws):4d}  " + "  ".join(f"{x:14.2f}" for x in med) + f"  {med.sum():7.2f}  ({skew:.2f})")
    k = len(layers)
    print("mean  " + "      " + "  ".join(f"{x / k:14.2f}" for x in tot) + f"  {tot.sum() / k:7.2f}")
    # inside the body, from the layer's wait end (stamp 1): transform wave 4 start / loads issued /
    # step 0 stored, MFMA wave 0 start / ring step 0 seen
    sub = []
    for l in layers:
        ws = [w for ll, w in used if ll == l]
        s = a[l, ws]
        sub.append(np.median(np.stack([s[:, 7] - s[:, 1], s[:, 8] - s[:, 1], s[:, 9] - s[:, 1],
                                       s[:, 10] - s[:, 1], s[:, 2] - s[:, 1]], 1) / 100.0, 0))
    sub = np.median(np.array(sub), 0)
    print("body timeline from the wait's end (us, median): transform start %.2f, 2 patch loads issued %.2f, "
          "step 0 stored %.2f; MFMA wave start %.2f, ring step 0 seen %.2f" % tuple(sub))
    first = min(a[l, w, 0] for l, w in used)
    last = max(a[l, w, 6] for l, w in used)
    print(f"chain wall {(last - first) / 100.0:.1f} us for {k} layers = {(last - first) / 100.0 / k:.2f} us per layer")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
