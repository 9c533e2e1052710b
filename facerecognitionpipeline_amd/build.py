"""Build recipe for libfrhip.so (gfx950 only), in-tree.

``python -m facerecognitionpipeline_amd.build`` or ``__graft_entry__.build()``.
Each source compiles to an object under ``build/`` (skipped when its content
hash and flags are unchanged), then everything links into
``facerecognitionpipeline_amd/libfrhip.so`` next to this file, so the built
library travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(REPO, "build", "frhip")
LIB = os.path.join(PKG, "libfrhip.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = "gfx950"
SOURCES = ["conv_winograd4.hip", "conv_winograd.hip", "conv_s2.hip", "conv_small.hip","conv_f32_w4.hip", "conv_f32_w8.hip", "conv_bf16x3.hip", "conv_det.hip", "conv_mfma.hip",
           "embed_misc.hip", "align.hip", "gallery.hip", "detect.hip", "frhip_runtime.cpp", "detector.cpp"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(REPO, "include"), "-I" + CSRC]
# F(4x4): the input / output transforms are packed f32 where the source says so (explicit f2
# vectors: measured 2-5% faster than their scalar form); the SLP vectorizer is kept
# from packing the rest (offset arithmetic, the MFMA waves' U-ring bookkeeping) behind our back
EXTRA = {"conv_winograd4.hip": ["-fno-slp-vectorize"],
         # the stem's MFMA accumulators in VGPRs: no v_accvgpr_read per output before its epilogue
         "embed_misc.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}
LDFLAGS = ["-shared", f"--offload-arch={ARCH}", f"-Wl,-rpath,{ROCM}/lib", "-Wl,--no-undefined"]


def _digest(path: str) -> str:
    h = hashlib.sha256()
    for p in [path, os.path.join(CSRC, "frhip_kernels.h"), os.path.join(CSRC, "conv_mfma_impl.h"),
              os.path.join(CSRC, "runtime.h"),
              os.path.join(REPO, "include", "frhip.h"), os.path.join(REPO, "include", "frhip_testing.h")]:
        with open(p, "rb") as f:
            h.update(f.read())
    # the flags without this checkout's absolute include paths: the digest (and the build id baked
    # into the library) must be the same wherever the tree is, e.g. on the GPU box's scratch copy
    flags = [f.replace(REPO, "<repo>") for f in CFLAGS + EXTRA.get(os.path.basename(path), [])]
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(src: str) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, f"{src}.{_digest(path)}.o")
    if not os.path.exists(obj):
        cmd = [HIPCC, *CFLAGS, *EXTRA.get(src, []), "-x", "hip", "-c", path, "-o", obj + ".tmp"]
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build_id() -> str:
    """Content hash of every source, header and flag that goes into libfrhip.so.  Compiled into the
    library (``fr_version()`` ends in ``build <id>``), so a profile stamped with it can be matched
    to the library a later run loads (bench.py attaches PMC figures only on a match)."""
    h = hashlib.sha256()
    for src in SOURCES:
        h.update(_digest(os.path.join(CSRC, src)).encode())
    return h.hexdigest()[:16]


def _build_id_obj(bid: str) -> str:
    src = os.path.join(BUILD, f"build_id_{bid}.cpp")
    obj = src + ".o"
    if not os.path.exists(obj):
        with open(src, "w") as f:
            f.write(f'extern "C" const char* frhip_build_id(void) {{ return "{bid}"; }}\n')
        subprocess.run([HIPCC, "-O2", "-fPIC", "-c", src, "-o", obj + ".tmp"], check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = True) -> str:
    """Compile every HIP source for gfx950 and link libfrhip.so; return its path."""
    os.makedirs(BUILD, exist_ok=True)
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, SOURCES))
    objs.append(_build_id_obj(build_id()))
    stamp = hashlib.sha256("".join(objs).encode()).hexdigest()[:16]
    stamp_file = os.path.join(BUILD, "libfrhip.stamp")
    if os.path.exists(LIB) and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return LIB
    subprocess.run([HIPCC, *LDFLAGS, *objs, "-o", LIB + ".tmp"], check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    if verbose:
        print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
