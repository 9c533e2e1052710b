#!/usr/bin/env python3
"""Stem kernel variants (text edits of csrc/embed_misc.hip) linked into full copies of
libfrhip.so under tools/wv/stem_<name>.so, for tools/stem_bench.py --so (tools only).
usage: python tools/stem_variants.py"""
import glob
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "facerecognitionpipeline_amd", "csrc")
OUT = os.path.join(REPO, "tools", "wv")
SRC = open(os.path.join(CSRC, "embed_misc.hip")).read()
VARIANTS = {
    "rows16": SRC,
    "rows8": SRC.replace("constexpr int STEM_ROWS = 16;", "constexpr int STEM_ROWS = 8;"),
    "rows28": SRC.replace("constexpr int STEM_ROWS = 16;", "constexpr int STEM_ROWS = 28;"),
}
STORE = """      *reinterpret_cast<stem_f4*>(out + pp * STEM_C + 4 * (lane & 15)) =
          *reinterpret_cast<const stem_f4*>(so + pp * 68 + 4 * (lane & 15));"""
NT = """      __builtin_nontemporal_store(*reinterpret_cast<const stem_f4*>(so + pp * 68 + 4 * (lane & 15)),
                                  reinterpret_cast<stem_f4*>(out + pp * STEM_C + 4 * (lane & 15)));"""
assert STORE in SRC
VARIANTS["nt"] = SRC.replace(STORE, NT)
VARIANTS["rows8nt"] = VARIANTS["rows8"].replace(STORE, NT)
VARIANTS["rows28nt"] = VARIANTS["rows28"].replace(STORE, NT)
ONLY = os.environ.get("ONLY")
if ONLY:
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in ONLY.split(",")}
objs = [o for o in glob.glob(os.path.join(REPO, "build", "frhip", "*.o")) if "embed_misc" not in os.path.basename(o)]
# newest object per source
latest = {}
for o in objs:
    src = os.path.basename(o).split(".")[0]
    if src not in latest or os.path.getmtime(o) > os.path.getmtime(latest[src]):
        latest[src] = o
os.makedirs(OUT, exist_ok=True)
for name, text in VARIANTS.items():
    assert name == "rows16" or text != SRC, name
    src = os.path.join(OUT, f"stem_{name}.hip")
    open(src, "w").write(text)
    obj = src + ".o"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm",
                    "-amdgpu-mfma-vgpr-form=1", "-I" + CSRC,
                    "-I" + os.path.join(REPO, "include"), "-x", "hip", "-c", src, "-o", obj], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", *latest.values(), obj, "-o",
                    os.path.join(OUT, f"stem_{name}.so")], check=True)
    print(name)
