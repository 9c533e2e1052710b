#!/usr/bin/env python3
"""A full libfrhip.so with one csrc file replaced by a text-edited copy (tools only, never
shipped): tools/wv/lib_<name>.so (or $LIBV_OUT/lib_<name>.so: tools/wv/ does not travel to the GPU
box), loadable by the serving / stem / detector tools through --so or FRHIP_LIB; compiled with the
file's extra flags from the package build.
usage: python tools/lib_variant.py NAME FILE.hip 'OLD' 'NEW' ['OLD2' 'NEW2' ...]"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "facerecognitionpipeline_amd", "csrc")
OUT = os.environ.get("LIBV_OUT", os.path.join(REPO, "tools", "wv"))
sys.path.insert(0, REPO)
from facerecognitionpipeline_amd.build import EXTRA, SOURCES  # noqa: E402


def main():
    name, fname, edits = sys.argv[1], sys.argv[2], sys.argv[3:]
    text = open(os.path.join(CSRC, fname)).read()
    for old, new in zip(edits[::2], edits[1::2]):
        assert old in text, old
        text = text.replace(old, new)
    latest = {}
    wanted = {f.split(".")[0] for f in SOURCES} | {"build_id"}
    for o in glob.glob(os.path.join(REPO, "build", "frhip", "*.o")):
        src = os.path.basename(o).split(".")[0]
        if src.startswith("build_id_"):
            src = "build_id"  # one build-stamp object: the latest
        if src == fname.split(".")[0] or src not in wanted:
            continue
        if src not in latest or os.path.getmtime(o) > os.path.getmtime(latest[src]):
            latest[src] = o
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, f"lib_{name}_{fname}")
    open(src, "w").write(text)
    obj = src + ".o"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", *EXTRA.get(fname, []),
                    "-I" + CSRC, "-I" + os.path.join(REPO, "include"), "-x", "hip", "-c", src, "-o", obj], check=True)
    so = os.path.join(OUT, f"lib_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", *latest.values(), obj, "-o", so],
                   check=True)
    print(so)


if __name__ == "__main__":
    main()
