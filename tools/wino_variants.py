#!/usr/bin/env python3
"""Schedule experiments on the Winograd kernel (tools only, not shipped).

Each variant is the product source (facerecognitionpipeline_amd/csrc/conv_winograd.hip)
with textual replacements, compiled together with tools/wino_bench.cpp's timing main into
tools/wv_<name>.  Run on the GPU box with ``tools/wino_variants.py run``.

usage: wino_variants.py build [names...] | run [names...]
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "facerecognitionpipeline_amd", "csrc", "conv_winograd.hip")
BENCH = os.path.join(REPO, "tools", "wino_bench.cpp")
OUT = os.path.join(REPO, "tools", "wv")

SCHED = "      if (i >= DSW_FROM) __builtin_amdgcn_sched_group_barrier(0x200, DSW_PER, 0);\n    }\n"

VARIANTS = {
    "base": [],
    "prio": [("  float4 dA[4], dB[4], pA[2], pB[2];",
              "  if (wid >= 4) __builtin_amdgcn_s_setprio(1);\n  float4 dA[4], dB[4], pA[2], pB[2];")],
    "nosched": [("    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);\n", ""),
                ("      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);\n"
                 "      __builtin_amdgcn_sched_group_barrier(0x020, VM_PER, 0);\n"
                 "      __builtin_amdgcn_sched_group_barrier(0x002, VALU_PER, 0);\n", ""),
                ("      if (i >= DSW_FROM) __builtin_amdgcn_sched_group_barrier(0x200, DSW_PER, 0);\n", "")],
    "valu2": [("constexpr int VALU_PER = PRE ? 8 : 4;", "constexpr int VALU_PER = 2;")],
    "valu12": [("constexpr int VALU_PER = PRE ? 8 : 4;", "constexpr int VALU_PER = PRE ? 12 : 8;")],
    "dswlate": [("constexpr int DSW_FROM = NMFMA / 2;", "constexpr int DSW_FROM = NMFMA - 4;")],
    "vm2": [("constexpr int VM_PER = (NVMEM + NMFMA - 1) / NMFMA;", "constexpr int VM_PER = 2;")],
}


def gen(name):
    s = open(SRC).read()
    for a, b in VARIANTS[name]:
        if a not in s:
            raise SystemExit(f"variant {name}: pattern not found: {a[:60]!r}")
        s = s.replace(a, b)
    b = open(BENCH).read().replace('#include "../facerecognitionpipeline_amd/csrc/conv_winograd.hip"',
                                   f'#include "wv_{name}.hip"')
    os.makedirs(OUT, exist_ok=True)
    open(os.path.join(OUT, f"wv_{name}.hip"), "w").write(s)
    open(os.path.join(OUT, f"wb_{name}.cpp"), "w").write(b)
    exe = os.path.join(OUT, f"wv_{name}")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(REPO, "include"),
           "-I" + os.path.join(REPO, "facerecognitionpipeline_amd", "csrc"), "-I" + OUT, "-x", "hip",
           os.path.join(OUT, f"wb_{name}.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-2000:])
        raise SystemExit(f"variant {name} failed to build")
    return exe


def main():
    mode = sys.argv[1]
    names = sys.argv[2:] or list(VARIANTS)
    if mode == "build":
        with ThreadPoolExecutor(8) as ex:
            for exe in ex.map(gen, names):
                print("built", exe)
    else:
        for n in names:
            print(f"== {n}", flush=True)
            subprocess.run(["timeout", "-k", "5", "60", os.path.join(OUT, f"wv_{n}"), "256", "20"], check=True)


if __name__ == "__main__":
    main()
