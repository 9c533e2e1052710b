#!/bin/bash
# Builds tools/w6/w6_bench (the experimental F(6x6) kernel + the shipping F(4x4) kernel, one binary),
# or with SRC=w4s tools/w6/w4s_bench (the symmetric-wave F(4x4) experiment).  Extra hipcc flags
# (e.g. -DW6_PSTART=6 -DW6_PSTRIDE=1, or -I<dir> to take a variant of a kernel source from <dir>) go in
# W6_FLAGS; NAME names the binary.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$REPO/facerecognitionpipeline_amd/csrc
mkdir -p "$REPO/tools/w6"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize ${W6_FLAGS:-} -I"$CSRC" -I"$REPO/include" \
  -I"$REPO/tools" -x hip "$REPO/tools/${SRC:-w6}_bench.cpp" -x hip "$CSRC/conv_winograd4.hip" -o "$REPO/tools/w6/${NAME:-${SRC:-w6}_bench}"
