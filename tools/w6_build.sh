#!/bin/bash
# Builds tools/w6/w6_bench (the experimental F(6x6) kernel + the shipping F(4x4) kernel, one binary),
# or with SRC=w4s tools/w6/w4s_bench (the symmetric-wave F(4x4) experiment; since round 6 both the
# symmetric kernel and the F(4x4) kernel it is compared with -- the round-5 form with the stream-K
# tail and the chained launch -- come from tools/w4_archive/, which the library no longer builds).
# Extra hipcc flags
# (e.g. -DW6_PSTART=6 -DW6_PSTRIDE=1, or -I<dir> to take a variant of a kernel source from <dir>) go in
# W6_FLAGS; NAME names the binary.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$REPO/facerecognitionpipeline_amd/csrc
W4SRC=$CSRC/conv_winograd4.hip
[ "${SRC:-w6}" = w4s ] && W4SRC=$REPO/tools/w4_archive/conv_winograd4_streamk_chain.hip
mkdir -p "$REPO/tools/w6"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize ${W6_FLAGS:-} -I"$REPO/tools/w4_archive" \
  -I"$CSRC" -I"$REPO/include" -I"$REPO/tools" -x hip "$REPO/tools/${SRC:-w6}_bench.cpp" -x hip "$W4SRC" \
  -o "$REPO/tools/w6/${NAME:-${SRC:-w6}_bench}"
