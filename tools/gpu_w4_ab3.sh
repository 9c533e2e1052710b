#!/bin/bash
# A/B of w4g_bench variants on the conv1 (pre-BN) shapes, alternating, 3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 14 256 256 1" "256 28 128 128 1" "256 56 64 64 1" "256 112 64 64 1" "256 7 512 512 1"; do
  for rep in 1 2 3; do
    for v in ${VARIANTS:-base noprio}; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 30 || { echo "failed rc=$?"; exit 3; }
    done
  done
done
