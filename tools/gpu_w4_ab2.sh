#!/bin/bash
# A/B of w4g_bench variants (VARIANTS, default "base nomad"), alternating, 3 reps, B = 256 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 56 64 64 1" "256 56 64 64 2" "256 112 64 64 1" "256 28 128 128 2" "256 14 256 256 1" "256 14 256 256 2" "1 14 256 256 2"; do
  for rep in 1 2 3; do
    for v in ${VARIANTS:-base nomad}; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 30 || { echo "failed rc=$?"; exit 3; }
    done
  done
done
