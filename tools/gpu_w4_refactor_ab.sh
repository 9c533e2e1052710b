#!/bin/bash
# A/B of two builds of the F(4x4) kernel on w4g_bench (B = 256 shapes + batch-1 split-K), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 14 256 256 2" "256 14 256 256 1" "256 28 128 128 2" "256 56 64 64 2" "1 14 256 256 2" "1 56 64 64 1"; do
  for rep in 1 2; do
    for v in ${VARIANTS:-old base}; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 50 || { echo "failed rc=$?"; exit 3; }
    done
  done
done
