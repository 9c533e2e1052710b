#!/bin/bash
# Stage-1 F(4x4): what the deferred epilogue's part B and the residual loads cost (wrong results by
# design, timing only), and the per-wave accounting without part B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 56 64 64 2" "256 56 64 64 1" "256 112 64 64 1" "256 14 256 256 2"; do
  for rep in 1 2; do
    for v in base nopartb nores2; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 30 || { echo "failed rc=$?"; exit 3; }
    done
  done
  echo -n "stamps_nopartb: "; timeout -k 5 60 tools/wv/w4g_stamps_nopartb $shp 20 0 1 1 || exit 3
done
