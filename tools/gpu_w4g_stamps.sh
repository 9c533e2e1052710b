#!/bin/bash
# Per-wave cycle accounting of the F(4x4) kernel (w4g_variants.py "stamps") next to the base timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 14 256 256 2" "256 14 256 256 1" "256 28 128 128 2" "256 56 64 64 2" "256 56 64 64 1" "256 7 512 512 2"; do
  for v in ${VARIANTS:-base stamps}; do
    echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 20 0 1 1 || { echo "failed rc=$?"; exit 3; }
  done
done
