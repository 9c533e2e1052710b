#!/bin/bash
# F(4x4) ablation variants (tools/w4g_variants.py) on the stage-1..4 shapes, one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base noepi nores nostore mfmaonly}; do
  for shp in "256 56 64 64 2" "256 56 64 64 1" "256 28 128 128 2" "256 14 256 256 2" "256 14 256 256 1"; do
    echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 20 0 1 1 || { echo "failed rc=$?"; exit 3; }
  done
done
