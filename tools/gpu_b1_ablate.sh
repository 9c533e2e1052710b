#!/bin/bash
# Batch-1 split-K F(4x4) layers: per-launch time (wino4 + its fixup) of the base kernel and of the
# ablation variants built by tools/w4g_variants.py (wrong results by design; timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "1 14 256 256 2" "1 14 256 256 1" "1 28 128 128 2" "1 56 64 64 2" "1 7 512 512 2"; do
  for v in ${VARIANTS:-base nouload noload notrans nomfma u18split}; do
    echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 200 0 0 1 || { echo "failed rc=$?"; exit 3; }
  done
done
