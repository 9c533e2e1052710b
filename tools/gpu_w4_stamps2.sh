#!/bin/bash
# Per-wave cycle accounting (w4g_variants.py "stamps") of the F(4x4) kernel by stage, B = 256,
# whole items (no stream-K tail), one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 112 64 64 1" "256 56 64 64 1" "256 56 64 64 2" "256 28 128 128 2" "256 14 256 256 1" "256 14 256 256 2" "256 7 512 512 2"; do
  echo "== $shp"
  timeout -k 5 60 tools/wv/w4g_stamps $shp 20 0 1 1 || { echo "failed rc=$?"; exit 3; }
done
