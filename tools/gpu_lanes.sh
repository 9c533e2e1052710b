#!/bin/bash
# Lane experiment: one F(4x4) layer launched back to back, one stream static / dynamic queue,
# or two half-batch streams (dynamic / static).  usage: bash tools/gpu_lanes.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for shp in "256 14 256 256 2" "256 14 256 256 1" "256 28 128 128 2" "256 56 64 64 2" "256 7 512 512 2"; do
  for mode in 1 2; do
    timeout -k 5 60 tools/wv/w4g_base $shp 20 0 1 $mode || { echo "failed rc=$?"; exit 3; }
  done
done
