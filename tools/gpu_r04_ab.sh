#!/bin/bash
# A/B of F(4x4) kernel builds (tools/wv/w4g_<v> for v in $V, the first is the reference) on the
# IR-101 layer shapes, whole items, one stream, REPS repetitions alternating.
# usage: V="cur fdiv" tools/gpu_r04_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_$(echo $V | tr ' ' '_').txt
: > $OUT
for rep in $(seq ${REPS:-3}); do
  for shp in "256 112 64 64 1" "256 56 64 64 1" "256 56 64 64 2" "256 28 128 128 1" "256 28 128 128 2" \
             "256 14 256 256 1" "256 14 256 256 2" "256 7 512 512 2"; do
    for v in $V; do
      echo -n "$v: " >> $OUT
      timeout -k 5 60 tools/wv/w4g_$v $shp 20 0 0 1 >> $OUT 2>&1 || { echo "w4g_$v failed"; exit 3; }
    done
  done
done
python3 tools/ab_table.py $OUT
