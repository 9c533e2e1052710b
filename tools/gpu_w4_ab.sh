#!/bin/bash
# Same-box A/B of F(4x4) kernel variants (tools/w4g_variants.py build <names> first, here).
# Every shape runs every variant in turn, REPS times, alternating, so clock drift hits all alike.
#   VARIANTS="base cblk" SHAPES="256 14 256 256 1;256 14 256 256 2" REPS=3 tools/gpu_w4_ab.sh
# A shape is "B H Cin Cout epi" (epi 1: pre-BN + BN + PReLU = conv1, 2: BN + residual = conv2).
# A variant name may carry a layout suffix "name:blk" (W4_BLK_* bits of Wino4Params.blk).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS=${VARIANTS:-"base"}
SHAPES=${SHAPES:-"256 112 64 64 1;256 56 64 64 1;256 56 64 64 2;256 28 128 128 1;256 28 128 128 2;256 14 256 256 1;256 14 256 256 2;256 7 512 512 2"}
REPS=${REPS:-2}
ITERS=${ITERS:-30}
IFS=';' read -ra SH <<< "$SHAPES"
for shp in "${SH[@]}"; do
  for rep in $(seq $REPS); do
    for vb in $VARIANTS; do
      v=${vb%%:*}; blk=0; [ "$vb" != "$v" ] && blk=${vb#*:}
      # argv: shape, iterations, sk_mode 0 (whole items: the runtime's default), no_split 1, lanes 1, layouts
      out=$(timeout -k 5 60 tools/wv/w4g_$v $shp $ITERS 0 1 1 $blk) || { echo "$vb $shp failed rc=$?"; exit 3; }
      echo "$vb | $out"
    done
  done
done
