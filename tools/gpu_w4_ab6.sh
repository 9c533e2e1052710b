#!/bin/bash
# Part-B output store cache policy (sc0 / sc1 / sc0 sc1) at stages 1 and 3, alternating, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 56 64 64 1" "256 112 64 64 1" "256 56 64 64 2" "256 28 128 128 2" "256 14 256 256 2"; do
  for rep in 1 2; do
    for v in base partb_sc0 partb_sc1 partb_sc01; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 30 || { echo "failed rc=$?"; exit 3; }
    done
  done
done
