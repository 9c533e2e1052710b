#!/bin/bash
# Stage-1 F(4x4): part B's store variants (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for shp in "256 56 64 64 1" "256 112 64 64 1" "256 56 64 64 2"; do
  for rep in 1 2; do
    for v in base nopartb partb_nostore partb_small partb_nt; do
      echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp 30 || { echo "failed rc=$?"; exit 3; }
    done
  done
done
