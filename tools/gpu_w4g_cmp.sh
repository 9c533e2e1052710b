#!/bin/bash
# Same-box timing of F(4x4) kernel builds (tools/wv/w4g_<name>) on the IR stage shapes.
# ARGS: iters sk_mode no_split lanes (default "20 0 1 1"; serving split-K: "50 0 0 1" with B = 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SHAPES=${SHAPES:-"256,14,256,256,2 256,14,256,256,1 256,28,128,128,2 256,28,128,128,1 256,56,64,64,2 256,56,64,64,1 256,7,512,512,2 128,14,256,256,2"}
for s in $SHAPES; do
  shp=${s//,/ }
  for v in ${VARIANTS:-old base}; do
    echo -n "$v: "; timeout -k 5 60 tools/wv/w4g_$v $shp ${ARGS:-20 0 1 1} || { echo "failed rc=$?"; exit 3; }
  done
done
