#!/bin/bash
# Round-3 same-box A/B: stem store variants (tools/stem_variants.py) and the split-K U ring
# depth at serving batch 1 (tools/w4g_variants.py u18split).  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${STEMS:-rows16 nt rows8nt rows28nt rows16}; do
  echo -n "stem $v: "
  timeout -k 10 120 python tools/stem_bench.py --so tools/wv/stem_$v.so 2>/dev/null | head -1 || { echo "stem $v failed"; exit 3; }
done
VARIANTS="${W4:-base u18split}" SHAPES="1,14,256,256,1 1,14,256,256,2 1,28,128,128,2 1,56,64,64,2 1,7,512,512,2 1,112,64,64,1" \
  ARGS="50 0 0 1" bash tools/gpu_w4g_cmp.sh
