#!/bin/bash
# Serving latency of libfrhip.so variants (VARIANTS: tools/wv/lib_<v>.so), alternating, 2 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in ${VARIANTS:-cs_oldlds cs_fold}; do
    echo -n "$v: "; timeout -k 10 120 python -u tools/serve_latency.py --algos winograd4 --ns 1 --so tools/wv/lib_$v.so 2>&1 | grep -v amdgpu.ids || { echo failed; exit 3; }
  done
done
