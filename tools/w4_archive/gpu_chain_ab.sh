#!/bin/bash
# Chained F(4x4) serving layers: batch-1/4 embed latency of library variants (tools/lib_variant.py
# builds: ch_base = the chain as shipped, ch_off = per-layer launches, ch_no* = one phase removed,
# wrong results by design).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-base off nolayerwait noitemwait noreduce nobody}; do
  echo "== $v"
  timeout -k 10 120 python -u tools/serve_latency.py --algos winograd4 --ns 1,4 --so tools/wv/lib_ch_$v.so 2>&1 | grep -v amdgpu.ids || { echo "failed"; exit 3; }
done
