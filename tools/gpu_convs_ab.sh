#!/bin/bash
# conv_small.hip variants (tools/lib_variant.py builds in tools/wv): µs per launch by layer shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-cs_w4c12 cs_w8c18 cs_w8c9 cs_w4c18 cs_w4c12p cs_w8c18p}; do
  echo "== $v"
  timeout -k 10 120 python -u tools/convs_bench.py --so tools/wv/lib_$v.so 2>&1 | grep -v amdgpu.ids || { echo failed; exit 3; }
done
