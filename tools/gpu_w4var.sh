#!/bin/bash
# Kernel-trace timing of the F(4x4) ablation variants (tools/w4_variants.sh) on one layer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LARGS=${LAYER_ARGS:-"--m 4 --B 256 --H 14 --cin 256 --cout 256 --epi 2 --iters 5"}
for L in tools/wv/lib_*.so; do
  V=$(basename $L .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wv/$V -o run -- python3 tools/w4_layer.py $LARGS --lib $L > gpurun_out/wv_$V.log 2>&1 || { echo "$V failed"; tail -5 gpurun_out/wv_$V.log; exit 3; }
  python3 tools/pmc_kernel.py wino4_kernel gpurun_out/wv/$V | tail -1 | sed "s#^#$V #"
done
