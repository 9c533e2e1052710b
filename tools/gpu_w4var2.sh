#!/bin/bash
# stage-3 and stage-2 layer timings of every tools/wv/lib_*.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LAYER_ARGS="--m 4 --B 256 --H 14 --cin 256 --cout 256 --epi 2 --iters 5" bash tools/gpu_w4var.sh || exit 3
for d in gpurun_out/wv/lib_*; do mv $d ${d}_s3; done
LAYER_ARGS="--m 4 --B 256 --H 28 --cin 128 --cout 128 --epi 2 --iters 5" bash tools/gpu_w4var.sh || exit 3
for d in gpurun_out/wv/lib_*; do case $d in *_s3) ;; *) mv $d ${d}_s2;; esac; done
