#!/bin/bash
# Full GPU suite on the tree's libfrhip.so, then (box-local copy only) on the batch-1 4096-pixel
# variant tools/wv/lib_m4096.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="allgpu smoke" bash tools/gpu_session.sh || exit 3
cp tools/wv/lib_m4096.so facerecognitionpipeline_amd/libfrhip.so
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rfE > gpurun_out/allgpu_m4096.log 2>&1
rc=$?; echo "m4096 allgpu rc=$rc"; tail -3 gpurun_out/allgpu_m4096.log
