#!/bin/bash
# Batch-1 latency A/B of libfrhip.so builds on one box, interleaved: bash tools/gpu_so_ab.sh NAME...
# (NAME = tools/wv/lib_NAME.so; "base" = the package's build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for v in base "$@"; do
    so=facerecognitionpipeline_amd/libfrhip.so; [ $v != base ] && so=tools/wv/lib_$v.so
    echo -n "$v: "; timeout -k 10 120 python -u tools/serve_latency.py --algos winograd4 --ns ${NS:-1} --so $so 2>&1 | grep -v amdgpu.ids || { echo failed; exit 3; }
  done
done
