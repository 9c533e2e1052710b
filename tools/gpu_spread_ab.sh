#!/bin/bash
# Serving conv kernel: one workgroup per CU (96 KiB dynamic LDS for grids <= 256) vs the
# hardware's placement -- batch-1 latency A/B (same box, interleaved) and stamps of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in base spread; do
    so=facerecognitionpipeline_amd/libfrhip.so; [ $v = spread ] && so=tools/wv/lib_cs_spread.so
    echo -n "$v: "; timeout -k 10 120 python -u tools/serve_latency.py --algos winograd4 --ns 1 --so $so 2>&1 | grep -v amdgpu.ids || { echo failed; exit 3; }
  done
done
timeout -k 10 200 python -u tools/convs_stamps.py run 1 tools/wv/lib_cs_stamps_spread.so > gpurun_out/convs_stamps_spread.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/convs_stamps_spread.txt
