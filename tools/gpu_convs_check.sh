#!/bin/bash
# Serving conv kernel change check: kernel + serving tests, batch-1 latency, per-launch stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serving.py tests/test_gpu_kernels.py -x -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_cc.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_cc.log; [ $rc -gt 0 ] && exit $rc
timeout -k 10 200 python -u tools/serve_latency.py --algos winograd4 --ns 1,2,4 2>&1 | grep -v amdgpu.ids || exit 3
timeout -k 10 200 python -u tools/convs_stamps.py run 1 > gpurun_out/convs_stamps_cc.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/convs_stamps_cc.txt
