#!/bin/bash
# Serving conv kernel line touching: tests, then batch 1 / 2 latency vs the no-touch build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serving.py tests/test_gpu_kernels.py -x -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_touch.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_touch.log; [ $rc -gt 0 ] && exit $rc
NS=1,2 bash tools/gpu_so_ab.sh notouch
