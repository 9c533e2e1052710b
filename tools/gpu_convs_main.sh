#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k serving --timeout 200 --timeout-method thread > gpurun_out/tests_cs.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests_cs.log; [ $rc -gt 0 ] && exit $rc
timeout -k 10 120 python -u tools/convs_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/convs_bench.py --n 4 2>&1 | grep -v amdgpu.ids
