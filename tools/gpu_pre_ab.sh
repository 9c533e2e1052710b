#!/bin/bash
# Serving conv kernel: conv1's pre-BN in the previous conv2's epilogue on / off (batch 1), the
# serving + kernel tests, a batch-1 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serving.py tests/test_gpu_kernels.py -x -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_pre.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_pre.log; [ $rc -gt 0 ] && exit $rc
timeout -k 10 300 python -u tools/serve_small_ab.py --pre-epilogue --ns 1 > gpurun_out/pre_ab.txt 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/pre_ab.txt
O=gpurun_out/b1pre
rm -rf $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/batch1_trace.py > gpurun_out/b1pre_trace.log 2>&1
echo "trace rc=$?"
python3 tools/batch1_summary.py $O > gpurun_out/b1pre_breakdown.txt 2>&1; head -16 gpurun_out/b1pre_breakdown.txt
