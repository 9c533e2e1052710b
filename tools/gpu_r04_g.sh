#!/bin/bash
# Round 4, GPU session G: the serving conv kernel (conv_small.hip) -- kernel + serving tests,
# latency vs the F(4x4) split-K path per batch size, a batch-1 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_serving.py -x -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_g.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests_g.log; [ $rc -gt 0 ] && exit $rc
timeout -k 10 300 python -u tools/serve_small_ab.py > gpurun_out/serve_small_ab.txt 2>&1
echo "ab rc=$?"; grep -v amdgpu.ids gpurun_out/serve_small_ab.txt
O=gpurun_out/b1g
rm -rf $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/batch1_trace.py > gpurun_out/b1g_trace.log 2>&1
echo "trace rc=$?"
python3 tools/batch1_summary.py $O > gpurun_out/b1g_breakdown.txt 2>&1; head -16 gpurun_out/b1g_breakdown.txt
