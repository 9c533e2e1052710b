#!/bin/bash
# Round 4, GPU session D: chained F(4x4) serving layers -- refactor A/B of the kernel body, the
# serving + hand-off tests, serving latency, one batch-1 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${AB:-1}" = 1 ]; then
  bash tools/gpu_w4_refactor_ab.sh > gpurun_out/refab.txt 2>&1 || { echo "refactor A/B failed"; cat gpurun_out/refab.txt; exit 3; }
  cut -c1-75 gpurun_out/refab.txt
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_serving.py tests/test_gpu_handoff_error.py -x -v --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_d.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/tests_d.log | tail -20; [ $rc -gt 0 ] && exit $rc
timeout -k 10 300 python -u tools/serve_latency.py --json gpurun_out/serve_latency.json > gpurun_out/serve_latency.txt 2>&1
echo "serve rc=$?"; cat gpurun_out/serve_latency.txt
O=gpurun_out/b1
rm -rf $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/batch1_trace.py > gpurun_out/b1_trace.log 2>&1
echo "trace rc=$?"
python3 tools/batch1_summary.py $O > gpurun_out/b1_breakdown.txt 2>&1; head -30 gpurun_out/b1_breakdown.txt
