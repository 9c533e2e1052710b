#!/bin/bash
# Round 4, GPU session E: F(4x4) transform-wave fixes (pre-BN shift applied at store time, no
# overrun loads for 1-2 step streams) -- parity, kernel A/B vs the previous build, serving
# latency chained vs per-layer, chain phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_winograd.py tests/test_gpu_serving.py -x -q --timeout 300 \
  --timeout-method thread -rfE > gpurun_out/tests_e.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_e.log; [ $rc -gt 0 ] && exit $rc
bash tools/gpu_w4_refactor_ab.sh > gpurun_out/refab2.txt 2>&1 || { echo "A/B failed"; exit 3; }
cut -c1-75 gpurun_out/refab2.txt
VARIANTS="base off" bash tools/gpu_chain_ab.sh > gpurun_out/chain_ab2.txt 2>&1 || { echo "chain A/B failed"; exit 3; }
cat gpurun_out/chain_ab2.txt
timeout -k 10 200 python3 tools/chain_stamps.py run 1 > gpurun_out/chain_stamps2.txt 2>&1 || { echo "stamps failed"; exit 3; }
grep -v amdgpu.ids gpurun_out/chain_stamps2.txt | tail -4
