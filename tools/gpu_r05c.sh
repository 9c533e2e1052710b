#!/bin/bash
# round 5 call c: channel-blocked F(4x4) activations -- bitwise tests, layout A/B per layer shape
# (all blocked, and both seam forms), C3 same-process A/B of the switch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_blocked.py \
  tests/test_gpu_winograd.py tests/test_gpu_pipeline.py > gpurun_out/r05c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="base:0 base:7 base:5 base:3" SHAPES="256 56 64 64 2;256 28 128 128 2;256 14 256 256 2;256 7 512 512 2" REPS=2 \
  timeout -k 10 400 tools/gpu_w4_ab.sh > gpurun_out/r05c_ab2.txt 2>&1 || exit $?
VARIANTS="base:0 base:5" SHAPES="256 112 64 64 1;256 56 64 64 1;256 28 128 128 1;256 14 256 256 1" REPS=2 \
  timeout -k 10 400 tools/gpu_w4_ab.sh > gpurun_out/r05c_ab1.txt 2>&1 || exit $?
python3 tools/ab_summary.py gpurun_out/r05c_ab2.txt; python3 tools/ab_summary.py gpurun_out/r05c_ab1.txt
timeout -k 10 500 python -u tools/c3_switch_ab.py frt_set_wino4_blocked --reps 6 > gpurun_out/r05c_c3ab.txt 2>&1 || exit $?
cat gpurun_out/r05c_c3ab.txt
