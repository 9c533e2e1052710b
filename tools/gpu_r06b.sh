#!/bin/bash
# round 6: detector row reduction + pipelined C4 -- tests, then the detector / C4 profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_detector_rows.py \
  tests/test_detector.py tests/test_gpu_c4_chain.py > gpurun_out/r06b_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r06b_tests.log
[ $rc -le 1 ] || exit $rc
TAG=${TAG:-r06b} timeout -k 10 1000 tools/gpu_det_profile.sh > gpurun_out/det_${TAG:-r06b}.log 2>&1
rc2=$?
tail -60 gpurun_out/det_${TAG:-r06b}.log
exit $(( rc2 ? rc2 : rc ))
