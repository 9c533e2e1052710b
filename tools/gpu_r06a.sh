#!/bin/bash
# round-6 first call: the changed blur / gate / process_image tests, then the detector profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_align.py \
  tests/test_gpu_gate.py > gpurun_out/r06a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r06a_tests.log
[ $rc -le 1 ] || exit $rc
TAG=r06 timeout -k 10 1000 tools/gpu_det_profile.sh > gpurun_out/det_r06.log 2>&1
rc2=$?
tail -70 gpurun_out/det_r06.log
exit $(( rc2 ? rc2 : rc ))
