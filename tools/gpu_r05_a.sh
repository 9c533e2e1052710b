#!/bin/bash
# round 5, call a: new GPU tests (pickle gallery, numpy-exact blur, reference gate fixture, bench
# exchange fields) then the F(4x4) A/B of channel-blocked / pre-BN-elsewhere variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_gate.py \
  tests/test_align.py tests/test_gpu_gallery.py tests/test_gpu_bench_launch.py > gpurun_out/r05a_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05a_tests.log
[ $rc -le 1 ] || exit $rc
VARIANTS="base cblk nopre y2store cblk_nopre_y2" REPS=2 timeout -k 10 600 tools/gpu_w4_ab.sh > gpurun_out/r05a_ab.txt 2>&1
echo ab rc=$?
