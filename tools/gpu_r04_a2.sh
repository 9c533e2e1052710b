#!/bin/bash
# Round 4, GPU session A2: hand-off error + F(4x4) parity tests, then an A/B of round 3's kernel
# (w4g_base) against the working tree (w4g_cur, sk 0 whole items / sk 1 stream-K tail), 3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_handoff_error.py tests/test_gpu_winograd.py -x -v --timeout 400 \
  --timeout-method thread -rfE > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -gt 1 ] && exit $rc
: > gpurun_out/w4ab2.txt
run() {  # variant sk lanes shape...
  local v=$1 sk=$2 nl=$3; shift 3
  echo -n "$v/sk$sk/l$nl: " >> gpurun_out/w4ab2.txt
  timeout -k 5 60 tools/wv/w4g_$v "$@" 20 $sk 0 $nl >> gpurun_out/w4ab2.txt 2>&1 || { echo "w4g_$v failed"; exit 3; }
}
for rep in 1 2 3; do
  for shp in "256 56 64 64 2" "256 28 128 128 1" "256 28 128 128 2" "256 14 256 256 1" "256 14 256 256 2"; do
    run base 0 1 $shp
    run cur 0 1 $shp
    run cur 1 1 $shp
  done
done
cat gpurun_out/w4ab2.txt
