#!/bin/bash
# Round 4, GPU session A: the new tests (hand-off error word, bench --gpus 2 launcher), the
# F(4x4) parity tests, an A/B of the F(4x4) kernel versions on the IR-101 layer shapes
# (tools/wv/w4g_base = round 3's kernel, w4g_defer = deferred epilogue, w4g_cur = working tree;
# cur at sk 0 = whole items, sk 1 = whole-item rounds + stream-K tail), then one C3 bench line.
# Every GPU step has its own time limit; a step that ends abnormally (rc > 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  return $rc
}
step tests 900 python -u -m pytest tests/test_gpu_handoff_error.py tests/test_gpu_winograd.py tests/test_gpu_bench_launch.py \
  -x -v --timeout 400 --timeout-method thread -rfE
rc=$?; [ $rc -gt 1 ] && exit $rc
: > gpurun_out/w4ab.txt
run() {  # variant sk lanes shape...
  local v=$1 sk=$2 nl=$3; shift 3
  echo -n "$v/sk$sk/l$nl: " >> gpurun_out/w4ab.txt
  timeout -k 5 60 tools/wv/w4g_$v "$@" 20 $sk 0 $nl >> gpurun_out/w4ab.txt 2>&1 || { echo "w4g_$v failed"; exit 3; }
}
for rep in 1 2; do
  for shp in "256 112 64 64 1" "256 56 64 64 1" "256 56 64 64 2" "256 28 128 128 1" "256 28 128 128 2" \
             "256 14 256 256 1" "256 14 256 256 2" "256 7 512 512 2"; do
    run base 0 1 $shp
    run defer 0 1 $shp
    run cur 0 1 $shp
    run cur 1 1 $shp
  done
done
for shp in "256 28 128 128 2" "256 14 256 256 1" "256 14 256 256 2"; do
  run cur 0 2 $shp
  run cur 1 2 $shp
done
cat gpurun_out/w4ab.txt
step bench 400 python -u bench.py
