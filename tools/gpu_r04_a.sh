#!/bin/bash
# Round 4, GPU session A: the new tests (hand-off error word, bench --gpus 2 launcher), the
# F(4x4) parity tests, an A/B of the deferred MODE-0 epilogue (tools/wv/w4g_base = HEAD's kernel,
# w4g_defer = working tree) on the IR-101 layer shapes, then one C3 bench line.
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
for rep in 1 2; do
  for shp in "256 112 64 64 1" "256 56 64 64 1" "256 56 64 64 2" "256 28 128 128 1" "256 28 128 128 2" "256 14 256 256 1" "256 14 256 256 2" "256 7 512 512 2"; do
    for v in base defer defer0; do
      echo -n "$v: " >> gpurun_out/w4ab.txt
      timeout -k 5 60 tools/wv/w4g_$v $shp 20 0 0 1 >> gpurun_out/w4ab.txt 2>&1 || { echo "w4g_$v failed"; exit 3; }
    done
  done
done
cat gpurun_out/w4ab.txt
step bench 400 python -u bench.py
