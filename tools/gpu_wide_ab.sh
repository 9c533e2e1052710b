#!/bin/bash
# Wide / tall F(4x4) items (round 6): the parity tests of the kernel and the detector, then fr_detect
# timed with frt_set_wino4_shapes 1 / 0 / 1 / 0 (separate processes) and the C4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wide
mkdir -p $OUT
python3 -c "from facerecognitionpipeline_amd import _lib; print(_lib.load().fr_version().decode())" > $OUT/build.txt
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_winograd.py::test_winograd4_item_shapes tests/test_detector.py tests/test_gpu_detector_rows.py tests/test_gpu_c4_chain.py \
  > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $OUT/tests.log; exit 3; }
tail -3 $OUT/tests.log
for w in 1 0 1 0; do
  timeout -k 10 300 python3 tools/det_time.py --frames 32 --reps 30 --shapes $w >> $OUT/det_ab.txt 2>&1 \
    || { echo "det_time failed"; tail -20 $OUT/det_ab.txt; exit 3; }
done
cat $OUT/det_ab.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4_$i.json 2> $OUT/bench_c4_$i.err \
    || { echo "c4 bench failed rc=$?"; tail -20 $OUT/bench_c4_$i.err; exit 3; }
  cat $OUT/bench_c4_$i.json
done
