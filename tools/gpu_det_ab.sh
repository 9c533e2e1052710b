#!/bin/bash
# Detector change check: the detector parity tests, fr_detect timing (twice), the C4 bench (twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/detab
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_detector.py tests/test_gpu_detector_rows.py tests/test_gpu_c4_chain.py ${EXTRA_TESTS:-} \
  > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $OUT/tests.log; exit 3; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 tools/det_time.py --frames 32 --reps 30 >> $OUT/det.txt 2>&1 || { tail -20 $OUT/det.txt; exit 3; }
done
grep frames $OUT/det.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4_$i.json 2> $OUT/bench_c4_$i.err \
    || { echo "c4 bench failed rc=$?"; tail -20 $OUT/bench_c4_$i.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/bench_c4_$i.json'));print('c4', d['value'], d['ms_per_step'])"
done
