#!/bin/bash
# round 6: changed tests, then C4 / C3 lines (lanes A/B for C4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_detector_rows.py \
  tests/test_gpu_gallery.py tests/test_align.py tests/test_gpu_gate.py tests/test_gpu_c4_chain.py > gpurun_out/r06d_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r06d_tests.log
[ $rc -le 1 ] || exit $rc
for a in "--config c4" "--config c4 --lanes-min 0" "--config c3" "--config c4"; do
  timeout -k 10 300 python3 bench.py $a --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06d_b.json 2>gpurun_out/r06d_b.err || exit 3
  python3 -c "import json;d=json.load(open('gpurun_out/r06d_b.json'));print('$a', d['value'], d['ms_per_step'])"
done
exit $rc
