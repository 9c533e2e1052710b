#!/bin/bash
# Lanes: serving tests (lanes equivalence), then C3 bench at lane sizes 0 (off) / 128 / 85 / 64.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_serving.py -x -q --timeout 300 --timeout-method thread > gpurun_out/serving.log 2>&1 || { echo "serving tests failed"; tail -30 gpurun_out/serving.log; exit 3; }
tail -2 gpurun_out/serving.log
for cfg in ${CFGS:-"256 0" "256 128" "256 85" "256 64" "128 64" "128 42"}; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --batch $1 --lanes-min $2 > gpurun_out/bench_b$1_l$2.json 2> gpurun_out/bench_b$1_l$2.err || { echo "bench $cfg failed"; tail -5 gpurun_out/bench_b$1_l$2.err; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_b$1_l$2.json').read().strip().splitlines()[-1]); print('batch $1 lanes_min $2:', d['value'], d['ms_per_step'])"
done
