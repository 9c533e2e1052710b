#!/bin/bash
# Round 4, GPU session C: the stride-2 band kernel -- its parity tests, a one-lane rocprof trace of
# the C3 bench summarised per layer, then one C3 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -x -v --timeout 400 \
  --timeout-method thread -rfE > gpurun_out/tests_c.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_c.log; [ $rc -gt 0 ] && exit $rc
O=gpurun_out/prof_c
rm -rf $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --lanes-min 0 > gpurun_out/prof_c.log 2>&1 || { echo "trace failed"; exit 3; }
python3 tools/prof_summary.py $O > gpurun_out/layers_c.txt 2>&1
head -12 gpurun_out/layers_c.txt; tail -5 gpurun_out/layers_c.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c.json 2>/dev/null
echo "bench rc=$?"; cat gpurun_out/bench_c.json | cut -c1-400
