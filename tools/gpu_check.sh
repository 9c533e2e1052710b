#!/bin/bash
# GPU box: full -m gpu suite, then (only if pytest ended normally, no timeout) one C3 bench line.
# usage: tools/gpu_check.sh [pytest selection...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
SEL="${@:-tests}"
timeout -k 10 1500 python -u -m pytest $SEL -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|error" gpurun_out/gputest.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/gputest.log | head -20
if [ $rc -gt 1 ] || grep -q "Timeout" gpurun_out/gputest.log; then
  echo "pytest did not end normally: no further GPU steps"; exit $rc
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
echo "bench rc=$?"
cat gpurun_out/bench_c3.json
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
  echo "rocprof rc=$?"
  python3 tools/prof_summary.py gpurun_out/prof/ > gpurun_out/layers.txt 2>&1 || true
  head -5 gpurun_out/prof/*/run_kernel_stats.csv 2>/dev/null | cut -c1-200
fi
