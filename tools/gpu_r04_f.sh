#!/bin/bash
# Round 4, GPU session F: the whole GPU suite, a one-lane rocprof trace of the C3 bench per layer,
# the C3 bench line, serving latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -rfE > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -gt 0 ] && exit $rc
O=gpurun_out/prof_f
rm -rf $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --lanes-min 0 > gpurun_out/prof_f.log 2>&1 || { echo "trace failed"; exit 3; }
python3 tools/prof_summary.py $O > gpurun_out/layers_f.txt 2>&1
head -14 gpurun_out/layers_f.txt; tail -5 gpurun_out/layers_f.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_f.json 2>/dev/null
echo "bench rc=$?"; cut -c1-300 gpurun_out/bench_f.json
timeout -k 10 300 python -u tools/serve_latency.py --json gpurun_out/serve_latency.json > gpurun_out/serve_latency.txt 2>&1
echo "serve rc=$?"; grep -v amdgpu.ids gpurun_out/serve_latency.txt
