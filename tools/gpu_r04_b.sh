#!/bin/bash
# Round 4, GPU session B: rocprofv3 kernel trace + PMC passes (HBM bytes, MFMA busy cycles) of the
# one-lane C3 bench (tools/gpu_profile.sh), the per-layer summary, then the C2 / C4 / C5 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04 BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --lanes-min 0" bash tools/gpu_profile.sh || exit 3
O=gpurun_out/prof_r04
python3 tools/prof_summary.py $O/trace --pmc $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/pmc_SQ_VALU_MFMA_BUSY_CYCLES \
  --json $O/layers_pmc.json > $O/layers_pmc.txt 2>&1
python3 tools/prof_summary.py $O/trace > $O/layers.txt 2>&1
cat $O/layers_pmc.txt | tail -30
for c in c2 c5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; exit 3; }
  echo "$c: $(cat gpurun_out/bench_$c.json)"
done
timeout -k 10 400 python -u bench.py --config c4 --steps 10 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench c4 failed"; exit 3; }
echo "c4: $(cat gpurun_out/bench_c4.json)"
