#!/bin/bash
# Copies the evidence of `TAG=rNN tools/gpu_round_profile.sh` (merged back into gpurun_out/) into
# profiles/rNN/: the bench line, the stamped PMC profile, the kernel-trace summary, the GPU suite
# log and smoke().  Run here after the gpurun call:  TAG=r05 tools/collect_round.sh
set -euo pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:?set TAG, e.g. TAG=r05}
P=gpurun_out/prof_$TAG
D=profiles/$TAG
mkdir -p "$D"
cp "$P/layers_pmc.txt" "$P/layers_pmc.json" "$P/build.txt" "$D/"
cp "$P/trace/run_kernel_stats.csv" "$D/rocprof_kernel_stats.csv"
cp "gpurun_out/${TAG}_tests.log" "$D/pytest_gpu_log.txt"
cp "gpurun_out/${TAG}_smoke.log" "$D/smoke.txt"
cp "gpurun_out/${TAG}_bench.json" "$D/bench_c3.json"
echo "collected $(cat "$D/build.txt") into $D"
