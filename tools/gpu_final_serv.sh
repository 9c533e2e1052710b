#!/bin/bash
# Serving: pixel threshold 1024 vs 4096 (batch 1 / 2), the batch-1 kernel trace breakdown, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NS=1,2 bash tools/gpu_so_ab.sh m4096 || exit 3
O=gpurun_out/b1f
rm -rf $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/batch1_trace.py > gpurun_out/b1f_trace.log 2>&1 || exit 3
python3 tools/batch1_summary.py $O > gpurun_out/b1f_breakdown.txt 2>&1; head -16 gpurun_out/b1f_breakdown.txt
timeout -k 10 200 python -u tools/convs_stamps.py run 1 > gpurun_out/convs_stamps_final.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/convs_stamps_final.txt
