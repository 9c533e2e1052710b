#!/bin/bash
# Bench lines for every BASELINE config preset (one process each, own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/benches
for C in ${CONFIGS:-c3 c2 c4 c5}; do
  timeout -k 10 400 python bench.py --config $C ${EXTRA:-} > gpurun_out/benches/$C.log 2>&1 || { echo "$C failed rc=$?"; tail -5 gpurun_out/benches/$C.log; exit 3; }
  grep '^{' gpurun_out/benches/$C.log | tail -1 > gpurun_out/benches/$C.json
  python3 -c "import json;d=json.load(open('gpurun_out/benches/$C.json'));print('$C', d['value'], d['unit'], d['ms_per_step'], 'ms/step')"
done
