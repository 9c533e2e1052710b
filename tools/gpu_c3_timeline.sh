#!/bin/bash
# kernel trace of the C3 bench (two lanes, and one lane) -> tools/c4_timeline.py (GPU idle per step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c3tl
mkdir -p $OUT
for L in "" "--lanes-min 0"; do
  D=$OUT/trace$(echo $L | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- \
    python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline $L > $D.log 2>&1 || { echo "trace failed"; tail $D.log; exit 3; }
  echo "== C3 $L"; tail -1 $D.log | cut -c1-200
  python3 tools/c4_timeline.py $D --skip 3 --gaps 8
done
