#!/bin/bash
# One box's C3 and C4 lines back to back (box-to-box spread of the pool): appends to
# gpurun_out/c3c4_samples/<box>.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c3c4_samples
mkdir -p $OUT
F=$OUT/$(hostname)_$(date +%s).txt
python3 -c "from facerecognitionpipeline_amd import _lib; print(_lib.load().fr_version().decode())" > $F
for c in c3 c4 c3 c4; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $OUT/line.json 2> $OUT/line.err \
    || { echo "bench $c failed"; tail -20 $OUT/line.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/line.json'));print('$c', d['value'], d['ms_per_step'])" | tee -a $F
done
rm -f $OUT/line.json $OUT/line.err
