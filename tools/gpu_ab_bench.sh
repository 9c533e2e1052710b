#!/bin/bash
# Same-box A/B of the C3 bench: this tree's libfrhip.so vs tools/wv/libfrhip_old.so (built from
# an earlier commit), alternating, ROUNDS times each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OLD=/tmp/ab_old
rm -rf $OLD && mkdir -p $OLD && cp -r facerecognitionpipeline_amd oracle bench.py __graft_entry__.py $OLD/ && \
  cp tools/wv/libfrhip_old.so $OLD/facerecognitionpipeline_amd/libfrhip.so || exit 2
for r in $(seq ${ROUNDS:-2}); do
  for side in new old; do
    d=.; [ $side = old ] && d=$OLD
    (cd $d && timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null) | python3 -c "
import json,sys
j=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$side', j['value'], 'faces/s', j['ms_per_step'], 'ms/step profiled', j.get('ms_per_step_profiled_pass'), 'frac', j['roofline']['frac'], 'avg_launch_ms', j['roofline']['avg_launch_ms'])" || exit 3
  done
done
