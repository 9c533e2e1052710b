#!/bin/bash
# round 6: the whole -m gpu suite after the library cleanup, then C3 A/B of the pre-cleanup build
# (tools/wv/libfrhip_pre_cleanup.so via FRHIP_LIB) against this tree's, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests \
  > gpurun_out/r06f_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06f_tests.log
[ $rc -le 1 ] || exit $rc
for i in 1 2 3; do
  for v in pre new; do
    if [ $v = pre ]; then export FRHIP_LIB=$PWD/tools/wv/libfrhip_pre_cleanup.so; else unset FRHIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06f_b.json 2>gpurun_out/r06f_b.err || exit 3
    python3 -c "import json;d=json.load(open('gpurun_out/r06f_b.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['library_build'][-16:])"
  done
done
unset FRHIP_LIB
exit $rc
