#!/bin/bash
# One GPU call of experiment runs: each argument after OUT is a command line (run by bash -c, so
# "W6_ZERO_SHIFT=1 tools/w6/w6_bench 3 14 256 256 1 5 3" and inner quotes work), run under its own
# `timeout -k 10 ${T:-60}`, output appended to gpurun_out/OUT.  Exit status 1 (a bench's
# "values beyond tolerance") is recorded and the list goes on; anything else (fault, abort, time
# limit) ends the call there.
#   gpurun -- 'tools/gpu_exp.sh w4s.txt "tools/w6/w4s_bench 256 14 256 256 2 20" "tools/w6/w4s_ur6 256 14 256 256 2 20"'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/$1
shift
mkdir -p gpurun_out
: > "$out"
for cmd in "$@"; do
  echo "== $cmd" >> "$out"
  timeout -k 10 "${T:-60}" bash -c "$cmd" >> "$out" 2>&1
  rc=$?
  echo "rc=$rc" >> "$out"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cat "$out"; exit $rc; fi
done
cat "$out"
