#!/bin/bash
# One GPU-box session: kernel parity, pipeline parity, bench.  Each GPU step has its
# own time limit; a step that crashes (exit >1: signal, abort, timeout) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  return $rc
}
STEPS=${STEPS:-"kernels pipeline bench"}
for s in $STEPS; do
  case $s in
    kernels)  step kernels 900 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -rfE; rc=$? ;;
    pipeline) step pipeline 1200 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread -rfE; rc=$? ;;
    allgpu)   step allgpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rfE; rc=$? ;;
    sweep)    step sweep 900 python tools/conv_sweep.py --json gpurun_out/sweep.json; rc=$? ;;
    smoke)    step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"; rc=$? ;;
    bench)    step bench 900 python bench.py ${BENCH_ARGS:-}; rc=$? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  if [ $rc -gt 1 ]; then echo "stopping after $s (rc=$rc)"; exit $rc; fi
done
