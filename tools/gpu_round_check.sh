#!/bin/bash
# The driver's round-end sequence on one GPU, each step under its own limit, stopping at the first
# GPU failure: the whole -m gpu suite, smoke(), the default bench line (C3), then EXTRA (a command
# line, optional).  Logs under gpurun_out/$TAG_*.
#   TAG=r05b EXTRA="python -u tools/serve_small_ab.py --ns 1 --pixels 1024,4096" tools/gpu_round_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-check}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
tail -c 400 gpurun_out/${TAG}_bench.json
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 $EXTRA > gpurun_out/${TAG}_extra.txt 2>&1 || exit $?
  tail -5 gpurun_out/${TAG}_extra.txt
fi
exit $rc
