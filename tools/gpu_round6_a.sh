#!/bin/bash
# Round-6 evidence, call A: the driver's round-end sequence (-m gpu suite, smoke, C3 bench line),
# then the C3 kernel trace + PMC profile of this build (tools/gpu_profile.sh, TAG=r06).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r06 tools/gpu_round_check.sh
rc=$?; [ $rc -le 1 ] || exit $rc
TAG=r06 PMC=1 timeout -k 10 900 tools/gpu_profile.sh > gpurun_out/r06_profile.log 2>&1 || { tail -20 gpurun_out/r06_profile.log; exit 3; }
tail -22 gpurun_out/prof_r06/layers_pmc.txt
exit $rc
