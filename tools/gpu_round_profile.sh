#!/bin/bash
# The round's evidence in one call: the driver's round-end sequence (tools/gpu_round_check.sh:
# -m gpu suite, smoke, the default bench line), then tools/gpu_profile.sh (kernel trace + the three
# PMC passes + prof_summary, stamped with the library build) for the C3 workload, then the bench
# line again so that its roofline carries this build's PMC figures once they are committed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05} tools/gpu_round_check.sh
rc=$?; [ $rc -le 1 ] || exit $rc   # 1: a test failed (its log says which); anything else: stop here
TAG=${TAG:-r05} PMC=1 timeout -k 10 1500 tools/gpu_profile.sh || exit $?
tail -25 gpurun_out/prof_${TAG:-r05}/layers_pmc.txt
exit $rc
