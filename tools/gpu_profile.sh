#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Each pass has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
# the library build the profile is of (fr_version(): "... build <content hash>"); bench.py attaches
# the PMC figures only to runs of the same build
python3 -c "from facerecognitionpipeline_amd import _lib; print(_lib.load().fr_version().decode())" > $OUT/build.txt
echo "build: $(cat $OUT/build.txt)"
PARGS=${PMC_ARGS:-"--steps 1 --warmup 1 --no-cpu-baseline --lanes-min 0"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $BARGS > $OUT/trace_bench.log 2>&1 || { echo "trace pass failed rc=$?"; tail -20 $OUT/trace_bench.log; exit 3; }
echo trace ok; tail -1 $OUT/trace_bench.log
if [ "${PMC:-1}" = "1" ]; then
# one pass per counter set: FETCH_SIZE (3 TCC), WRITE_SIZE (2 TCC), MFMA busy + GPU clock (1 SQ + 1 GRBM)
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  D=$(echo $C | cut -d' ' -f1)
  timeout -k 10 -s KILL 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$D -o run -- \
    python3 bench.py $PARGS > $OUT/pmc_$D.log 2>&1 || { echo "pmc $C failed rc=$?"; tail -20 $OUT/pmc_$D.log; exit 3; }
  echo pmc $C ok
done
fi
if [ "${PMC:-1}" = "1" ]; then
  python3 tools/prof_summary.py $OUT/trace --batch ${SUMMARY_BATCH:-256} --pmc $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE \
    $OUT/pmc_SQ_VALU_MFMA_BUSY_CYCLES --build "$(cat $OUT/build.txt)" --json $OUT/layers_pmc.json > $OUT/layers_pmc.txt
else
  python3 tools/prof_summary.py $OUT/trace --batch ${SUMMARY_BATCH:-256} --build "$(cat $OUT/build.txt)" > $OUT/layers.txt
fi
find $OUT -name "*.csv" | head -20
