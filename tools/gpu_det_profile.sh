#!/bin/bash
# rocprofv3 passes over the C4 detector and the C4 step: a kernel trace + stats of
# tools/det_time.py (fr_detect on 32 seeded 1080p frames, alone on the GPU), one PMC pass per
# counter set over the same program, tools/det_prof_summary.py -> det_layers_pmc.{txt,json}
# (stamped with the library build), then a kernel trace + the same PMC passes of
# `bench.py --config c4` for the align / blur kernels (by kernel name).  Each pass has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/det_$TAG
mkdir -p $OUT
python3 -c "from facerecognitionpipeline_amd import _lib; print(_lib.load().fr_version().decode())" > $OUT/build.txt
echo "build: $(cat $OUT/build.txt)"
if [ "${DET:-1}" = "1" ]; then
timeout -k 10 300 python3 tools/det_time.py --frames 32 --reps 20 > $OUT/det_time.txt 2>&1 \
  || { echo "det_time failed rc=$?"; tail -20 $OUT/det_time.txt; exit 3; }
cat $OUT/det_time.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 tools/det_time.py --frames 32 --reps 5 > $OUT/trace.log 2>&1 \
  || { echo "trace pass failed rc=$?"; tail -20 $OUT/trace.log; exit 3; }
echo trace ok
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  D=$(echo $C | cut -d' ' -f1)
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$D -o run -- \
    python3 tools/det_time.py --frames 32 --reps 2 > $OUT/pmc_$D.log 2>&1 \
    || { echo "pmc $C failed rc=$?"; tail -20 $OUT/pmc_$D.log; exit 3; }
  echo pmc $C ok
done
python3 tools/det_prof_summary.py $OUT/trace --frames 32 --pmc $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE \
  $OUT/pmc_SQ_VALU_MFMA_BUSY_CYCLES --build "$(cat $OUT/build.txt)" --json $OUT/det_layers_pmc.json \
  > $OUT/det_layers_pmc.txt || { echo "summary failed"; exit 4; }
cat $OUT/det_layers_pmc.txt
fi
if [ "${C4:-1}" = "1" ]; then
  timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err \
    || { echo "c4 bench failed rc=$?"; tail -20 $OUT/bench_c4.err; exit 3; }
  cat $OUT/bench_c4.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4trace -o run -- \
    python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/c4trace.log 2>&1 \
    || { echo "c4 trace failed rc=$?"; tail -20 $OUT/c4trace.log; exit 3; }
  for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    D=$(echo $C | cut -d' ' -f1)
    timeout -k 10 -s KILL 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/c4pmc_$D -o run -- \
      python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c4pmc_$D.log 2>&1 \
      || { echo "c4 pmc $C failed rc=$?"; tail -20 $OUT/c4pmc_$D.log; exit 3; }
  done
  python3 -c "
import sys; sys.path.insert(0, '.')
from tools.prof_summary import by_kernel
by_kernel('$OUT/c4trace', ['$OUT/c4pmc_FETCH_SIZE', '$OUT/c4pmc_WRITE_SIZE', '$OUT/c4pmc_SQ_VALU_MFMA_BUSY_CYCLES'])
" > $OUT/c4_kernels_pmc.txt || { echo "c4 summary failed"; exit 4; }
  cat $OUT/c4_kernels_pmc.txt
  python3 tools/c4_timeline.py $OUT/c4trace --skip 3 > $OUT/c4_timeline.txt; cat $OUT/c4_timeline.txt
fi
