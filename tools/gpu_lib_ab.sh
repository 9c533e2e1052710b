#!/bin/bash
# Same-box A/B of library builds (the package's and tools/lib_variant.py variants): fr_detect time
# (tools/det_time.py --so) alternating ROUNDS times, then, with C4=1, one C4 line per build
# (FRHIP_LIB), C4 rounds of them.  usage: LIBS="tools/ab_libs/lib_x.so ..." [ROUNDS=3] [C4=2] tools/gpu_lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lib_ab
mkdir -p $OUT
: > $OUT/det.txt
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in "" ${LIBS}; do
    timeout -k 10 300 python3 tools/det_time.py --frames 32 --reps 30 ${so:+--so $so} 2>/dev/null | grep frames >> $OUT/det.txt \
      || { echo "det_time failed ($so)"; exit 3; }
  done
done
cat $OUT/det.txt
if [ "${C4:-0}" -ge 1 ]; then
  for r in $(seq 1 ${C4}); do for so in "" ${LIBS}; do
    FRHIP_LIB=${so:+$PWD/$so} timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err \
      || { echo "c4 failed ($so)"; tail -5 $OUT/c4.err; exit 3; }
    python3 -c "import json;d=json.load(open('$OUT/c4.json'));print('c4 ${so:-package}', d['value'], d['ms_per_step'])" | tee -a $OUT/det.txt
  done; done
fi
