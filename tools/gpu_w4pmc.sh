#!/bin/bash
# PMC passes over one Winograd layer (tools/w4_layer.py); each pass is its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/w4pmc${TAG:-}
mkdir -p $OUT
LARGS=${LAYER_ARGS:-"--m 4 --B 256 --H 14 --cin 256 --cout 256 --epi 2 --iters 5"}
timeout -k 10 120 python3 tools/w4_layer.py $LARGS || exit 3
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/w4_layer.py $LARGS > $OUT/trace.log 2>&1 || { echo trace failed; exit 3; }
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 tools/w4_layer.py $LARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 3; }
done
echo pmc ok
