#!/bin/bash
# PMC passes over one conv layer shape (tools/conv_sweep.py --filter), to see where a
# kernel's cycles go.  usage: FILTER="conv2 256->256 @14 s1" TILES=3 TAG=x bash tools/gpu_pmc_layer.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-layer}
mkdir -p $OUT
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
P3="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/conv_sweep.py --filter "$FILTER" --tiles "${TILES:-1}" --reps 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 3; }
  echo "pass $i ok"
done
