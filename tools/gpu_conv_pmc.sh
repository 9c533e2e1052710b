#!/bin/bash
# PMC passes over one direct-conv shape of tools/conv_sweep.py (one pass per counter group).
# usage: FILTER="conv2 64->64 @112" TILE=8 bash tools/gpu_conv_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/conv_pmc
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/conv_sweep.py --filter "${FILTER}" --tiles ${TILE} --reps 3 > $OUT/p$i.log 2>&1 || { echo "pmc p$i failed"; tail -5 $OUT/p$i.log; exit 3; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(d + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "conv_mfma_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print({k: round(v / max(1, n[k]), 0) for k, v in sorted(tot.items())})
PY
