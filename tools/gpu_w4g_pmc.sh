#!/bin/bash
# PMC passes over the F(4x4) GEMM kernel of tools/w4g_bench variants (one pass per run).
# usage: VARIANTS="base noepi" SHAPE="256 56 64 64 2" bash tools/gpu_w4g_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/w4g_pmc
mkdir -p $OUT
SHAPE=${SHAPE:-"256 56 64 64 2"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
for V in ${VARIANTS:-base noepi}; do
  i=0; mkdir -p $OUT/$V
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$V/p$i -o run -- \
      tools/wv/w4g_$V $SHAPE 3 > $OUT/$V/p$i.log 2>&1 || { echo "pmc $V p$i failed"; exit 3; }
  done
  python3 - "$OUT/$V" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(d + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "wino4_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(d.split("/")[-1], {k: round(v / max(1, n[k] / (1 if k.startswith("GRBM") or k.startswith("TCC") else 1)), 0) for k, v in sorted(tot.items())})
PY
done
