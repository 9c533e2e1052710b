#!/bin/bash
# Memory-path PMC passes over one F(4x4) launch shape (tools/wv/w4g_<V>), one pass per run.
# usage: V=base SHAPE="256 14 256 256 2" bash tools/gpu_w4g_pmc2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${V:-base}; SHAPE=${SHAPE:-"256 14 256 256 2"}
OUT=gpurun_out/w4g_pmc2/$V; mkdir -p $OUT
i=0
for P in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
         "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
         "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
         "TD_TD_BUSY_sum TD_TC_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    tools/wv/w4g_$V $SHAPE 3 0 1 1 > $OUT/p$i.log 2>&1 || { echo "pmc $V p$i failed"; tail -3 $OUT/p$i.log; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
vals = collections.defaultdict(list); dur = []
for f in sorted(glob.glob(d + "/p*/*counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "wino4_kernel" not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for (di, c), v in per.items():
        vals[c].append(v)
print(d, "median dispatch us", sorted(dur)[len(dur) // 2] if dur else None)
for c, v in sorted(vals.items()):
    v = sorted(v)
    print(f"  {c:40s} {v[len(v) // 2]:.4g}")
PY
