#!/bin/bash
# conv_small.hip variants: GPU time per launch from a rocprofv3 kernel trace of tools/convs_bench.py
# (the script's own event timing is host-bound at ~12 us per call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-cs_base}; do
  O=gpurun_out/cprof_$v
  rm -rf $O
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/convs_bench.py --so tools/wv/lib_$v.so --iters 50 > $O.log 2>&1 || { echo "$v failed"; exit 3; }
  echo "== $v"
  python3 - $O <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if "convs_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the bench runs 7 shapes x (5 warm + 50 timed) launches, in order
names = ["s3.conv2", "s3.conv1", "s2.conv2", "s1.conv1@56", "s4.conv2", "s1.conv1@112", "s3.conv2+sc/s2"]
per = 55
for k, n in enumerate(names):
    seg = rows[k * per + 5:(k + 1) * per]
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in seg)
    if d:
        print(f"{n:16s} median {d[len(d) // 2]:7.2f} us  min {d[0]:7.2f}  (grid {seg[0].get('Grid_Size_X', '?')})")
PY
done
