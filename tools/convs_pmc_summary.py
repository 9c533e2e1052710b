"""Per-launch PMC medians of the serving conv kernel by grid size, from rocprofv3 --pmc passes over
tools/batch1_trace.py (tools/gpu_convs_pmc.sh).  usage: python tools/convs_pmc_summary.py DIR..."""
import csv
import glob
import sys
from collections import defaultdict

import numpy as np

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "convs_kernel" not in name:
                continue
            grid = int(r["Grid_Size"]) // 256 if "Grid_Size" in r else int(r.get("Grid_Size_X", 0)) // 256
            key = (name.split("convs_kernel")[1][:12], grid)
            vals[key][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
for key in sorted(vals, key=lambda k: -k[1]):
    per = defaultdict(list)
    for (cn, _), v in vals[key].items():
        per[cn].append(sum(v))
    line = "  ".join(f"{cn} {np.median(v):.4g}" for cn, v in sorted(per.items()))
    print(f"{key[0]} grid {key[1]:4d}: {line}")
