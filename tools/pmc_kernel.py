#!/usr/bin/env python3
"""Average PMC counters per dispatch of kernels matching a name pattern (rocprofv3 csv dirs)."""
import collections
import csv
import glob
import os
import sys


def main():
    pat = sys.argv[1]
    dirs = sys.argv[2:]
    agg = collections.defaultdict(list)
    for d in dirs:
        f = glob.glob(os.path.join(d, "*counter_collection.csv"))
        if not f:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f[0])):
            if pat not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"][:50]
        for k, cs in per.items():
            for c, v in cs.items():
                agg[c].append(v)
    for c, v in sorted(agg.items()):
        print(f"{c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
    for d in dirs:
        t = glob.glob(os.path.join(d, "*kernel_trace.csv"))
        if t and "trace" in d:
            ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(t[0]))
                  if pat in r["Kernel_Name"]]
            if ds:
                print(f"{d}: {len(ds)} dispatches, avg {sum(ds) / len(ds) / 1e3:.1f} us, min {min(ds) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
