#!/usr/bin/env python3
"""Concurrency of the two lanes in a rocprofv3 kernel trace of bench.py (two-lane pass): the
share of the GPU-busy time in which two kernels run at once, and how many launches start while
another is still running.  usage: lane_overlap.py TRACE_DIR"""
import csv
import glob
import os
import sys

rows = list(csv.DictReader(open(glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the two-lane forwards: from the first half-batch stem (128 crops: 128 * 28 blocks of 256) to the
# last head reduce before the one-lane profiled pass's first full-batch stem
lane_stem = [i for i, r in enumerate(rows) if "stem_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 128 * 28 * 256]
full_stem = [i for i, r in enumerate(rows) if "stem_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 256 * 28 * 256]
lo = lane_stem[0]
hi = min([i for i in full_stem if i > lo] or [len(rows)])
rows = rows[lo:hi]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# busy time with >= 1 and >= 2 kernels in flight (sweep over start/end events)
ev = sorted([(s, 1) for s, _e, _n in iv] + [(e, -1) for _s, e, _n in iv])
busy = both = 0
depth, last = 0, ev[0][0]
for t, d in ev:
    if depth >= 1:
        busy += t - last
    if depth >= 2:
        both += t - last
    depth += d
    last = t
starts_in_flight = sum(1 for i in range(1, len(iv)) if iv[i][0] < max(e for _s, e, _n in iv[max(0, i - 8):i]))
print(f"kernels {len(iv)}; GPU busy {busy / 1e6:.1f} ms; two or more kernels in flight {100 * both / busy:.1f}% "
      f"of it; launches starting while another runs {starts_in_flight} ({100 * starts_in_flight / len(iv):.0f}%)")
