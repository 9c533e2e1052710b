"""Summarise the last batch-1 IR-101 forward of a rocprofv3 kernel trace of tools/batch1_trace.py:
per kernel name, time and launches from the last stem launch to the last head reduce.
    python tools/batch1_summary.py gpurun_out/b1
"""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
stems = [i for i, r in enumerate(rows) if "stem_kernel" in r["Kernel_Name"]]
heads = [i for i, r in enumerate(rows) if "head_reduce" in r["Kernel_Name"]]
a = stems[-1]
b = [h for h in heads if h > a][0]
agg = collections.defaultdict(lambda: [0.0, 0])
for r in rows[a:b + 1]:
    k = r["Kernel_Name"][:100]
    agg[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    agg[k][1] += 1
wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) * 1e-3
print("One batch-1 IR-101 forward (last one of tools/batch1_trace.py under rocprofv3 --kernel-trace)")
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{t:9.1f} us {n:4d} launches  {k}")
print(f"kernel sum {sum(v[0] for v in agg.values()):.1f} us, stem start -> head end {wall:.1f} us")
# gaps: start of a kernel minus the end of the one before it, by the later kernel's name
gap = collections.defaultdict(lambda: [0.0, 0])
for p, r in zip(rows[a:b], rows[a + 1:b + 1]):
    g = (int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) * 1e-3
    k = r["Kernel_Name"][:60]
    gap[k][0] += g
    gap[k][1] += 1
print("gaps before each kernel (start - previous end):")
for k, (t, n) in sorted(gap.items(), key=lambda kv: -kv[1][0]):
    print(f"{t:9.1f} us {n:4d} gaps ({t / n:5.2f} avg)  {k}")
# per wino4 shape: split launch duration by grid size (a proxy for the layer)
byg = collections.defaultdict(list)
for r in rows[a:b + 1]:
    if "wino4_kernel" in r["Kernel_Name"]:
        byg[(r["Kernel_Name"][30:60], int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for (k, g), v in sorted(byg.items()):
    print(f"wino4 grid {g // 512:4d} WGs x{len(v):3d}: {sum(v) / len(v):6.1f} us avg  {k}")
