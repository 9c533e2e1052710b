#!/usr/bin/env python3
"""Summarise a w4g A/B log (tools/gpu_r04_ab.sh): per shape, median us of each variant and the change."""
import collections
import re
import statistics
import sys

rows = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for line in open(sys.argv[1]):
    m = re.match(r"(\S+): B=(\d+) H=(\d+) (\d+)->(\d+) epi=(\d+).*?: ([\d.]+) us", line)
    if not m:
        continue
    v, shape = m.group(1), f"H={m.group(3)} {m.group(4)}->{m.group(5)} epi={m.group(6)}"
    if shape not in order:
        order.append(shape)
    rows[shape][v].append(float(m.group(7)))
vs = []
for sh in order:
    for v in rows[sh]:
        if v not in vs:
            vs.append(v)
print(f"{'shape':28s} " + " ".join(f"{v:>18s}" for v in vs) + "   (change vs the first)")
for sh in order:
    med = [statistics.median(rows[sh][v]) for v in vs]
    print(f"{sh:28s} " + " ".join(f"{x:9.1f} {100 * (x / med[0] - 1):+6.1f}%  " for x in med))
