#!/usr/bin/env python3
"""Summarise tools/gpu_w4_ab.sh output: per shape, each variant's best time and its change vs base."""
import collections
import re
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    m = re.match(r"(\S+) \| B=(\d+) H=(\d+) (\d+)->(\d+) epi=(\d)[^:]*: ([\d.]+) us", line)
    if m:
        d[f"B{m[2]} {m[4]}->{m[5]}@{m[3]} epi{m[6]}"][m[1]].append(float(m[7]))
for shape, v in d.items():
    base = min(v["base"]) if "base" in v else None
    cells = [f"{n} {min(t):.1f}" + (f" ({(min(t) / base - 1) * 100:+.1f}%)" if base else "") for n, t in v.items()]
    print(f"{shape:26s} " + " | ".join(cells))
