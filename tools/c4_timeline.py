#!/usr/bin/env python3
"""Where a C4 step's wall time goes, from a rocprofv3 kernel trace of ``bench.py --config c4``.

Steps are cut at the end of each step's match (``topk*`` kernel: one per embed + match).  Per
step: wall time between consecutive cuts, GPU-busy time (union of all kernel intervals), idle
time (gaps between kernels, the largest ones listed with the kernels on either side), the kernel
time of the detector stream (the stream ``letterbox_kernel`` runs on) and of the embedding
streams, and the time both ran at once.

usage: c4_timeline.py TRACE_DIR [--skip N] [--gaps 5]
"""
import argparse
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.prof_summary import read_csv, kernel_short  # noqa: E402


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(u):
    return sum(b - a for a, b in u)


def intersect(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--skip", type=int, default=3, help="steps to skip at the start (warmup)")
    ap.add_argument("--gaps", type=int, default=5)
    a = ap.parse_args()
    rows = read_csv(glob.glob(os.path.join(a.trace_dir, "*kernel_trace.csv"))[0])
    rows = [r for r in rows if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    det_streams = {(r["Queue_Id"], r["Stream_Id"]) for r in rows if "letterbox_kernel" in r["Kernel_Name"]}
    cuts = [int(r["End_Timestamp"]) for r in rows if "topk" in r["Kernel_Name"]]
    if len(cuts) < a.skip + 2:
        sys.exit(f"only {len(cuts)} steps in the trace")
    stats = []
    for s in range(a.skip, len(cuts) - 1):
        t0, t1 = cuts[s], cuts[s + 1]
        ks = [r for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
        iv = [(max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1)) for r in ks]
        det = [x for x, r in zip(iv, ks) if (r["Queue_Id"], r["Stream_Id"]) in det_streams]
        emb = [x for x, r in zip(iv, ks) if (r["Queue_Id"], r["Stream_Id"]) not in det_streams]
        ub, ud, ue = union(iv), union(det), union(emb)
        gaps = []
        prev_end, prev_name = t0, "(step start)"
        for x, r in sorted(zip(iv, ks), key=lambda z: z[0][0]):
            if x[0] > prev_end:
                gaps.append((x[0] - prev_end, prev_name, kernel_short(r["Kernel_Name"])))
            if x[1] > prev_end:
                prev_end, prev_name = x[1], kernel_short(r["Kernel_Name"])
        stats.append({"wall": t1 - t0, "busy": length(ub), "det": length(ud), "emb": length(ue),
                      "both": intersect(ud, ue), "det_sum": sum(b - x for x, b in det),
                      "emb_sum": sum(b - x for x, b in emb), "gaps": sorted(gaps, reverse=True)})
    def med(k):
        return statistics.median(x[k] for x in stats) / 1e6
    print(f"steps analysed: {len(stats)} (of {len(cuts) - 1}; first {a.skip} skipped)")
    print(f"median per step (ms): wall {med('wall'):.3f}, GPU busy {med('busy'):.3f}, idle "
          f"{med('wall') - med('busy'):.3f}; detector stream busy {med('det'):.3f} (kernel sum {med('det_sum'):.3f}), "
          f"embedding streams busy {med('emb'):.3f} (kernel sum {med('emb_sum'):.3f}), both at once {med('both'):.3f}")
    mid = sorted(stats, key=lambda x: x["wall"])[len(stats) // 2]
    print(f"largest idle gaps of the median step (us): " + "; ".join(
        f"{g / 1e3:.1f} after {p} before {n}" for g, p, n in mid["gaps"][:a.gaps]))
    idle_hist = {}
    for g, p, n in mid["gaps"]:
        key = f"{p} -> {n}"
        idle_hist[key] = idle_hist.get(key, 0) + g
    print("idle by transition (median step, us): " + "; ".join(
        f"{k}: {v / 1e3:.1f}" for k, v in sorted(idle_hist.items(), key=lambda kv: -kv[1])[:8]))


if __name__ == "__main__":
    main()
