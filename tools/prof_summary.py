#!/usr/bin/env python3
"""Per-layer view of a rocprofv3 kernel trace of bench.py (+ optional PMC passes).

Aligns each B-image forward (stem_kernel dispatch -> conv dispatches ->
head_reduce) with the IR layer list, then prints per-layer-class average
duration, achieved TFLOP/s, and (with PMC csvs) HBM bytes per launch.

usage: prof_summary.py TRACE_DIR [--arch ir_101] [--batch 256] [--pmc DIR ...] [--json OUT]
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from facerecognitionpipeline_amd.arch import block_specs  # noqa: E402

PEAK = 157.3


def layers(arch, B):
    out = [("stem", 2.0 * B * 112 * 112 * 64 * 27)]
    hw = 112
    for i, (cin, d, s) in enumerate(block_specs(arch)):
        st = {64: 1, 128: 2, 256: 3, 512: 4}[d]
        out.append((f"s{st}.conv1.{cin}->{d}@{hw}", 2.0 * B * hw * hw * d * 9 * cin))
        ho = hw // s
        if cin != d:
            out.append((f"s{st}.shortcut1x1.{cin}->{d}@{ho}", 2.0 * B * ho * ho * d * cin))
        out.append((f"s{st}.conv2.{d}->{d}@{ho}{'/s2' if s == 2 else ''}", 2.0 * B * ho * ho * d * 9 * d))
        hw = ho
    out.append(("head.fc7x7", 2.0 * B * 512 * 25088))
    out.append(("head_reduce", 0.0))
    return out


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--arch", default="ir_101")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = read_csv(glob.glob(os.path.join(a.trace_dir, "*kernel_trace.csv"))[0])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    L = layers(a.arch, a.batch)
    stem_grid = a.batch * 112 * 256
    per = collections.defaultdict(list)
    fwd = 0
    i = 0
    while i < len(rows):
        r = rows[i]
        if "stem_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == stem_grid and i + len(L) <= len(rows):
            seq = rows[i:i + len(L)]
            if "head_reduce" in seq[-1]["Kernel_Name"]:
                for (name, flop), d in zip(L, seq):
                    ns = int(d["End_Timestamp"]) - int(d["Start_Timestamp"])
                    per[name].append((ns, flop, d["Kernel_Name"], int(d.get("Dispatch_Id", 0))))
                fwd += 1
                i += len(L)
                continue
        i += 1
    # PMC bytes keyed by dispatch id
    pmc = {}
    for d in a.pmc:
        for c in read_csv(glob.glob(os.path.join(d, "*counter_collection.csv"))[0]):
            pmc.setdefault(c["Counter_Name"], {})
            pmc[c["Counter_Name"]].setdefault((c["Kernel_Name"], int(c["Grid_Size"])), []).append(
                float(c["Counter_Value"]))
    # group layer names into classes (strip block index by shape)
    cls = collections.OrderedDict()
    for name, _f in L:
        cls.setdefault(name, [])
    tot_ns = tot_flop = conv_ns = conv_flop = 0.0
    print(f"forwards aligned: {fwd}")
    print(f"{'layer class':38s} {'n/fwd':>5s} {'avg us':>9s} {'TF/s':>7s} {'%peak':>6s} {'%time':>6s}")
    agg = collections.OrderedDict()
    for name, flop in L:
        v = per[name]
        if not v:
            continue
        key = name
        agg.setdefault(key, [0, 0.0, 0.0])
        agg[key][0] += 1
    total_time = sum(sum(x[0] for x in per[n]) for n in per) / max(fwd, 1)
    summary = []
    for name in agg:
        v = per[name]
        cnt = agg[name][0]
        avg_ns = sum(x[0] for x in v) / len(v)
        flop = v[0][1]
        tf = flop / (avg_ns * 1e-9) / 1e12 if avg_ns else 0.0
        share = avg_ns * cnt / total_time
        tot_ns += avg_ns * cnt
        tot_flop += flop * cnt
        if "conv" in name or "shortcut" in name or "head.fc" in name:
            conv_ns += avg_ns * cnt
            conv_flop += flop * cnt
        summary.append({"layer": name, "per_fwd": cnt, "avg_us": avg_ns / 1e3, "tflops": tf, "kernel": v[0][2]})
        print(f"{name:38s} {cnt:5d} {avg_ns / 1e3:9.1f} {tf:7.1f} {100 * tf / PEAK:6.1f} {100 * share:6.1f}")
    print(f"forward: {tot_ns / 1e6:.3f} ms, {tot_flop / 1e12:.3f} TFLOP -> {tot_flop / tot_ns / 1e3:.1f} TF/s; "
          f"conv family {conv_flop / conv_ns / 1e3:.1f} TF/s = {100 * conv_flop / conv_ns / 1e3 / PEAK:.1f}% of peak")
    res = {"forwards": fwd, "forward_ms": tot_ns / 1e6, "conv_tflops": conv_flop / conv_ns / 1e3, "layers": summary}
    if pmc:
        # per-launch HBM bytes of the conv family: FETCH_SIZE (KB, x2 on gfx950 wide streams) + WRITE_SIZE (KB)
        f_tot = w_tot = n_l = 0.0
        for (kname, grid), vals in pmc.get("FETCH_SIZE", {}).items():
            if "conv_mfma" in kname:
                f_tot += sum(vals)
                n_l += len(vals)
        for (kname, grid), vals in pmc.get("WRITE_SIZE", {}).items():
            if "conv_mfma" in kname:
                w_tot += sum(vals)
        if n_l:
            fetch_b = 2 * f_tot * 1024 / n_l
            write_b = w_tot * 1024 / n_l
            res["hbm_bytes_per_conv_launch"] = fetch_b + write_b
            res["fetch_bytes_per_conv_launch_x2"] = fetch_b
            res["write_bytes_per_conv_launch"] = write_b
            print(f"PMC conv family: {n_l:.0f} launches, FETCH x2 {fetch_b / 1e6:.1f} MB + WRITE {write_b / 1e6:.1f} MB "
                  f"per launch")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
