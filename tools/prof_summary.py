#!/usr/bin/env python3
"""Per-layer view of a rocprofv3 kernel trace of bench.py (+ optional PMC passes).

Aligns each B-image forward (stem_kernel dispatch -> conv dispatches ->
head_reduce) with the IR layer list, then prints per-layer-class average
duration, achieved TFLOP/s, and (with PMC csvs) HBM bytes per launch.

usage: prof_summary.py TRACE_DIR [--arch ir_101] [--batch 256] [--pmc DIR ...] [--json OUT]
                       [--build "fr_version() string"]

Also prints every kernel of the PMC passes by name (dispatches, average duration, HBM bytes,
MFMA busy), whether or not it aligns with a forward -- e.g. the serving kernel of a batch-1 run,
whose split-K layers do not align one dispatch per layer.  --build stamps the JSON with the
library build the profile was taken on (fr_version(): "... build <id>"); bench.py attaches the
PMC figures only to a run of the same build.
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


def layers(arch, B, fused=True):
    """(name, algorithmic FLOP, algorithmic HBM bytes) per launch of one B-image forward.
    fused: the stride-2 conv2 of a block with a conv shortcut runs that shortcut as extra K-steps
    (one launch, frt_set_fuse_shortcut default)."""
    f4 = 4.0
    out = [("stem", 2.0 * B * 112 * 112 * 64 * 27, B * 112 * 112 * 3 + f4 * B * 112 * 112 * 64)]
    hw = 112
    for i, (cin, d, s) in enumerate(block_specs(arch)):
        st = {64: 1, 128: 2, 256: 3, 512: 4}[d]
        x_b = f4 * B * hw * hw * cin
        out.append((f"s{st}.conv1.{cin}->{d}@{hw}", 2.0 * B * hw * hw * d * 9 * cin,
                    x_b + f4 * d * 9 * cin + f4 * B * hw * hw * d))
        ho = hw // s
        y_b = f4 * B * ho * ho * d
        sc = (2.0 * B * ho * ho * d * cin, x_b / (s * s) + f4 * d * cin) if cin != d else None
        if sc and not fused:
            out.append((f"s{st}.shortcut1x1.{cin}->{d}@{ho}", sc[0], sc[1] + y_b))
        if sc and fused:  # conv2 + shortcut: reads r, x at stride 2, both weights; writes y
            out.append((f"s{st}.conv2+sc.{d}+{cin}->{d}@{ho}/s2", 2.0 * B * ho * ho * d * 9 * d + sc[0],
                        f4 * B * hw * hw * d + f4 * d * 9 * d + sc[1] + y_b))
        else:  # conv2 reads r (B*hw*hw*d), weights, the residual (y-sized) and writes y
            out.append((f"s{st}.conv2.{d}->{d}@{ho}{'/s2' if s == 2 else ''}", 2.0 * B * ho * ho * d * 9 * d,
                        f4 * B * hw * hw * d + f4 * d * 9 * d + 2 * y_b))
        hw = ho
    out.append(("head.fc7x7", 2.0 * B * 512 * 25088, f4 * B * 25088 + f4 * 512 * 25088 + f4 * 32 * B * 512))
    out.append(("head_reduce", 0.0, f4 * 32 * B * 512 + f4 * B * 512))
    return out


def wino4_tiles(h, B):
    """4x4 canvas tiles of an h x h layer at batch B (mirrors wino4_canvas in conv_winograd4.hip)."""
    P = h if h % 4 == 0 else h + 1
    NC = 1 if P % 4 == 0 else min(4 if P % 2 else 2, B)
    crow = (B + NC - 1) // NC
    return ((NC * P + 3) // 4) * ((crow * P + 3) // 4)


def align(rows, L, B):
    """[(layer name, row)] for every B-image forward found in a sorted kernel-trace."""
    # the stem's grid is B x (112 / rows per workgroup) x 256 threads (1, 4 or 16 rows by round)
    found = []
    i = 0
    while i < len(rows):
        r = rows[i]
        if "stem_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) % (B * 256) == 0 and i + len(L) <= len(rows):
            seq = rows[i:i + len(L)]
            if "head_reduce" in seq[-1]["Kernel_Name"]:
                found.append([(n[0], d) for n, d in zip(L, seq)])
                i += len(L)
                continue
        i += 1
    return found


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def kernel_short(n):
    """'void frhip::(anonymous namespace)::wino4_kernel<true, 1, 0, false>(frhip::Wino4Params)' ->
    'wino4_kernel<true, 1, 0, false>'"""
    return n.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "").split("::")[-1][:48]


def by_kernel(trace_dir, pmc_dirs):
    """Per kernel name (template arguments dropped): dispatches and average duration in the trace,
    HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, x 1 KiB) and MFMA busy per dispatch in the PMC passes."""
    short = kernel_short
    dur = collections.defaultdict(list)
    for r in read_csv(glob.glob(os.path.join(trace_dir, "*kernel_trace.csv"))[0]):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in pmc_dirs:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for c in read_csv(glob.glob(os.path.join(d, "*counter_collection.csv"))[0]):
            k = int(c["Dispatch_Id"])
            per[k][c["Counter_Name"]] += float(c["Counter_Value"])
            names[k] = short(c["Kernel_Name"])
        for k, cs in per.items():
            for cn, v in cs.items():
                cnt[names[k]][cn].append(v)
    out = {}
    print(f"{'kernel':48s} {'disp':>6s} {'avg us':>8s} {'HBM MB':>8s} {'MFMAbusy':>8s}")
    for name, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        row = {"dispatches": len(ds), "avg_us": sum(ds) / len(ds) / 1e3}
        c = cnt.get(name, {})
        if c.get("FETCH_SIZE") and c.get("WRITE_SIZE"):
            row["hbm_bytes"] = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) + 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
            busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
            clk = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"]) / 8.0
            row["mfma_busy_frac"] = busy / (1024.0 * clk) if clk else 0.0
        out[name] = row
        print(f"{name:48s} {len(ds):6d} {row['avg_us']:8.1f} "
              + (f"{row['hbm_bytes'] / 1e6:8.1f} " if "hbm_bytes" in row else f"{'-':>8s} ")
              + (f"{100 * row['mfma_busy_frac']:7.1f}%" if "mfma_busy_frac" in row else f"{'-':>8s}"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--arch", default="ir_101")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--json", default=None)
    ap.add_argument("--unfused-shortcut", action="store_true", help="traces taken with frt_set_fuse_shortcut(h, 0)")
    ap.add_argument("--build", default=None, help="fr_version() of the library the profile was taken on")
    a = ap.parse_args()
    rows = read_csv(glob.glob(os.path.join(a.trace_dir, "*kernel_trace.csv"))[0])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    L = layers(a.arch, a.batch, fused=not a.unfused_shortcut)
    fwds = align(rows, L, a.batch)
    per = collections.defaultdict(list)
    kname = {}
    for fw in fwds:
        for name, d in fw:
            per[name].append(int(d["End_Timestamp"]) - int(d["Start_Timestamp"]))
            kname.setdefault(name, d["Kernel_Name"])
    # PMC: counters per dispatch of the aligned forwards in each PMC pass
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))  # counter -> layer -> [values]
    for d in a.pmc:
        prow = read_csv(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])
        prow.sort(key=lambda r: int(r["Start_Timestamp"]))
        vals = collections.defaultdict(dict)
        for c in read_csv(glob.glob(os.path.join(d, "*counter_collection.csv"))[0]):
            k = int(c["Dispatch_Id"])
            vals[k][c["Counter_Name"]] = vals[k].get(c["Counter_Name"], 0.0) + float(c["Counter_Value"])
        for fw in align(prow, L, a.batch):
            for name, r in fw:
                for cn, v in vals.get(int(r["Dispatch_Id"]), {}).items():
                    pmc[cn][name].append(v)
    print(f"forwards aligned: {len(fwds)}")
    hdr = f"{'layer':38s} {'kernel':18s} {'n/fwd':>5s} {'avg us':>9s} {'TF/s':>7s} {'%peak':>6s} {'%time':>6s} {'alg MB':>8s}"
    if pmc:
        hdr += f" {'HBM MB':>8s} {'HBM/alg':>7s}"
    mf = "SQ_VALU_MFMA_BUSY_CYCLES" in pmc and "GRBM_GUI_ACTIVE" in pmc
    if mf:
        hdr += f" {'MHz':>6s} {'cyc/MFMA':>8s} {'MFMAbusy':>8s} {'fracTF':>6s}"
    print(hdr)
    counts = collections.Counter(n for n, _f, _b in L)
    total_time = sum(counts[n] * sum(v) / len(v) for n, v in per.items()) if per else 1.0
    summary, seen = [], set()
    tot_ns = tot_flop = conv_ns = conv_flop = 0.0
    conv_alg = conv_hbm = conv_n = 0.0
    fam = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel family -> totals per forward
    for name, flop, alg in L:
        if name in seen or not per[name]:
            continue
        seen.add(name)
        v = per[name]
        cnt = counts[name]
        avg_ns = sum(v) / len(v)
        tf = flop / (avg_ns * 1e-9) / 1e12 if avg_ns else 0.0
        share = avg_ns * cnt / total_time
        tot_ns += avg_ns * cnt
        tot_flop += flop * cnt
        row = {"layer": name, "per_fwd": cnt, "avg_us": avg_ns / 1e3, "tflops": tf, "alg_bytes": alg}
        kshort = kernel_short(kname.get(name, "")).split("<")[0][:18]
        line = (f"{name:38s} {kshort:18s} {cnt:5d} {avg_ns / 1e3:9.1f} {tf:7.1f} {100 * tf / PEAK:6.1f} {100 * share:6.1f}"
                f" {alg / 1e6:8.1f}")
        is_conv = "conv" in name or "shortcut" in name or "head.fc" in name
        kn = kname.get(name, "")
        family = "winograd" if "wino" in kn else ("direct" if is_conv else "other")
        exec_flop = flop
        if family == "winograd":
            hw = int(name.split("@")[1].split("/")[0])
            if "wino4" in kn:  # 36 products per 4x4 canvas tile (launch_wino4's canvas) instead of 144
                exec_flop = flop * 36.0 / 144.0 * wino4_tiles(hw, a.batch) * 16 / (a.batch * hw * hw)
            else:  # F(2x2): 16 products per (padded) 2x2 tile instead of 36 per 4 pixels
                exec_flop = flop * 16.0 / 36.0 * (2 * ((hw + 1) // 2)) ** 2 / hw ** 2
        row["kernel"] = kn.split("(")[0][:60]
        row["family"] = family
        row["exec_tflops"] = exec_flop / (avg_ns * 1e-9) / 1e12 if avg_ns else 0.0
        fa = fam[family]
        fa["ns"] += avg_ns * cnt
        fa["flop"] += flop * cnt
        fa["exec_flop"] += exec_flop * cnt
        fa["alg_bytes"] += alg * cnt
        fa["launches"] += cnt
        if is_conv:
            conv_ns += avg_ns * cnt
            conv_flop += flop * cnt
        if pmc:
            fe = pmc.get("FETCH_SIZE", {}).get(name, [])
            wr = pmc.get("WRITE_SIZE", {}).get(name, [])
            if fe and wr:
                hbm = 2 * 1024 * sum(fe) / len(fe) + 1024 * sum(wr) / len(wr)
                row["hbm_bytes"] = hbm
                fa["hbm_bytes"] += hbm * cnt
                fa["pmc_launches"] += cnt
                line += f" {hbm / 1e6:8.1f} {hbm / alg:7.2f}"
                if is_conv:
                    conv_alg += alg * cnt
                    conv_hbm += hbm * cnt
                    conv_n += cnt
            # MFMA pipe: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over the chip's 1,024 SIMDs) over
            # the dispatch's cycles per XCD (GRBM_GUI_ACTIVE / 8, rocprofv3 sums the 8 XCDs) x 1,024.
            # cyc/MFMA = busy cycles per f32 MFMA instruction (each 2,048 FLOP) counted from the
            # layer's executed FLOPs: 32 if the counter's unit is what the guide says.  fracTF is
            # the same launch's executed TF/s over the 157.3 TF peak (2.4 GHz), i.e. the bench's frac.
            mb = pmc.get("SQ_VALU_MFMA_BUSY_CYCLES", {}).get(name, [])
            ga = pmc.get("GRBM_GUI_ACTIVE", {}).get(name, [])
            if mf and mb and ga and is_conv:
                busy = sum(mb) / len(mb)
                clk = sum(ga) / len(ga) / 8.0
                n_mfma = exec_flop / 2048.0
                row["mfma_busy_cycles"] = busy
                row["gui_active_cycles_per_xcd"] = clk
                row["mhz"] = clk / (sum(v) / len(v) * 1e-9) / 1e6 if v else 0.0
                row["cycles_per_mfma"] = busy / n_mfma if n_mfma else 0.0
                row["mfma_busy_frac"] = busy / (1024.0 * clk) if clk else 0.0
                fa["mfma_busy"] += busy * cnt
                fa["mfma_clk"] += clk * cnt
                line += (f" {row['mhz']:6.0f} {row['cycles_per_mfma']:8.1f} {100 * row['mfma_busy_frac']:7.1f}%"
                         f" {100 * row['exec_tflops'] / PEAK:5.1f}%")
        summary.append(row)
        print(line)
    print(f"forward: {tot_ns / 1e6:.3f} ms, {tot_flop / 1e12:.3f} TFLOP -> {tot_flop / tot_ns / 1e3:.1f} TF/s; "
          f"conv family {conv_flop / conv_ns / 1e3:.1f} TF/s = {100 * conv_flop / conv_ns / 1e3 / PEAK:.1f}% of peak")
    res = {"forwards": len(fwds), "forward_ms": tot_ns / 1e6, "conv_tflops": conv_flop / conv_ns / 1e3,
           "conv_launches_per_forward": sum(counts[n] for n in counts if "conv" in n or "shortcut" in n or "head.fc" in n),
           "layers": summary}
    if conv_n:
        res["hbm_bytes_per_conv_launch"] = conv_hbm / conv_n
        res["alg_bytes_per_conv_launch"] = conv_alg / conv_n
        print(f"PMC conv family per launch: HBM {conv_hbm / conv_n / 1e6:.1f} MB (FETCH x2 + WRITE) vs algorithmic "
              f"{conv_alg / conv_n / 1e6:.1f} MB -> {conv_hbm / conv_alg:.2f}x")
    kernels = {}
    for family, fa in fam.items():
        k = {"launches_per_forward": int(fa["launches"]), "ms_per_forward": fa["ns"] / 1e6,
             "avg_launch_ms": fa["ns"] / 1e6 / fa["launches"], "alg_flop_per_launch": fa["flop"] / fa["launches"],
             "exec_flop_per_launch": fa["exec_flop"] / fa["launches"],
             "alg_tflops": fa["flop"] / fa["ns"] / 1e3 if fa["ns"] else 0.0,
             "exec_tflops": fa["exec_flop"] / fa["ns"] / 1e3 if fa["ns"] else 0.0,
             "alg_bytes_per_launch": fa["alg_bytes"] / fa["launches"]}
        if fa["pmc_launches"]:
            k["hbm_bytes_per_launch"] = fa["hbm_bytes"] / fa["pmc_launches"]
        if fa["mfma_clk"]:
            k["mfma_busy_frac"] = fa["mfma_busy"] / (1024.0 * fa["mfma_clk"])
            k["exec_frac_of_peak"] = k["exec_tflops"] / PEAK
            print(f"{family:9s}: MFMA busy {100 * k['mfma_busy_frac']:.1f}% of the SIMD cycles (PMC) vs executed "
                  f"{100 * k['exec_frac_of_peak']:.1f}% of the 2.4-GHz peak (FLOP / time)")
        kernels[family] = k
        print(f"{family:9s}: {k['launches_per_forward']:3d} launches/fwd, {k['ms_per_forward']:.3f} ms/fwd, "
              f"avg {k['avg_launch_ms']:.4f} ms, alg {k['alg_tflops']:.1f} TF/s, executed {k['exec_tflops']:.1f} TF/s"
              + (f", HBM {k['hbm_bytes_per_launch'] / 1e6:.1f} MB/launch vs alg {k['alg_bytes_per_launch'] / 1e6:.1f}"
                 if "hbm_bytes_per_launch" in k else ""))
    res["kernels"] = kernels
    res["by_kernel"] = by_kernel(a.trace_dir, a.pmc)
    if a.build:
        res["build"] = a.build
        res["build_id"] = a.build.rsplit("build ", 1)[-1].strip() if "build " in a.build else None
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
