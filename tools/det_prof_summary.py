#!/usr/bin/env python3
"""Per-layer view of a rocprofv3 kernel trace of the SCRFD-10G detector (+ optional PMC passes).

The trace is of ``tools/det_time.py`` (fr_detect on B letterboxed 1080p frames, nothing else on
the GPU), so every detect is one run of dispatches from ``letterbox_kernel`` to ``nms_kernel``.
Each run is aligned with the detector's launch order (csrc/detector.cpp forward_chunk +
detector_run): split-K fixups and runtime copies / fills attach to the layer before them.

Per layer: kernel, average duration, algorithmic FLOP (unpadded channels, direct-conv count, the
figure detector_arch.detector_macs sums), executed MFMA FLOP (channels padded to the kernel's
granularity; F(4x4) counts 36 products per 4x4 tile), TF/s of both, algorithmic HBM bytes (the
layer's tensors as laid out: padded NHWC f32 in, weights, out, residual) and, with PMC passes,
HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, KiB units as in prof_summary.py) and MFMA busy.

usage: det_prof_summary.py TRACE_DIR [--frames 32] [--pmc DIR ...] [--json OUT] [--build STR]
"""
import argparse
import collections
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.prof_summary import read_csv, kernel_short  # noqa: E402

PEAK = 157.3  # dense fp32 MFMA TF/s at 2.4 GHz
HBM_PEAK = 8000.0  # GB/s
STAGE_BLOCKS = (3, 4, 2, 3)
STAGE_PLANES = (56, 88, 88, 224)
STEM, NECK, HEAD = 56, 56, 80


def pad32(c):
    return (c + 31) // 32 * 32


def det_layers(B, W=640, H=640, src=(1080, 1920), skip=192, skip2=64):
    """[(name, kind, alg_flop, exec_flop_wino4, exec_flop_direct, alg_bytes)] in launch order.
    kind: 'conv3' (3x3 stride 1: F(4x4) when eligible), 'convd' (direct: strided / 1x1 / 2x2),
    or the elementwise kernel's name.  alg_flop is the reference network's (full 640-row canvas);
    the executed FLOPs and bytes of the stem and stage 1 count the (H - skip)-row canvas they run
    on (detector.cpp row_plan; 192 rows for a 1080p frame; stage 2: skip2 = 64), and 'row_expand'
    (optional: absent when nothing is skipped) restores stage 1's / stage 2's output height."""
    f4 = 4.0
    L = []
    red = [(H - skip) / H]

    def conv(name, ci, co, hw_in, k, s, res=False):
        ho = (hw_in + 2 * (k // 2 if k == 3 else 0) - k) // s + 1
        cip, cop = pad32(ci), pad32(co)
        alg = 2.0 * B * ho * ho * co * ci * k * k
        # F(4x4): 36 products per 4x4 tile (H % 4 == 0 here: no canvas separators), couts in
        # quarters of 16 (an idle quarter of a 64-cout item issues no MFMAs)
        ex_w4 = red[0] * 2.0 * 36 * B * (ho // 4) * (ho // 4) * cip * ((cop + 15) // 16 * 16)
        ex_d = red[0] * 2.0 * B * ho * ho * cop * cip * k * k
        by = red[0] * f4 * (B * hw_in * hw_in * cip + cop * cip * k * k + B * ho * ho * cop * (2 if res else 1))
        L.append((name, "conv3" if (k == 3 and s == 1) else "convd", alg, ex_w4, ex_d, by))
        return ho

    L.append(("letterbox", "letterbox", 0.0, 0.0, 0.0,
              # reads the frame rows the resize touches once (at most the whole frame), writes the canvas
              float(B * src[0] * src[1] * 3 + red[0] * B * W * H * 3)))
    h = H // 2
    L.append(("stem0 3->28 s2 @640 (+blob)", "det_stem", 2.0 * B * h * h * 28 * 27,
              red[0] * 2.0 * B * h * h * 32 * 28, 0.0, red[0] * (float(B * W * H * 3) + f4 * B * h * h * 32)))
    conv("stem1 28->28 @320", 28, 28, h, 3, 1)
    conv("stem2 28->56 @320", 28, 56, h, 3, 1)
    L.append(("maxpool3 s2 @320", "maxpool3", 0.0, 0.0, 0.0, red[0] * f4 * B * (h * h + (h // 2) ** 2) * 64))
    hw = h // 2
    cin = STEM
    for st, (n, c) in enumerate(zip(STAGE_BLOCKS, STAGE_PLANES)):
        if st == 1:
            r2 = (H - skip2) / H
            L.append(("row_expand s1 out @160", "row_expand?", 0.0, 0.0, 0.0,
                      f4 * B * hw * hw * 64 * (r2 + red[0]) if skip else 0.0))
            red[0] = r2
        if st == 2:
            L.append(("row_expand s2 out @80", "row_expand?", 0.0, 0.0, 0.0,
                      f4 * B * hw * hw * 96 * (1 + red[0]) if skip2 else 0.0))
            red[0] = 1.0
        for u in range(n):
            ci = cin if u == 0 else c
            s = 2 if (u == 0 and st > 0) else 1
            ho = conv(f"s{st + 1}.{u}.conv1 {ci}->{c} @{hw}{'/s2' if s == 2 else ''}", ci, c, hw, 3, s)
            if u == 0 and (st > 0 or ci != c):
                if s == 2:  # AvgPool2d(2, 2) then the 1x1 conv
                    L.append((f"s{st + 1}.{u}.avgpool2 @{hw}", "avgpool2", 0.0, 0.0, 0.0,
                              red[0] * f4 * B * (hw * hw + ho * ho) * pad32(ci)))
                conv(f"s{st + 1}.{u}.down 1x1 {ci}->{c} @{ho}", ci, c, ho, 1, 1)
            conv(f"s{st + 1}.{u}.conv2 {c}->{c} @{ho} +res", c, c, ho, 3, 1, res=True)
            hw = ho
        cin = c
    lv = (H // 8, H // 16, H // 32)
    for i, c in enumerate(STAGE_PLANES[1:]):
        conv(f"neck.lateral{i} 1x1 {c}->56 @{lv[i]}", c, NECK, lv[i], 1, 1)
    for i in (2, 1):
        L.append((f"neck.upsample_add {lv[i]}->{lv[i - 1]}", "upsample_add", 0.0, 0.0, 0.0,
                  f4 * B * (lv[i] ** 2 + 2 * lv[i - 1] ** 2) * 64))
    for i in range(3):
        conv(f"neck.fpn{i} 56->56 @{lv[i]}", NECK, NECK, lv[i], 3, 1)
    for i in range(2):
        conv(f"neck.down{i} 56->56 s2 @{lv[i]} +res", NECK, NECK, lv[i], 3, 2, res=True)
    for i in (1, 2):
        conv(f"neck.pafpn{i - 1} 56->56 @{lv[i]}", NECK, NECK, lv[i], 3, 1)
    for i in range(3):
        conv(f"head{i}.tower0 56->80 @{lv[i]}", NECK, HEAD, lv[i], 3, 1)
        conv(f"head{i}.tower1 80->80 @{lv[i]}", HEAD, HEAD, lv[i], 3, 1)
        conv(f"head{i}.tower2 80->80 @{lv[i]}", HEAD, HEAD, lv[i], 3, 1)
        conv(f"head{i}.out 80->30 @{lv[i]}", HEAD, 30, lv[i], 3, 1)
    L.append(("decode", "decode", 0.0, 0.0, 0.0, f4 * B * sum(x * x for x in lv) * 32))
    L.append(("nms", "nms", 0.0, 0.0, 0.0, 0.0))
    return L


CONV_KERNELS = ("wino4_kernel", "wino4w_kernel", "wino4t_kernel", "wino_kernel", "conv_mfma_kernel", "convs_kernel", "s2c64_kernel")


def is_attach(name):
    """Dispatches that belong to the layer launched before them."""
    return "fixup" in name or name.startswith("__amd_rocclr") or "fill" in name.lower() or "copy" in name.lower()


def segments(rows, L):
    """Aligned detects: [[(layer index, [rows])]] from letterbox_kernel to nms_kernel."""
    out, i = [], 0
    while i < len(rows):
        if "letterbox_kernel" not in rows[i]["Kernel_Name"]:
            i += 1
            continue
        seg, li, ok = [], 0, True
        j = i
        while j < len(rows) and li <= len(L):
            kn = rows[j]["Kernel_Name"]
            if is_attach(kn) and seg:
                seg[-1][1].append(rows[j])
                j += 1
                continue
            if li == len(L):
                break
            kind = L[li][1]
            if kind.endswith("?"):  # optional layer: present only when its kernel ran
                if kind[:-1] + "_kernel" in kn:
                    seg.append((li, [rows[j]]))
                    j += 1
                li += 1
                continue
            want = any(c in kn for c in CONV_KERNELS) if kind in ("conv3", "convd") else (kind + "_kernel" in kn
                                                                                          or kind + "_mfma" in kn)
            if not want:
                ok = False
                break
            seg.append((li, [rows[j]]))
            li += 1
            j += 1
            if L[li - 1][1] == "nms":
                break
        if ok and li == len(L):
            out.append(seg)
            i = j
        else:
            i += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--json", default=None)
    ap.add_argument("--build", default=None)
    ap.add_argument("--skip", type=int, default=None,
                    help="canvas rows the stem and stage 1 skipped (default: 192 if row_expand_kernel ran, else 0)")
    a = ap.parse_args()
    rows = read_csv(glob.glob(os.path.join(a.trace_dir, "*kernel_trace.csv"))[0])
    nexp = sum("row_expand" in r["Kernel_Name"] for r in rows) / max(1, sum("letterbox" in r["Kernel_Name"]
                                                                            for r in rows))
    skip = a.skip if a.skip is not None else (192 if nexp >= 1 else 0)
    skip2 = 64 if nexp >= 2 else 0
    L = det_layers(a.frames, skip=skip, skip2=skip2)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs = segments(rows, L)
    if not segs:
        sys.exit("no detect aligned with the detector's launch order")
    dur = collections.defaultdict(list)
    kname = {}
    detect_ns = []
    for seg in segs:
        t0 = int(seg[0][1][0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for _li, rs in seg for r in rs)
        detect_ns.append(t1 - t0)
        for li, rs in seg:
            dur[li].append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs))
            kname.setdefault(li, "+".join(kernel_short(r["Kernel_Name"]) for r in rs))
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))  # counter -> layer -> values
    for d in a.pmc:
        prow = read_csv(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])
        prow.sort(key=lambda r: int(r["Start_Timestamp"]))
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        for c in read_csv(glob.glob(os.path.join(d, "*counter_collection.csv"))[0]):
            vals[int(c["Dispatch_Id"])][c["Counter_Name"]] += float(c["Counter_Value"])
        for seg in segments(prow, L):
            for li, rs in seg:
                acc = collections.defaultdict(float)
                for r in rs:
                    for cn, v in vals.get(int(r["Dispatch_Id"]), {}).items():
                        acc[cn] += v if cn != "GRBM_GUI_ACTIVE" else 0.0
                    # the clock of the layer = its main dispatch's
                ga = vals.get(int(rs[0]["Dispatch_Id"]), {}).get("GRBM_GUI_ACTIVE")
                if ga is not None:
                    acc["GRBM_GUI_ACTIVE"] = ga
                for cn, v in acc.items():
                    pmc[cn][li].append(v)
    print(f"detects aligned: {len(segs)} (B = {a.frames} frames of 1080p, 640x640 letterbox; stem + stage 1 on "
          f"{640 - skip} canvas rows, stage 2 on {640 - skip2})")
    print(f"detect wall (first dispatch start -> nms end), median: "
          f"{sorted(detect_ns)[len(detect_ns) // 2] / 1e6:.3f} ms")
    hdr = (f"{'layer':36s} {'kernel':22s} {'avg us':>8s} {'%time':>6s} {'algGF':>7s} {'algTF':>6s} {'exeTF':>6s}"
           f" {'%pk':>5s} {'alg MB':>7s} {'GB/s':>6s}")
    has_hbm = "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc
    has_mf = "SQ_VALU_MFMA_BUSY_CYCLES" in pmc and "GRBM_GUI_ACTIVE" in pmc
    if has_hbm:
        hdr += f" {'HBM MB':>7s} {'x alg':>5s} {'HBMGB/s':>7s}"
    if has_mf:
        hdr += f" {'MFMAbusy':>8s}"
    print(hdr)
    total = sum(sum(v) / len(v) for v in dur.values())
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    out_layers = []
    for li, (name, kind, alg, ex_w4, ex_d, by) in enumerate(L):
        v = dur.get(li)
        if not v:
            continue
        ns = sum(v) / len(v)
        kn = kname[li]
        base = kn.split("+")[0].split("<")[0]
        ex = ex_w4 if "wino4" in base else (ex_d if kind in ("conv3", "convd") else (ex_w4 if kind == "det_stem" else 0.0))
        row = {"layer": name, "kernel": kn, "avg_us": ns / 1e3, "share": ns / total, "alg_flop": alg,
               "exec_flop": ex, "alg_tflops": alg / ns / 1e3, "exec_tflops": ex / ns / 1e3, "alg_bytes": by,
               "alg_GBps": by / ns}
        line = (f"{name[:36]:36s} {kn[:22]:22s} {ns / 1e3:8.1f} {100 * ns / total:6.1f} {alg / 1e9:7.2f}"
                f" {row['alg_tflops']:6.1f} {row['exec_tflops']:6.1f} {100 * row['exec_tflops'] / PEAK:5.1f}"
                f" {by / 1e6:7.1f} {by / ns:6.0f}")
        # the wide / tall item instances (wino4w_kernel, wino4t_kernel) are the same kernel body: one family
        f = fam["wino4_kernel" if base in ("wino4_kernel", "wino4w_kernel", "wino4t_kernel") else base]
        f["ns"] += ns
        f["alg"] += alg
        f["exec"] += ex
        f["bytes"] += by
        f["n"] += 1
        if has_hbm and pmc["FETCH_SIZE"].get(li) and pmc["WRITE_SIZE"].get(li):
            fe, wr = pmc["FETCH_SIZE"][li], pmc["WRITE_SIZE"][li]
            hbm = 2 * 1024 * sum(fe) / len(fe) + 1024 * sum(wr) / len(wr)
            row["hbm_bytes"] = hbm
            row["hbm_GBps"] = hbm / ns
            f["hbm"] += hbm
            line += f" {hbm / 1e6:7.1f} {hbm / by if by else 0.0:5.2f} {hbm / ns:7.0f}"
        if has_mf and pmc["SQ_VALU_MFMA_BUSY_CYCLES"].get(li) and pmc["GRBM_GUI_ACTIVE"].get(li):
            mb, ga = pmc["SQ_VALU_MFMA_BUSY_CYCLES"][li], pmc["GRBM_GUI_ACTIVE"][li]
            busy, clk = sum(mb) / len(mb), sum(ga) / len(ga) / 8.0
            row["mfma_busy_frac"] = busy / (1024.0 * clk) if clk else 0.0
            f["busy"] += busy
            f["clk"] += clk
            line += f" {100 * row['mfma_busy_frac']:7.1f}%"
        out_layers.append(row)
        print(line)
    print(f"kernel sum per detect: {total / 1e6:.3f} ms; algorithmic {sum(x[2] for x in L) / 1e9:.1f} GFLOP "
          f"-> {sum(x[2] for x in L) / total / 1e3:.1f} TF/s direct-conv equivalent")
    fams = {}
    print(f"{'family':22s} {'launches':>8s} {'ms':>7s} {'%':>5s} {'algTF':>6s} {'exeTF':>6s} {'%pk':>5s} "
          f"{'algGB/s':>7s} {'HBM/alg':>7s} {'MFMAbusy':>8s}")
    for base, f in sorted(fam.items(), key=lambda kv: -kv[1]["ns"]):
        d = {"layers": int(f["n"]), "ms": f["ns"] / 1e6, "share": f["ns"] / total,
             "alg_tflops": f["alg"] / f["ns"] / 1e3, "exec_tflops": f["exec"] / f["ns"] / 1e3,
             "alg_flop": f["alg"], "exec_flop": f["exec"], "alg_bytes": f["bytes"],
             "alg_GBps": f["bytes"] / f["ns"]}
        if f["hbm"]:
            d["hbm_bytes"] = f["hbm"]
            d["hbm_GBps"] = f["hbm"] / f["ns"]
        if f["clk"]:
            d["mfma_busy_frac"] = f["busy"] / (1024.0 * f["clk"])
        fams[base] = d
        print(f"{base:22s} {d['layers']:8d} {d['ms']:7.3f} {100 * d['share']:5.1f} {d['alg_tflops']:6.1f} "
              f"{d['exec_tflops']:6.1f} {100 * d['exec_tflops'] / PEAK:5.1f} {d['alg_GBps']:7.0f} "
              + (f"{d['hbm_bytes'] / d['alg_bytes']:7.2f} " if "hbm_bytes" in d and d["alg_bytes"] else f"{'-':>7s} ")
              + (f"{100 * d['mfma_busy_frac']:7.1f}%" if "mfma_busy_frac" in d else f"{'-':>8s}"))
    res = {"frames": a.frames, "detects": len(segs), "skip_rows": skip, "skip_rows_stage2": skip2,
           "detect_wall_ms": sorted(detect_ns)[len(detect_ns) // 2] / 1e6,
           "kernel_ms": total / 1e6, "alg_flop": sum(x[2] for x in L), "layers": out_layers, "families": fams}
    if a.build:
        res["build"] = a.build
        res["build_id"] = a.build.rsplit("build ", 1)[-1].strip() if "build " in a.build else None
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
