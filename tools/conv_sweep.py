#!/usr/bin/env python3
"""Time every conv layer shape of an IR backbone under every tile config (GPU).

usage: python tools/conv_sweep.py [--arch ir_101] [--batch 256] [--reps 5] [--json out.json]
Prints per (layer shape, tile): microseconds per launch and TF/s.  Used to
choose the per-shape tile table of the runtime.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from facerecognitionpipeline_amd.arch import block_specs  # noqa: E402
from tests import _frt  # noqa: E402

TILES = {0: "256x64", 1: "128x128", 2: "128x64", 3: "64x128", 4: "256x128", 5: "128x256", 6: "128x128w8",
         7: "256x128w8", 8: "128x64w8", 9: "64x256w8", 10: "256x64w8"}


def shapes(arch):
    seen = {}
    hw = 112
    for cin, d, s in block_specs(arch):
        seen.setdefault(("conv1", cin, d, hw, 1, 3, 1), 0)
        seen[("conv1", cin, d, hw, 1, 3, 1)] += 1
        ho = hw // s
        if cin != d:
            seen.setdefault(("short", cin, d, hw, 2, 1, 0), 0)
            seen[("short", cin, d, hw, 2, 1, 0)] += 1
        key = ("conv2", d, d, hw, s, 3, 1)
        seen[key] = seen.get(key, 0) + 1
        hw = ho
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ir_101")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tiles", default="0,1,2,3,4,5")
    ap.add_argument("--json", default=None)
    ap.add_argument("--filter", default=None, help="substring of the layer label to run")
    ap.add_argument("--sk", type=int, default=1, help="1 = persistent stream-K schedule, 0 = one block per tile")
    ap.add_argument("--precision", type=int, default=0, help="0 = f32 MFMA, 1 = bf16x3 split")
    a = ap.parse_args()
    B = a.batch
    dev = torch.device("cuda", 0)
    tiles = [int(t) for t in a.tiles.split(",")]
    results = []
    for (kind, cin, cout, hw, stride, k, pad), count in shapes(a.arch).items():
        x = torch.randn(B, hw, hw, cin, device=dev)
        w = torch.randn(cout, k, k, cin, device=dev) / (cin * k * k) ** 0.5
        ho = (hw + 2 * pad - k) // stride + 1
        sc = torch.rand(cout, device=dev) + 0.5
        sh = torch.rand(cout, device=dev) - 0.5
        al = torch.full((cout,), 0.25, device=dev)
        psc = torch.rand(cin, device=dev) + 0.5
        psh = torch.rand(cin, device=dev) - 0.5
        if kind == "conv1":
            kw = dict(pre=(psc, psh), post=(sc, sh), prelu=al, epi=1)
        elif kind == "short":
            kw = dict(post=(sc, sh), epi=0)
        elif stride == 2 and cin == cout and cin == 64:
            kw = dict(post=(sc, sh), res=torch.randn(B, hw, hw, cout, device=dev), res_hw=(hw, hw), epi=3)
        else:
            kw = dict(post=(sc, sh), res=torch.randn(B, ho, ho, cout, device=dev), epi=2)
        flop = 2.0 * B * ho * ho * cout * k * k * cin
        label = f"{kind} {cin}->{cout} @{hw} s{stride}"
        if a.filter and a.filter not in label:
            continue
        row = {"layer": label, "count": count, "flop": flop, "tiles": {}}
        for t in tiles:
            try:
                _frt.conv2d(x, w, B, hw, hw, cin, cout, k, k, stride, pad, tile=t, stream_k=a.sk, precision=a.precision, **kw)
            except Exception as e:  # noqa: BLE001
                row["tiles"][TILES[t]] = str(e)
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                _frt.conv2d(x, w, B, hw, hw, cin, cout, k, k, stride, pad, tile=t, stream_k=a.sk, precision=a.precision, **kw)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            row["tiles"][TILES[t]] = {"us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}
        best = min((v["us"], n) for n, v in row["tiles"].items() if isinstance(v, dict))
        row["best"] = best[1]
        results.append(row)
        print(f"{row['layer']:28s} x{count:2d} " + " ".join(
            f"{n}:{v['tflops'] if isinstance(v, dict) else 'ERR':>6}" for n, v in row["tiles"].items())
            + f"  best {best[1]}", flush=True)
    tot_best = sum(r["count"] * min(v["us"] for v in r["tiles"].values() if isinstance(v, dict)) for r in results)
    tot_flop = sum(r["count"] * r["flop"] for r in results)
    print(f"sum of best per-shape conv time: {tot_best / 1e3:.2f} ms -> {tot_flop / tot_best / 1e6:.1f} TF/s")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
