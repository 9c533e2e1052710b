#!/usr/bin/env python3
"""Time the SCRFD-10G detector's implicit-GEMM convs (stride-2 3x3, 1x1 laterals and shortcuts) at
their C4 shapes (32 frames, 1080p letterbox rows of detector.cpp's row_plan) under every tile the
kernel instances allow (GPU).

usage: python tools/det_conv_sweep.py [--frames 32] [--reps 10] [--sk 1]
Prints per layer: microseconds per launch for each tile, and the runtime's current choice (the
detector branch of the tile rule in frhip_runtime.cpp run_conv).  Conv + BN + ReLU (epi 1 without
pre-BN) runs on the detector's own instance set (conv_det.hip: tiles 128x64w8, 128x128w8,
256x128w8); conv + BN (epi 0) and conv + BN + residual (epi 2) on the network's sets.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import _frt  # noqa: E402

TILES = {0: "256x64", 1: "128x128", 2: "128x64", 3: "64x128", 4: "256x128", 5: "128x256", 6: "128x128w8",
         7: "256x128w8", 8: "128x64w8", 9: "64x256w8", 10: "256x64w8"}
DET_TILES = (6, 7, 8)

# (layer, cin, cout, H, W, k, stride, epi, current tile): channels padded to 32 as the detector
# stores them; stage 2 runs on 576 of 640 canvas rows (144 at stride 4)
LAYERS = [
    ("s2.0.conv1 3x3 s2", 64, 96, 144, 160, 3, 2, 1, 6),
    ("s2.0.down 1x1", 64, 96, 72, 80, 1, 1, 0, 6),
    ("s3.0.conv1 3x3 s2", 96, 96, 80, 80, 3, 2, 1, 6),
    ("s3.0.down 1x1", 96, 96, 40, 40, 1, 1, 0, 6),
    ("s4.0.conv1 3x3 s2", 96, 224, 40, 40, 3, 2, 1, 6),
    ("s4.0.down 1x1", 96, 224, 20, 20, 1, 1, 0, 6),
    ("lateral0 1x1", 96, 64, 80, 80, 1, 1, 0, 0),
    ("lateral1 1x1", 96, 64, 40, 40, 1, 1, 0, 8),
    ("lateral2 1x1", 224, 64, 20, 20, 1, 1, 0, 8),
    ("neck.down0 3x3 s2 +res", 64, 64, 80, 80, 3, 2, 2, 8),
    ("neck.down1 3x3 s2 +res", 64, 64, 40, 40, 3, 2, 2, 8),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sk", type=int, default=1, help="1 = persistent stream-K schedule (the detector's), 0 = one block per tile")
    a = ap.parse_args()
    B = a.frames
    dev = torch.device("cuda", 0)
    tot_cur = tot_best = 0.0
    for name, cin, cout, H, W, k, s, epi, cur in LAYERS:
        pad = 1 if k == 3 else 0
        Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        x = torch.randn(B, H, W, cin, device=dev)
        w = torch.randn(cout, k, k, cin, device=dev) / (cin * k * k) ** 0.5
        kw = dict(post=(torch.rand(cout, device=dev) + 0.5, torch.rand(cout, device=dev) - 0.5), epi=epi)
        if epi == 1:
            kw["prelu"] = torch.zeros(cout, device=dev)
        if epi == 2:
            kw["res"] = torch.randn(B, Ho, Wo, cout, device=dev)
        tiles = DET_TILES if epi == 1 else tuple(TILES)
        res = {}
        ref = None
        for t in tiles:
            try:
                y = _frt.conv2d(x, w, B, H, W, cin, cout, k, k, s, pad, tile=t, stream_k=a.sk, **kw)
            except Exception:  # noqa: BLE001  (a tile the instance set lacks)
                continue
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            elif (ref - y).abs().max() > 1e-5 * ref.abs().max():  # (stream-K sums partial tiles in another order)
                res[t] = None
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                _frt.conv2d(x, w, B, H, W, cin, cout, k, k, s, pad, tile=t, stream_k=a.sk, **kw)
            e1.record()
            torch.cuda.synchronize()
            res[t] = e0.elapsed_time(e1) * 1e3 / a.reps
        ok = {t: v for t, v in res.items() if v is not None}
        best = min(ok, key=ok.get)
        tot_cur += ok.get(cur, float("nan"))
        tot_best += ok[best]
        print(f"{name:24s} M={B * Ho * Wo:7d} N={cout:3d} K={k * k * cin:4d} "
              + " ".join(f"{TILES[t]}:{'MISMATCH' if v is None else f'{v:.1f}'}" for t, v in res.items())
              + f"  current {TILES[cur]} {ok.get(cur, float('nan')):.1f}  best {TILES[best]} {ok[best]:.1f}", flush=True)
    print(f"sum: current tiles {tot_cur:.1f} us, best per layer {tot_best:.1f} us")


if __name__ == "__main__":
    main()
