#!/usr/bin/env python3
"""Same-process A/B of the C3 step (IR-101 embed + top-5 match of 256 crops vs G = 1,000, two
lanes, fp32) with one runtime switch of tests/_frt.py set to each of --values in turn (the order
rotating per rep), every run kept.

    python tools/c3_switch_ab.py frt_set_wino4_blocked [--reps 6] [--steps 20]      (handle, 0 / 1)
    python tools/c3_switch_ab.py frt_set_conv2sc_tile --global --values -1,2,6,8   (process-wide knob)
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from facerecognitionpipeline_amd import weights as W  # noqa: E402
from facerecognitionpipeline_amd.face_embedder import FaceEmbedder  # noqa: E402
from tests import _frt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("switch")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--global", dest="glob", action="store_true", help="the switch takes (value), not (handle, value)")
    args = ap.parse_args()
    vals = [int(v) for v in args.values.split(",")]
    L = _frt.lib()
    fn = getattr(L, args.switch)
    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=256)
    h = emb.model
    gal_crops = W.synthetic_crops(1000, W.CROP_SEED_GALLERY)
    h.gallery_set(emb.embed_tensor(torch.from_numpy(gal_crops).cuda()))
    rgb = torch.from_numpy(W.probe_crops(gal_crops, 256, seed=W.CROP_SEED_PROBE)).cuda()
    idx = torch.empty((256, 5), dtype=torch.int32, device="cuda")
    sc = torch.empty((256, 5), dtype=torch.float32, device="cuda")
    t = {v: [] for v in vals}
    fam = {v: [] for v in vals}  # ms per one-lane forward of the direct-conv family (HIP events)
    famw = {v: [] for v in vals}  # ... and of the Winograd family
    setv = (lambda v: fn(v)) if args.glob else (lambda v: fn(h.h, v))
    for rep in range(args.reps):
        for on in vals[rep % len(vals):] + vals[:rep % len(vals)]:
            assert setv(on) == 0
            for _ in range(3):
                h.embed_match(rgb, 5, idx, sc)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                h.embed_match(rgb, 5, idx, sc)
            torch.cuda.synchronize()
            t[on].append((time.perf_counter() - t0) / args.steps * 1e3)
            assert (idx[:, 0].cpu().numpy() == np.arange(256)).all()
            h.profile_enable(True)
            h.profile_read()
            for _ in range(3):
                h.embed_match(rgb, 5, idx, sc)
            torch.cuda.synchronize()
            pr = h.profile_read()
            h.profile_enable(False)
            fam[on].append(pr["direct"]["ms"] / 3)
            famw[on].append(pr["winograd"]["ms"] / 3)
    assert setv(vals[0] if args.glob else 1) == 0
    for on in vals:
        v = sorted(t[on])
        print(f"{args.switch}({on}): median {v[len(v) // 2]:.3f} ms/step = {256 / v[len(v) // 2] * 1e3:.0f} faces/s, "
              f"min {v[0]:.3f}, max {v[-1]:.3f} (runs {' '.join(f'{x:.3f}' for x in t[on])}); direct-conv family "
              f"{sorted(fam[on])[len(fam[on]) // 2]:.3f} ms, Winograd family {sorted(famw[on])[len(famw[on]) // 2]:.3f} ms "
              f"per one-lane forward", flush=True)


if __name__ == "__main__":
    main()
