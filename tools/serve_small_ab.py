"""Serving latency with conv_small.hip's kernel for every body 3x3 conv (frt_set_small_conv)
against the F(4x4) split-K path, per batch size (embed + match, IR-101, G = 1000, top-3).

    python tools/serve_small_ab.py [--ns 1,2,4,8,16]
    python tools/serve_small_ab.py --pre-epilogue [--ns 1]   (conv1 pre-BN in conv2's epilogue on / off)
    python tools/serve_small_ab.py --pixels 1024,4096 [--reps 8]  (batch-1 pixel limit, interleaved)
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from facerecognitionpipeline_amd import weights as W  # noqa: E402
from facerecognitionpipeline_amd.face_embedder import FaceEmbedder  # noqa: E402
from tests import _frt  # noqa: E402


def timed(fn, iters):
    fn()
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8,16")
    ap.add_argument("--pre-epilogue", action="store_true")
    ap.add_argument("--pixels", default=None, help="batch-1 serving-kernel pixel limits to interleave")
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=64, graph_batch=0)
    h = emb.model
    G = 1000
    gal = emb.embed_tensor(torch.from_numpy(W.synthetic_crops(G, seed=W.CROP_SEED_GALLERY)).cuda())
    h.gallery_set(gal)
    probes = torch.from_numpy(W.probe_crops(W.synthetic_crops(64, seed=W.CROP_SEED_GALLERY), 64)).cuda()
    L = _frt.lib()
    for n in [int(x) for x in args.ns.split(",")]:
        rgb = probes[:n].contiguous()
        idx = torch.empty((n, 3), dtype=torch.int32, device="cuda")
        sc = torch.empty((n, 3), dtype=torch.float32, device="cuda")
        if args.pixels:
            # one process, the limits interleaved rep by rep, every run kept: the spread is the
            # yardstick for the difference
            lims = [int(x) for x in args.pixels.split(",")]
            t = {m: [] for m in lims}
            for rep in range(args.reps):
                for m in (lims if rep % 2 == 0 else lims[::-1]):
                    assert L.frt_set_small_conv_pixels(h.h, m) == 0
                    t[m].append(timed(lambda: h.embed_match(rgb, 3, idx, sc), 200))
            assert L.frt_set_small_conv_pixels(h.h, 4096) == 0
            for m in lims:
                v = sorted(t[m])
                print(f"n={n} pixel limit {m}: median {v[len(v) // 2]:.4f} ms, min {v[0]:.4f}, max {v[-1]:.4f} "
                      f"(runs {' '.join(f'{x:.4f}' for x in t[m])})", flush=True)
            continue
        if args.pre_epilogue:
            assert L.frt_set_small_conv(h.h, n) == 0
            t = {0: [], 1: []}
            for rep in range(4):
                for on in (1, 0):
                    assert L.frt_set_small_conv_pre_epilogue(h.h, on) == 0
                    t[on].append(timed(lambda: h.embed_match(rgb, 3, idx, sc), 100))
            assert L.frt_set_small_conv_pre_epilogue(h.h, 1) == 0
            print(f"n={n:3d} embed+match: pre-BN per tap {min(t[0]):.3f} ms (runs {' '.join(f'{x:.3f}' for x in t[0])}), "
                  f"in conv2's epilogue {min(t[1]):.3f} ms (runs {' '.join(f'{x:.3f}' for x in t[1])})", flush=True)
            continue
        row = []
        for mode in (0, n):
            assert L.frt_set_small_conv(h.h, mode) == 0
            row.append(timed(lambda: h.embed_match(rgb, 3, idx, sc), 50))
        print(f"n={n:3d} embed+match: F(4x4) split-K path {row[0]:.3f} ms, serving conv kernel {row[1]:.3f} ms "
              f"({row[0] / row[1]:.2f}x)", flush=True)
    assert L.frt_set_small_conv(h.h, 1) == 0


if __name__ == "__main__":
    main()
