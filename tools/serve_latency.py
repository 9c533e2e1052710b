"""Serving-path latency on the GPU: small-batch embed+match, eager vs hipGraph replay, and
MatchBatcher under concurrent request threads vs the reference's one-request-at-a-time pattern.

    python tools/serve_latency.py [--json gpurun_out/serve_latency.json]

Every number is wall-clock per call on the host (what a server thread sees), IR-101,
G = 1000 gallery rows, top-3.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from facerecognitionpipeline_amd import weights as W  # noqa: E402
from facerecognitionpipeline_amd.face_embedder import FaceEmbedder  # noqa: E402
from facerecognitionpipeline_amd.face_matcher import FaceMatcher  # noqa: E402
from facerecognitionpipeline_amd.gallery_manager import GalleryManager  # noqa: E402
from facerecognitionpipeline_amd.pipeline import MatchBatcher  # noqa: E402


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
    ap.add_argument("--json", default="gpurun_out/serve_latency.json")
    ap.add_argument("--gallery", type=int, default=1000)
    ap.add_argument("--algos", default="", help="only sweep these conv algorithms (comma list) x --ns")
    ap.add_argument("--ns", default="1,4,16,64")
    ap.add_argument("--graph", type=int, default=0, help="--algos: fr_set_graph_batch value")
    ap.add_argument("--so", default=None, help="a libfrhip.so build to load instead of the package's (A/B)")
    args = ap.parse_args()
    if args.so:
        from facerecognitionpipeline_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.so)
    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=256, graph_batch=0)
    G = args.gallery
    base = W.synthetic_crops(G, seed=W.CROP_SEED_GALLERY)
    E = emb.extract_embeddings_batch(list(base))
    gm = GalleryManager(gallery_path="/tmp/frhip_serve/students.npz", device="cuda:0", verbose=False)
    for i in range(G):
        gm.add_student(f"S{i}", f"N{i}", E[i])
    fm = FaceMatcher(embedder=emb, gallery=gm)
    probes = W.probe_crops(base, 256)
    dev = emb.device
    h = emb.model
    k = 3
    if args.algos:
        for algo in args.algos.split(","):
            h.set_conv_algorithm(algo)
            h.set_graph_batch(args.graph)
            for n in [int(x) for x in args.ns.split(",")]:
                rgb = torch.from_numpy(probes[:n]).to(dev)
                o = torch.empty((n, 512), dtype=torch.float32, device=dev)
                ms = timed(lambda: h.embed(rgb, o, True), 20)
                hh = gm._sync_device()
                idx = torch.empty((n, 5), dtype=torch.int32, device=dev)
                sc = torch.empty((n, 5), dtype=torch.float32, device=dev)
                ms2 = timed(lambda: hh.embed_match(rgb, 5, idx, sc), 20)
                h.profile_enable(True)
                h.profile_read()
                ms3 = timed(lambda: hh.embed_match(rgb, 5, idx, sc), 20)
                h.profile_read()
                h.profile_enable(False)
                print(f"{algo:10s} n={n:3d} embed {ms:.3f} ms, embed+match {ms2:.3f} ms, "
                      f"with HIP-event profiling {ms3:.3f} ms", flush=True)
        return
    out = {"arch": "ir_101", "gallery": G, "top_k": k, "embed_match_ms": {}}
    for n in (1, 2, 4, 8, 16, 32):
        rgb = torch.from_numpy(probes[:n]).to(dev)
        idx = torch.empty((n, k), dtype=torch.int32, device=dev)
        sc = torch.empty((n, k), dtype=torch.float32, device=dev)
        hh = gm._sync_device()
        row = {}
        for mode, gb in (("eager", 0), ("graph", 32)):
            h.set_graph_batch(gb)
            row[mode] = timed(lambda: hh.embed_match(rgb, k, idx, sc), 50)
        row["faces_per_s_graph"] = n / row["graph"] * 1e3
        out["embed_match_ms"][n] = row
        print(f"n={n:3d} embed+match eager {row['eager']:.3f} ms, graph {row['graph']:.3f} ms "
              f"({row['eager'] / row['graph']:.2f}x)", flush=True)
    # reference serving pattern: one match_single_face per request, in sequence
    h.set_graph_batch(16)
    reqs = 128
    fm.match_single_face(probes[0], top_k=k)
    t = time.perf_counter()
    for i in range(reqs):
        fm.match_single_face(probes[i], top_k=k)
    seq = time.perf_counter() - t
    out["sequential_match_single_face"] = {"requests": reqs, "ms_per_request": seq / reqs * 1e3,
                                           "requests_per_s": reqs / seq}
    print(f"sequential match_single_face: {seq / reqs * 1e3:.3f} ms/request", flush=True)
    for threads in (8, 32):
        with MatchBatcher(fm, max_batch=16, max_wait_ms=1.0) as mb:
            for i in range(threads):  # warm every batch size the run can form
                mb.match_single_face(probes[i], top_k=k)
            mb.batches.clear()
            lat = []

            def worker(t0):
                for i in range(t0, reqs * 2, threads):
                    s = time.perf_counter()
                    mb.match_single_face(probes[i % 256], top_k=k)
                    lat.append(time.perf_counter() - s)

            ts = [threading.Thread(target=worker, args=(j,)) for j in range(threads)]
            t = time.perf_counter()
            for th in ts:
                th.start()
            for th in ts:
                th.join()
            wall = time.perf_counter() - t
            out[f"batcher_{threads}_threads"] = {
                "requests": reqs * 2, "requests_per_s": reqs * 2 / wall,
                "p50_ms": float(np.percentile(lat, 50) * 1e3), "p99_ms": float(np.percentile(lat, 99) * 1e3),
                "mean_batch": float(np.mean(mb.batches))}
            print(f"MatchBatcher {threads} threads: {reqs * 2 / wall:.1f} req/s, "
                  f"p50 {np.percentile(lat, 50) * 1e3:.2f} ms, mean batch {np.mean(mb.batches):.1f}", flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.json)), exist_ok=True)
    with open(args.json, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
