"""Serving-batch forward latency vs the F(4x4) split-K cap (frt_set_wino4_max_split), IR-101,
eager (no graph replay), n = 1/4/16 crops: which split count the small grids should use.
    python tools/batch1_sweep.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from facerecognitionpipeline_amd import weights as W  # noqa: E402
from facerecognitionpipeline_amd.face_embedder import FaceEmbedder  # noqa: E402
from tests import _frt  # noqa: E402

emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=64, graph_batch=0)
lib = _frt.lib()
for n in (1, 4, 16):
    crops = torch.from_numpy(W.synthetic_crops(n)).cuda()
    row = []
    for cap in (0, 16, 8, 4, 2):
        lib.frt_set_wino4_max_split(cap)
        for _ in range(5):
            emb.embed_tensor(crops)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(30):
            emb.embed_tensor(crops)
        torch.cuda.synchronize()
        row.append(f"cap {cap:2d}: {(time.perf_counter() - t) / 30 * 1e3:.3f} ms")
    print(f"n={n:2d} " + " | ".join(row), flush=True)
lib.frt_set_wino4_max_split(0)
