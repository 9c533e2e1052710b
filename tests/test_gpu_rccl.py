"""The RCCL code path of C5 / bench.py --gpus N, executed on the one GPU of the test box.

bench.py initialises ``init_process_group("nccl", device_id=...)`` (backend "nccl" is RCCL on
ROCm) and moves the gallery and the results with ``distributed.py``.  A one-GPU box cannot run
two RCCL ranks (RCCL refuses two ranks on one device), so this test runs that exact code at
world size 1 in a fresh process: RCCL communicator init on cuda:0, ``broadcast_gallery`` of a
100k x 512 device tensor, ``embed_match_sharded(device_embed_match)`` with ``gather_topk`` on
device tensors (RCCL all_gather), and a row-delta ``sync_gallery`` (RCCL broadcasts of the
header, ops and rows).  Bars: bit-identical to a direct ``fr_embed_match`` of the same batch,
results left on the GPU, and the delta-synced handle equal to a fresh upload.  What it cannot
show is xGMI speed or a 1->8 scaling curve.
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
G = 100_000
N = 300


def _worker(init_file, out_path):
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="file://" + init_file, rank=0, world_size=1, device_id=dev)
    try:
        from facerecognitionpipeline_amd import weights as W
        from facerecognitionpipeline_amd.distributed import (apply_gallery_update, broadcast_gallery,
                                                              broadcast_gallery_update, device_embed_match,
                                                              embed_match_sharded, sync_gallery)
        from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
        from facerecognitionpipeline_amd.gallery_manager import GalleryManager
        assert dist.get_backend() == "nccl"
        emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", device=dev, max_batch=256)
        gal_crops = W.synthetic_crops(1000, W.CROP_SEED_GALLERY)
        g0 = emb.embed_tensor(torch.from_numpy(gal_crops).to(dev)).cpu().numpy()
        E = torch.from_numpy(W.expand_gallery(g0, G)).to(dev)
        gallery = broadcast_gallery(E, G, dev, src=0)
        assert gallery.is_cuda and torch.equal(gallery, E)
        emb.model.gallery_set(gallery)
        probes = torch.from_numpy(W.probe_crops(gal_crops, N, seed=W.CROP_SEED_PROBE)).to(dev)
        idx, score = embed_match_sharded(probes, device_embed_match(emb, 5))
        assert idx.is_cuda and score.is_cuda  # RCCL all_gather keeps results on the device
        # direct fr_embed_match of the same batch
        di = torch.empty((N, 5), dtype=torch.int32, device=dev)
        ds = torch.empty((N, 5), dtype=torch.float32, device=dev)
        emb.model.embed_match(probes, 5, di, ds)
        # gallery lifecycle over RCCL: rank 0's manager drives this rank's handle (emb.model)
        gm = GalleryManager(gallery_path="/tmp/frhip_rccl/students.npz", device=dev, verbose=False)
        gm.attach_handle(emb.model)
        for i in range(40):
            gm.add_student(f"S{i}", f"N{i}", g0[i])
        sync_gallery(gm, emb.model, dev, src=0)  # first sync: the full matrix
        gm.add_student("S40", "N40", g0[40])
        gm.delete_student("S3")
        with gm._lock:  # sync_gallery's steps, keeping the mode for the assertion
            mode, payload = broadcast_gallery_update(gm, dev, src=0)
            apply_gallery_update(mode, payload, handle=emb.model)
            gm._mark_synced(list(gm.students.keys()))
        h_rank = emb.model
        q = torch.from_numpy(g0[:64]).to(dev)
        qi = torch.empty((64, 3), dtype=torch.int32, device=dev)
        qs = torch.empty((64, 3), dtype=torch.float32, device=dev)
        h_rank.match(q, 3, qi, qs)
        fresh = FaceEmbedder(architecture="ir_50", model_path="synthetic", device=dev, max_batch=1).model
        fresh.gallery_set(torch.from_numpy(gm.get_gallery_embeddings()[0].astype(np.float32)).to(dev))
        fi = torch.empty_like(qi)
        fs = torch.empty_like(qs)
        fresh.match(q, 3, fi, fs)
        np.savez(out_path, idx=idx.cpu().numpy(), score=score.cpu().numpy(), di=di.cpu().numpy(),
                 ds=ds.cpu().numpy(), qi=qi.cpu().numpy(), qs=qs.cpu().numpy(), fi=fi.cpu().numpy(),
                 fs=fs.cpu().numpy(), mode=np.int64(mode))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_broadcast_shard_gather_delta(tmp_path):
    init_file = str(tmp_path / "rccl_init")
    out = str(tmp_path / "rccl.npz")
    p = mp.get_context("spawn").Process(target=_worker, args=(init_file, out))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0
    r = np.load(out)
    assert np.array_equal(r["idx"], r["di"]) and np.array_equal(r["score"], r["ds"])
    assert int(r["mode"]) == 1  # the enrolment + delete travelled as a row delta, not the matrix
    assert np.array_equal(r["qi"], r["fi"]) and np.array_equal(r["qs"], r["fs"])
