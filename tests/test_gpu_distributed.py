"""C5's sharded form on the HIP kernels: world_size 2 (gloo), both ranks on cuda:0.

bench.py --gpus N runs one rank per GPU over RCCL; RCCL refuses two ranks on one GPU, so
this test drives the same distributed.py code (broadcast_gallery of a 100k-row gallery,
embed_match_sharded with device_embed_match, gather_topk) under gloo with two processes
sharing the box's single GPU.  Each rank runs the real fr_embed_match on its 256-probe
shard.  Bars: the gathered (idx, score) equal the single-rank fr_embed_match of the whole
batch bit for bit (same 256-crop chunks), and top-1 equals the CPU oracle on sampled rows.
What this cannot show is the RCCL/xGMI broadcast's speed.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
G = 100_000
N = 512  # 256 probes per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gallery_and_probes(emb, dev):
    from facerecognitionpipeline_amd import weights as W
    gal_crops = W.synthetic_crops(1000, W.CROP_SEED_GALLERY)
    g0 = emb.embed_tensor(torch.from_numpy(gal_crops).to(dev)).cpu().numpy()
    probes = W.probe_crops(gal_crops, N, seed=W.CROP_SEED_PROBE)
    return W.expand_gallery(g0, G), probes


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from facerecognitionpipeline_amd.distributed import broadcast_gallery, device_embed_match, embed_match_sharded
        from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
        dev = torch.device("cuda", 0)
        emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", device=dev, max_batch=256)
        E, probes = _gallery_and_probes(emb, dev) if rank == 0 else (None, None)
        gallery = broadcast_gallery(None if E is None else torch.from_numpy(E).to(dev), G, dev, src=0)
        emb.model.gallery_set(gallery)
        # every rank holds the whole batch (host); each embeds + matches only its slice
        if rank != 0:
            from facerecognitionpipeline_amd import weights as W
            probes = W.probe_crops(W.synthetic_crops(1000, W.CROP_SEED_GALLERY), N, seed=W.CROP_SEED_PROBE)
        idx, score = embed_match_sharded(torch.from_numpy(probes), device_embed_match(emb, 5))
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), idx=idx.cpu().numpy(), score=score.cpu().numpy(),
                 gallery_sum=np.float64(gallery.double().sum().item()))
    finally:
        dist.destroy_process_group()


def test_sharded_embed_match_world2_on_one_gpu(tmp_path):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    r0, r1 = (np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2))
    assert float(r0["gallery_sum"]) == float(r1["gallery_sum"])  # the broadcast replicated it
    assert np.array_equal(r0["idx"], r1["idx"]) and np.array_equal(r0["score"], r1["score"])

    # single rank, whole batch, same kernels and 256-crop chunks
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from oracle.adaface_net import load_oracle
    from oracle import reference_path as rp
    from facerecognitionpipeline_amd import weights as W
    dev = torch.device("cuda", 0)
    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", device=dev, max_batch=256)
    E, probes = _gallery_and_probes(emb, dev)
    emb.model.gallery_set(torch.from_numpy(E).to(dev))
    idx = torch.empty((N, 5), dtype=torch.int32, device=dev)
    sc = torch.empty((N, 5), dtype=torch.float32, device=dev)
    e_out = torch.empty((N, 512), dtype=torch.float32, device=dev)
    emb.model.embed_match(torch.from_numpy(probes).to(dev), 5, idx, sc, e_out)
    assert np.array_equal(r0["idx"], idx.cpu().numpy())
    assert np.array_equal(r0["score"], sc.cpu().numpy())
    # top-1 vs the CPU oracle on sampled probes of both shards (probe i is a noisy copy of row i % 1000)
    torch.set_num_threads(16)
    sel = np.array([0, 7, 100, 255, 256, 300, 411, 511])
    ref = rp.extract_embeddings_batch(load_oracle("ir_101", W.synthetic_state_dict("ir_101")), list(probes[sel]))
    ri, rs = rp.topk_policy(np.stack([rp.search_scores(E, q) for q in ref]), 5)
    assert np.array_equal(r0["idx"][sel, 0], ri[:, 0])
    assert np.abs(r0["score"][sel] - rs).max() <= 1e-4
