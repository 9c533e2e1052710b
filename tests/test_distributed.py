"""world_size-2 gloo test of the multi-GPU orchestration (CPU tensors).

The per-rank compute is the CPU oracle's search here (the HIP kernels need a
GPU); what is tested is the sharding, the gallery broadcast and the result
gather that bench.py / distributed.py run over RCCL on MI355X.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from facerecognitionpipeline_amd.distributed import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, golden, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from facerecognitionpipeline_amd.distributed import broadcast_gallery, embed_match_sharded
        from oracle.reference_path import search_scores, topk_policy
        f = np.load(golden)
        E_src = torch.from_numpy(f["ref_template"]) if rank == 0 else None
        E = broadcast_gallery(E_src, f["ref_template"].shape[0], torch.device("cpu"))
        probes = torch.from_numpy(f["embeddings"].reshape(-1, 512))

        def local(shard):
            S = np.stack([search_scores(E.numpy(), x) for x in shard.numpy()]) if len(shard) else np.zeros((0, 23))
            i, s = topk_policy(S, 5) if len(shard) else (np.zeros((0, 5), np.int32), np.zeros((0, 5), np.float32))
            return torch.from_numpy(i), torch.from_numpy(s)

        idx, score = embed_match_sharded(probes, local)
        if rank == 0:
            q.put((idx.numpy(), score.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 256, 2048, 2049):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


@pytest.mark.parametrize("world", [2])
def test_gloo_broadcast_shard_gather_matches_single_rank(world, golden_dir):
    golden = os.path.join(golden_dir, "backup_adaface_ir_101.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, golden, q)) for r in range(world)]
    for p in procs:
        p.start()
    idx, score = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f = np.load(golden)
    assert np.array_equal(idx, f["search_idx"])
    assert np.abs(score - f["search_score"]).max() <= 1e-6


class _TagOnlyHandle:
    """Stands in for a libfrhip handle on CPU: only the gallery tag the sync protocol reads."""
    device = torch.device("cpu")
    gallery_tag = None


def _sync_worker(rank, world, port, tmp, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from facerecognitionpipeline_amd.distributed import sync_gallery
        from facerecognitionpipeline_amd.gallery_manager import GalleryManager
        dev = torch.device("cpu")
        rng = np.random.default_rng(5)
        gm = None
        if rank == 0:
            gm = GalleryManager(gallery_path=os.path.join(tmp, "g", "s.npz"), verbose=False)
            gm.attach_handle(_TagOnlyHandle())
            for i in range(5):
                gm.add_student(f"S{i}", f"N{i}", rng.normal(size=(3, 512)).astype(np.float32))
        modes, M = [], None
        M = sync_gallery(gm, None, dev, matrix=M)                    # first: full
        modes.append(M.shape[0])
        if rank == 0:
            gm.add_student("S5", "N5", rng.normal(size=(2, 512)).astype(np.float32))
            gm.update_embeddings("S1", rng.normal(size=(1, 512)).astype(np.float32))
            gm.delete_student("S2")
            gm.add_student("S6", "N6", rng.normal(size=(4, 512)).astype(np.float32))
            gm.add_student("S0", "N0b", rng.normal(size=(3, 512)).astype(np.float32), overwrite=True)
            gm.add_student("S7", "N7", rng.normal(size=(1, 512)).astype(np.float32))
            gm.delete_student("S7")
            assert gm.pending_delta() is not None
        M = sync_gallery(gm, None, dev, matrix=M)                    # delta
        modes.append(M.shape[0])
        M2 = sync_gallery(gm, None, dev, matrix=M)                   # nothing changed
        assert M2 is M
        want = None
        if rank == 0:
            want = torch.from_numpy(gm.get_gallery_embeddings()[0].astype(np.float32))
        q.put((rank, modes, M.numpy(), None if want is None else want.numpy()))
    finally:
        dist.destroy_process_group()


def test_gloo_gallery_delta_sync(tmp_path):
    """Enrollment changes on rank 0 reach every rank as a row delta (gallery lifecycle,
    SURVEY §8(f) rank 3), and every rank ends with rank 0's template matrix."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict()
    for _ in range(world):
        r, modes, M, want = q.get(timeout=120)
        out[r] = (modes, M, want)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = out[0][2]
    assert want.shape == (6, 512)
    for r in range(world):
        assert out[r][0] == [5, 6]
        assert np.array_equal(out[r][1], want)
