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
