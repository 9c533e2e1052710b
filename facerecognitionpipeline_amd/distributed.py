"""Multi-GPU form of the hot path: one process per GPU, probes sharded, gallery broadcast.

The reference is single-device (``face_embedder.py:33``).
Faces are independent, so the path shards with no data-path collective:

* gallery exchange — rank ``src`` holds the G x 512 template matrix (it built
  it from its gallery); one ``broadcast`` (RCCL over xGMI on MI355X,
  backend "nccl") replicates it into every rank's HBM, once per gallery
  version: 100k rows = 204.8 MB.
* probes — rank r takes the contiguous slice ``shard_range(n, world, r)`` and
  runs embed + match locally.
* results — optionally ``all_gather``ed (n x k x 8 B) so every rank, or just
  the caller on rank 0, sees the whole batch in input order.

Everything here is backend-agnostic; the same code runs under ``gloo`` on CPU
tensors in the tests (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, end) of ``n`` probes for ``rank``; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_gallery(gallery: Optional[torch.Tensor], rows: int, device: torch.device, src: int = 0,
                      group=None) -> torch.Tensor:
    """Replicate the [rows, 512] f32 template matrix from ``src`` to every rank."""
    if dist.get_rank(group) == src:
        if gallery is None or tuple(gallery.shape) != (rows, 512):
            raise ValueError("source rank must pass the [rows, 512] gallery")
        buf = gallery.to(device=device, dtype=torch.float32).contiguous()
    else:
        buf = torch.empty((rows, 512), dtype=torch.float32, device=device)
    dist.broadcast(buf, src=src, group=group)
    return buf


def gather_topk(idx: torch.Tensor, score: torch.Tensor, n_total: int, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """all_gather every rank's [n_r, k] results back into input order [n_total, k]."""
    world = dist.get_world_size(group)
    k = idx.shape[1]
    longest = shard_range(n_total, world, 0)[1]
    pad_i = torch.full((longest, k), -1, dtype=torch.int32, device=idx.device)
    pad_s = torch.zeros((longest, k), dtype=torch.float32, device=score.device)
    pad_i[: idx.shape[0]] = idx
    pad_s[: score.shape[0]] = score
    all_i = [torch.empty_like(pad_i) for _ in range(world)]
    all_s = [torch.empty_like(pad_s) for _ in range(world)]
    dist.all_gather(all_i, pad_i, group=group)
    dist.all_gather(all_s, pad_s, group=group)
    out_i, out_s = [], []
    for r in range(world):
        a, b = shard_range(n_total, world, r)
        out_i.append(all_i[r][: b - a])
        out_s.append(all_s[r][: b - a])
    return torch.cat(out_i), torch.cat(out_s)


def embed_match_sharded(probes: torch.Tensor, local_fn: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]],
                        group=None, gather: bool = True):
    """Run ``local_fn`` (embed + match of a probe shard) on this rank's slice of ``probes``.

    ``probes`` is the full batch (host or device); each rank only touches its slice.
    Returns the gathered [n, k] (idx, score) if ``gather`` else this rank's shard.
    """
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    a, b = shard_range(probes.shape[0], world, rank)
    idx, score = local_fn(probes[a:b])
    if not gather:
        return idx, score
    return gather_topk(idx, score, probes.shape[0], group)


def device_embed_match(embedder, k: int) -> Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]:
    """local_fn for a FaceEmbedder whose handle already holds the (broadcast) gallery."""

    def fn(rgb: torch.Tensor):
        rgb = rgb.to(embedder.device).contiguous()
        n = rgb.shape[0]
        idx = torch.empty((n, k), dtype=torch.int32, device=embedder.device)
        score = torch.empty((n, k), dtype=torch.float32, device=embedder.device)
        if n:
            embedder.model.embed_match(rgb, k, idx, score)
        return idx, score

    return fn
