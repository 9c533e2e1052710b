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
    """all_gather every rank's [n_r, k] results back into input order [n_total, k], on ``idx``'s device
    whatever the backend (gloo gathers through the host, RCCL in place)."""
    world = dist.get_world_size(group)
    k = idx.shape[1]
    longest = shard_range(n_total, world, 0)[1]
    # gloo gathers host tensors only: device results go through the host there (RCCL gathers
    # them in place)
    dev = idx.device if (idx.device.type == "cpu" or dist.get_backend(group) != "gloo") else torch.device("cpu")
    pad_i = torch.full((longest, k), -1, dtype=torch.int32, device=dev)
    pad_s = torch.zeros((longest, k), dtype=torch.float32, device=dev)
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
    return torch.cat(out_i).to(idx.device), torch.cat(out_s).to(score.device)


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


SYNC_NONE, SYNC_DELTA, SYNC_FULL = 0, 1, 2


def broadcast_gallery_update(gm, device: torch.device, src: int = 0, group=None):
    """Ship rank ``src``'s gallery changes to every rank with one small exchange.

    On ``src`` pass the GalleryManager (others pass None).  When every rank holds the
    previous version, only the row delta travels (ops [n,2] int32 + changed rows [m,512]
    f32: an enrollment of one student is 2 KB, not the whole G x 512 matrix); otherwise
    the full matrix is broadcast.  Returns ``(mode, payload)`` where payload is
    (ops, rows) for SYNC_DELTA, the [G,512] matrix for SYNC_FULL, None for SYNC_NONE;
    apply it with ``apply_gallery_update``.  Lockstep contract: every rank applies every
    update it receives, in order.
    """
    rank = dist.get_rank(group)
    hdr = torch.zeros(3, dtype=torch.int64, device=device)
    ops = rows = E = None
    if rank == src:
        if gm._device_version == gm._version and gm._device_current():
            mode = SYNC_NONE
        else:
            delta = gm.pending_delta()
            if delta is None:
                mode = SYNC_FULL
                E_np, _ids = gm.get_gallery_embeddings()
                E = torch.as_tensor(E_np.reshape(-1, 512), dtype=torch.float32)
                hdr[:] = torch.tensor([mode, E.shape[0], 0])
            else:
                mode = SYNC_DELTA
                ops, rows, _ids = delta
                hdr[:] = torch.tensor([mode, ops.shape[0], rows.shape[0]])
        hdr[0] = mode
    dist.broadcast(hdr, src=src, group=group)
    mode, a, b = (int(x) for x in hdr.tolist())
    if mode == SYNC_NONE:
        return mode, None
    if mode == SYNC_FULL:
        return mode, broadcast_gallery(E, a, device, src=src, group=group)
    ops_b = (ops.to(device) if rank == src else torch.empty((a, 2), dtype=torch.int32, device=device)).contiguous()
    rows_b = (rows.to(device) if rank == src else torch.empty((b, 512), dtype=torch.float32, device=device)).contiguous()
    dist.broadcast(ops_b, src=src, group=group)
    if b:
        dist.broadcast(rows_b, src=src, group=group)
    return mode, (ops_b, rows_b)


def apply_gallery_update(mode: int, payload, handle=None, matrix: Optional[torch.Tensor] = None):
    """Apply what ``broadcast_gallery_update`` returned to a libfrhip handle (GPU ranks) or
    to a plain [G,512] tensor (returns the new tensor; the CPU/gloo form)."""
    from .gallery_manager import apply_gallery_delta, apply_gallery_delta_matrix
    if mode == SYNC_NONE:
        return matrix
    if mode == SYNC_FULL:
        if handle is not None:
            handle.gallery_set(payload)
        return payload
    ops, rows = payload
    if handle is not None:
        apply_gallery_delta(handle, ops, rows)
        return None
    return apply_gallery_delta_matrix(matrix, ops, rows)


def sync_gallery(gm, handle, device: torch.device, src: int = 0, group=None,
                 matrix: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Every rank: bring ``handle`` (this rank's libfrhip handle; on ``src`` the one the
    GalleryManager is attached to) or ``matrix`` up to ``src``'s gallery.  ``gm`` on src only."""
    import contextlib
    # on src, the gallery lock spans building the delta, applying it and marking it synced
    with (gm._lock if gm is not None else contextlib.nullcontext()):
        mode, payload = broadcast_gallery_update(gm, device, src=src, group=group)
        out = apply_gallery_update(mode, payload, handle=handle, matrix=matrix)
        if dist.get_rank(group) == src and mode != SYNC_NONE:
            gm._mark_synced(list(gm.students.keys()))
    return out
