"""PyTorch-ROCm operator surface of the hot path: ``torch.ops.frhip.*``.

SURVEY.md §8(b) asks for ``frhip::embed`` and ``frhip::match_topk`` as
``torch.library`` ops over PyTorch tensors, next to the C ABI.  They run the same
libfrhip entry points on the tensors' device and the current stream (no copy, no
CPU fallback).  A model or gallery is named by the integer id ``register``
returns for a ``FaceEmbedder`` / ``_lib.Handle``:

    hid = torch_ops.register(embedder)                       # once
    e = torch.ops.frhip.embed(rgb_u8_nhwc, hid, True)        # [N,512] f32
    idx, score = torch.ops.frhip.match_topk(e, hid, 5)       # [N,5] i32 / f32
    idx, score, e = torch.ops.frhip.embed_match(rgb, hid, 5)

Each op has a fake (meta) implementation, so the ops trace under
``torch.fx`` / ``torch.export`` with the right output shapes.
"""
from __future__ import annotations

import itertools
import threading
from typing import Dict, Tuple

import torch

from . import _lib

_handles: Dict[int, "_lib.Handle"] = {}
_ids = itertools.count(1)
_lock = threading.Lock()


def register(obj) -> int:
    """Id for a FaceEmbedder (its model handle) or a raw ``_lib.Handle``."""
    h = obj.model if hasattr(obj, "model") and isinstance(obj.model, _lib.Handle) else obj
    if not isinstance(h, _lib.Handle):
        raise TypeError("register() takes a FaceEmbedder or a facerecognitionpipeline_amd._lib.Handle")
    with _lock:
        hid = next(_ids)
        _handles[hid] = h
    return hid


def unregister(hid: int) -> None:
    with _lock:
        _handles.pop(hid, None)


def _get(hid: int) -> "_lib.Handle":
    try:
        return _handles[hid]
    except KeyError:
        raise ValueError(f"frhip handle id {hid} is not registered") from None


def _check_rgb(rgb: torch.Tensor, h: "_lib.Handle") -> torch.Tensor:
    if rgb.dtype != torch.uint8 or rgb.dim() != 4 or tuple(rgb.shape[1:]) != (112, 112, 3):
        raise ValueError("expected a uint8 [N,112,112,3] RGB tensor")
    if rgb.device != h.device:
        raise ValueError(f"input is on {rgb.device}, the model on {h.device} (no CPU fallback)")
    return rgb.contiguous()


@torch.library.custom_op("frhip::embed", mutates_args=())
def embed(rgb: torch.Tensor, handle: int, normalize: bool) -> torch.Tensor:
    h = _get(handle)
    rgb = _check_rgb(rgb, h)
    out = torch.empty((rgb.shape[0], 512), dtype=torch.float32, device=rgb.device)
    h.embed(rgb, out, normalize)
    return out


@embed.register_fake
def _(rgb, handle, normalize):
    return rgb.new_empty((rgb.shape[0], 512), dtype=torch.float32)


@torch.library.custom_op("frhip::match_topk", mutates_args=())
def match_topk(q: torch.Tensor, handle: int, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    h = _get(handle)
    if q.dtype != torch.float32 or q.dim() != 2 or q.shape[1] != 512 or q.device != h.device:
        raise ValueError("expected a float32 [N,512] query tensor on the model's device")
    q = q.contiguous()
    idx = torch.empty((q.shape[0], k), dtype=torch.int32, device=q.device)
    score = torch.empty((q.shape[0], k), dtype=torch.float32, device=q.device)
    h.match(q, k, idx, score)
    return idx, score


@match_topk.register_fake
def _(q, handle, k):
    return (q.new_empty((q.shape[0], k), dtype=torch.int32), q.new_empty((q.shape[0], k), dtype=torch.float32))


@torch.library.custom_op("frhip::embed_match", mutates_args=())
def embed_match(rgb: torch.Tensor, handle: int, k: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    h = _get(handle)
    rgb = _check_rgb(rgb, h)
    n = rgb.shape[0]
    idx = torch.empty((n, k), dtype=torch.int32, device=rgb.device)
    score = torch.empty((n, k), dtype=torch.float32, device=rgb.device)
    emb = torch.empty((n, 512), dtype=torch.float32, device=rgb.device)
    h.embed_match(rgb, k, idx, score, emb)
    return idx, score, emb


@embed_match.register_fake
def _(rgb, handle, k):
    n = rgb.shape[0]
    return (rgb.new_empty((n, k), dtype=torch.int32), rgb.new_empty((n, k), dtype=torch.float32),
            rgb.new_empty((n, 512), dtype=torch.float32))
