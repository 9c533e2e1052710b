"""Restatement of the reference's embed/match glue — ORACLE, test-only.

Every function cites the reference lines it follows.  Numerics are kept in
the same dtypes as the reference (float64 preprocessing rounded to float32,
numpy float32 renormalisation, float32 sgemv, argsort) so the oracle is the
reference's CPU path, not an idealisation of it.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

INPUT_SIZE = (112, 112)


def preprocess(face_image: np.ndarray) -> torch.Tensor:
    """``FaceEmbedder.preprocess`` adaface branch (face_embedder.py:93-104).

    ``cv2.resize(face_image, (112, 112))`` (INTER_LINEAR) when the crop is not
    112x112 (:94-96; cv2 is absent, so this is the fixed-point restatement
    ``oracle.scrfd.resize_linear_u8`` -- parity vs cv2 itself unpinned), then
    RGB->BGR view, ``(x/255.0 - 0.5)/0.5`` in float64, CHW, ``.float()``,
    batch dim.
    """
    if face_image.shape[:2] != INPUT_SIZE:
        from oracle.scrfd import resize_linear_u8
        face_image = resize_linear_u8(face_image, INPUT_SIZE[1], INPUT_SIZE[0])
    bgr = face_image[:, :, ::-1]
    bgr = (bgr / 255.0 - 0.5) / 0.5
    return torch.from_numpy(bgr.transpose(2, 0, 1)).float().unsqueeze(0)


def preprocess_lut() -> np.ndarray:
    """The 256-entry float32 table preprocess() realises per byte value."""
    v = np.arange(256, dtype=np.float64)
    return ((v / 255.0 - 0.5) / 0.5).astype(np.float32)


def extract_embeddings_batch(model, face_images: Sequence[np.ndarray], normalize: bool = True,
                             batch_size: int = 32) -> np.ndarray:
    """``FaceEmbedder.extract_embeddings_batch`` adaface branch (face_embedder.py:137-182)."""
    if len(face_images) == 0:
        return np.array([])
    out = []
    for i in range(0, len(face_images), batch_size):
        batch = torch.cat([preprocess(f) for f in face_images[i:i + batch_size]], dim=0)
        with torch.no_grad():
            features, _norm = model(batch)
        out.append(features.cpu().numpy())
    emb = np.vstack(out)
    if normalize:
        norms = np.linalg.norm(emb, axis=1, keepdims=True)
        emb = emb / (norms + 1e-8)
    return emb


def extract_embedding(model, face_image: np.ndarray, normalize: bool = True) -> np.ndarray:
    """``FaceEmbedder.extract_embedding`` adaface branch (face_embedder.py:112-135)."""
    with torch.no_grad():
        features, _norm = model(preprocess(face_image))
    emb = features.cpu().numpy().squeeze()
    if normalize:
        emb = emb / (np.linalg.norm(emb) + 1e-8)
    return emb


def search_scores(gallery: np.ndarray, query: np.ndarray) -> np.ndarray:
    """Score vector of ``GalleryManager.search`` (gallery_manager.py:195-196)."""
    q = query / (np.linalg.norm(query) + 1e-8)
    return np.dot(gallery, q)


def search(gallery: np.ndarray, ids: List[str], names: Dict[str, str], query: np.ndarray,
           top_k: int = 5) -> List[Tuple[str, str, float]]:
    """``GalleryManager.search`` (gallery_manager.py:189-205) on a vstacked gallery."""
    if len(ids) == 0:
        return []
    s = search_scores(gallery, query)
    top = np.argsort(s)[::-1][:top_k]
    return [(ids[i], names[ids[i]], float(s[i])) for i in top]


def topk_policy(scores: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Deterministic top-k: descending score, ties by DESCENDING index.

    That is ``np.argsort(s)[::-1][:k]`` (gallery_manager.py:197) whenever numpy's
    sort is stable (its insertion sort for <= 16 elements, or ``kind="stable"``):
    a stable ascending sort, reversed.  numpy's AVX-512 argsort (numpy >= 2 on
    such CPUs) leaves ties in no defined order, so the build fixes this policy;
    parity inputs are designed with margins.  Row-wise on 2-D.
    """
    s = np.atleast_2d(scores)
    n, g = s.shape
    k = min(k, g)
    idx = np.empty((n, k), dtype=np.int32)
    val = np.empty((n, k), dtype=np.float32)
    cols = np.arange(g)
    for r in range(n):
        order = np.lexsort((-cols, -s[r].astype(np.float64)))[:k]
        idx[r] = order
        val[r] = s[r, order]
    return idx, val


def filter_quality_embeddings(embeddings: np.ndarray, min_similarity: float = 0.70) -> np.ndarray:
    """``GalleryManager._filter_quality_embeddings`` (gallery_manager.py:104-122)."""
    if len(embeddings) <= 2:
        return embeddings
    sims = np.dot(embeddings, embeddings.T)
    np.fill_diagonal(sims, 0)
    avg = np.mean(sims, axis=1)
    filtered = embeddings[avg >= min_similarity]
    if len(filtered) < 2:
        filtered = embeddings[np.argsort(avg)[-2:]]
    return filtered


def aggregate_template(embeddings: np.ndarray, method: str = "mean") -> np.ndarray:
    """``GalleryManager._aggregate_embeddings`` (gallery_manager.py:297-317)."""
    if len(embeddings) == 1:
        return embeddings[0]
    e = filter_quality_embeddings(embeddings)
    if method == "median":
        agg = np.median(e, axis=0)
    elif method == "weighted_mean":
        w = np.mean(np.dot(e, e.T), axis=1)
        w = w / np.sum(w)
        agg = np.sum(e * w[:, np.newaxis], axis=0)
    else:
        agg = np.mean(e, axis=0)
    return agg / (np.linalg.norm(agg) + 1e-8)
