"""Deterministic synthetic AdaFace weights, checkpoint loading, synthetic crops.

No real checkpoints exist offline, so every parity and
throughput run uses seeded weights.  Each tensor is drawn from its own
``numpy`` PCG64 stream keyed by (seed, crc32(key)), so the values do not
depend on iteration order, machine or torch version.

Checkpoint loading mirrors ``face_embedder.py:51-53``: ``torch.load(path)
['state_dict']``, keep ``model.*`` keys, strip the prefix.  It always loads
with ``weights_only=True`` (never unpickles code).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np

from .arch import schema_for

DEFAULT_WEIGHT_SEED = 20251226
CROP_SEED_GALLERY = 0xFACE0001
CROP_SEED_PROBE = 0xFACE0002
GALLERY_EXPAND_SEED = 0xFACE0003


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(key.encode())])))


def synthetic_state_dict(architecture: str, seed: int = DEFAULT_WEIGHT_SEED,
                         model_type: str = "adaface") -> "OrderedDict[str, np.ndarray]":
    """AdaFace-keyed (or, with model_type='arcface', IResNet-keyed) state dict
    (no ``model.`` prefix) of numpy arrays.

    conv / linear: U(+-1/sqrt(fan_in)); BN: gamma U(0.9,1.1), beta N(0,0.02^2),
    running_mean N(0,0.1^2), running_var U(0.5,1.5); PReLU U(0.2,0.3).
    """
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape in schema_for(architecture, model_type).items():
        r = _rng(seed, key)
        leaf = key.rsplit(".", 1)[1]
        if leaf == "num_batches_tracked":
            sd[key] = np.array(0, dtype=np.int64)
            continue
        if len(shape) >= 2 or key in ("output_layer.3.bias", "fc.bias"):
            fan_in = int(np.prod(shape[1:])) if len(shape) >= 2 else 512 * 49
            bound = 1.0 / np.sqrt(fan_in)
            v = r.uniform(-bound, bound, size=shape)
        elif ".res_layer.3." in key or key.startswith("input_layer.2.") or key.endswith("prelu.weight"):
            v = r.uniform(0.2, 0.3, size=shape)            # PReLU slope
        elif leaf == "weight":
            v = r.uniform(0.9, 1.1, size=shape)            # BN gamma
        elif leaf == "bias":
            v = r.normal(0.0, 0.02, size=shape)            # BN beta
        elif leaf == "running_mean":
            v = r.normal(0.0, 0.1, size=shape)
        elif leaf == "running_var":
            v = r.uniform(0.5, 1.5, size=shape)
        else:  # pragma: no cover - schema has no other leaves
            raise KeyError(key)
        sd[key] = v.astype(np.float32)
    return sd


def load_checkpoint_state_dict(model_path: str) -> Dict[str, np.ndarray]:
    """``torch.load(path)['state_dict']`` with ``model.`` stripped (face_embedder.py:51-53)."""
    import torch
    ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
    statedict = ckpt["state_dict"]
    return {k[6:]: v.detach().cpu().numpy() for k, v in statedict.items() if k.startswith("model.")}


def load_arcface_state_dict(model_path: str, architecture: Optional[str] = None) -> Dict[str, np.ndarray]:
    """IResNet weights for the ArcFace branch: the ``.onnx`` export the reference opens with
    onnxruntime (``face_embedder.py:64-81``), read by ``onnx_import`` (no onnx packages), or an
    ``arcface_torch`` ``backbone.pth`` (plain state dict, optionally under ``'state_dict'`` and/or
    ``module.``-prefixed)."""
    if model_path.endswith(".onnx"):
        from .onnx_import import arcface_state_dict_from_onnx
        if architecture is None:
            raise ValueError("an ArcFace .onnx model needs its architecture ('ir_50' or 'ir_101')")
        return arcface_state_dict_from_onnx(model_path, architecture)
    import torch
    ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
    sd = ckpt.get("state_dict", ckpt) if isinstance(ckpt, dict) else ckpt
    out = {}
    for k, v in sd.items():
        k = k[7:] if k.startswith("module.") else k
        out[k] = v.detach().cpu().numpy()
    return out


def save_checkpoint(state_dict: Dict[str, np.ndarray], path: str) -> None:
    """Write a reference-format checkpoint ``{'state_dict': {'model.'+k: tensor}}``."""
    import torch
    torch.save({"state_dict": {"model." + k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}}, path)


def synthetic_crops(n: int, seed: int = CROP_SEED_GALLERY, size: int = 112) -> np.ndarray:
    """n uint8 RGB HWC crops, U{0..255} (SURVEY.md §8(d) gallery-base crops)."""
    r = np.random.Generator(np.random.PCG64(seed))
    return r.integers(0, 256, size=(n, size, size, 3), dtype=np.uint8)


def probe_crops(base: np.ndarray, n: int, sigma: float = 12.0, seed: int = CROP_SEED_PROBE) -> np.ndarray:
    """Probes ``clip(base[i mod G] + N(0, sigma^2))`` — near-duplicates with margins (§8(d))."""
    r = np.random.Generator(np.random.PCG64(seed))
    idx = np.arange(n) % base.shape[0]
    noise = r.normal(0.0, sigma, size=(n,) + base.shape[1:])
    return np.clip(np.rint(base[idx].astype(np.float64) + noise), 0, 255).astype(np.uint8)


def expand_gallery(emb: np.ndarray, g_total: int, scale: float = 0.0214,
                   seed: int = GALLERY_EXPAND_SEED) -> np.ndarray:
    """Grow a gallery to ``g_total`` rows: ``normalize(e[j mod G0] + scale*z)`` (§8(d), G=100k)."""
    g0 = emb.shape[0]
    if g_total <= g0:
        return emb[:g_total].astype(np.float32)
    r = np.random.Generator(np.random.PCG64(seed))
    extra = g_total - g0
    src = emb[np.arange(extra) % g0].astype(np.float32)
    z = r.standard_normal(size=src.shape, dtype=np.float32)
    rows = src + np.float32(scale) * z
    rows /= np.linalg.norm(rows, axis=1, keepdims=True)
    return np.concatenate([emb.astype(np.float32), rows.astype(np.float32)], axis=0)
