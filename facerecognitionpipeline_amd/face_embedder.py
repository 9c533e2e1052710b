"""Drop-in ``FaceEmbedder`` backed by the gfx950 HIP path (libfrhip).

Mirrors the reference class ``face_embedder.FaceEmbedder``
(``face_embedder.py:26-225``): same constructor arguments, method names,
return types and exceptions.  The forward runs entirely on the GPU: the
uint8 crops go to HBM once, the stem kernel fuses the BGR flip and the
``(x/255-0.5)/0.5`` normalisation, and the embedding comes back already
L2-normalised the way the reference's ``normalize=True`` path leaves it.

Crops of any other size go through the device restatement of the reference's
``cv2.resize(..., (112, 112), INTER_LINEAR)`` (face_embedder.py:94-96; OpenCV's
fixed-point bilinear, parity vs cv2 itself unpinned: cv2 is absent here).

Differences (documented in DESIGN.md): ``model_type='arcface'`` runs the same kernels with the insightface
IResNet weights, read from the ``.onnx`` file the reference opens with onnxruntime
(``onnx_import``: the graph's weights, no onnxruntime) or from an ``arcface_torch``
state dict, and ``device`` must be a HIP device — there is no CPU fallback.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from .arch import INPUT_SIZE, block_specs
from .weights import load_arcface_state_dict, load_checkpoint_state_dict, synthetic_state_dict

SCRIPT_DIR = Path(__file__).resolve().parent

# Same registry layout as face_embedder.py:16-24.
ADAFACE_MODELS = {
    "ir_50": str(SCRIPT_DIR / "pretrained" / "adaface_ir50_ms1mv2.ckpt"),
    "ir_101": str(SCRIPT_DIR / "pretrained" / "adaface_ir101_ms1mv3.ckpt"),
}
ARCFACE_MODELS = {
    "ir_50": str(SCRIPT_DIR / "pretrained" / "arcface_ir50_ms1mv3.onnx"),
    "ir_101": str(SCRIPT_DIR / "pretrained" / "arcface_ir101_ms1mv3.onnx"),
}

SYNTHETIC = "synthetic"  # model_path value selecting the seeded weights of weights.py


def _as_device(device) -> torch.device:
    if device is None:
        return torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
    return torch.device(device)


class FaceEmbedder:
    def __init__(self, architecture: str = "ir_101", model_path: Optional[str] = None,
                 model_type: str = "adaface", device=None, max_batch: int = 256,
                 state_dict=None, weight_seed: Optional[int] = None, precision: str = "fp32",
                 conv_algorithm: str = "winograd4", graph_batch: int = 16, lanes_min: Optional[int] = None):
        self.device = _as_device(device)
        self.model_type = model_type
        self.architecture = architecture
        if model_type not in ("adaface", "arcface"):
            raise ValueError(f"Unknown model_type: {model_type}. Must be 'adaface' or 'arcface'")
        registry = ADAFACE_MODELS if model_type == "adaface" else ARCFACE_MODELS
        if architecture not in registry:
            raise ValueError(f"Unknown architecture: {architecture}. "
                             f"Available: {list(registry.keys())}")
        if state_dict is None:
            if model_path == SYNTHETIC or weight_seed is not None:
                kw = {} if weight_seed is None else {"seed": weight_seed}
                state_dict = synthetic_state_dict(architecture, model_type=model_type, **kw)
            else:
                if model_path is None:
                    model_path = registry[architecture]
                if not os.path.exists(model_path):
                    raise FileNotFoundError(f"{'AdaFace checkpoint' if model_type == 'adaface' else 'ONNX model'} "
                                            f"not found at: {model_path}")
                state_dict = (load_checkpoint_state_dict(model_path) if model_type == "adaface"
                              else load_arcface_state_dict(model_path, architecture))
        block_specs(architecture)
        self.model = _lib.Handle(architecture, model_type, self.device, max_batch)
        self.model.load_state_dict(state_dict)
        self.precision = precision
        self.model.set_precision(precision)
        self.conv_algorithm = conv_algorithm
        self.model.set_conv_algorithm(conv_algorithm)
        # serving-sized forwards (n <= graph_batch: batch 1, one frame's faces) replay a
        # captured hipGraph instead of ~100 individual launches (bit-identical results)
        self.graph_batch = min(int(graph_batch), max_batch)
        self.model.set_graph_batch(self.graph_batch)
        # a forward of n >= 2 * lanes_min crops runs as two concurrent halves (fr_set_lanes;
        # None keeps the library default, 0 = one lane)
        if lanes_min is not None:
            self.model.set_lanes(lanes_min)
        self.input_size = INPUT_SIZE
        # face_embedder.py:60-61 (AdaFace) and :86-87 (ArcFace)
        self.mean, self.std = (0.5, 0.5) if model_type == "adaface" else (127.5, 127.5)
        self.is_onnx = False

    # -- reference API -------------------------------------------------------
    def preprocess(self, face_image: np.ndarray):
        """Host input exactly as face_embedder.py:93-110 builds it (for API parity; the
        GPU path does the same arithmetic inside the resize and stem kernels): a float32
        torch tensor for AdaFace, a float32 numpy array for ArcFace."""
        self._check_shape(face_image)
        if face_image.shape[:2] != self.input_size:
            x = torch.from_numpy(np.ascontiguousarray(self._as_u8(face_image))[None]).to(self.device)
            out = torch.empty((1,) + self.input_size + (3,), dtype=torch.uint8, device=self.device)
            self.model.resize_crops(x, out)
            face_image = out[0].cpu().numpy()
        bgr = face_image[:, :, ::-1]
        if self.model_type == "arcface":
            bgr = (bgr - self.mean) / self.std
            return np.expand_dims(bgr.transpose(2, 0, 1), axis=0).astype(np.float32)
        bgr = (bgr / 255.0 - self.mean) / self.std
        return torch.from_numpy(bgr.transpose(2, 0, 1).copy()).float().unsqueeze(0)

    def extract_embedding(self, face_image: np.ndarray, normalize: bool = True) -> np.ndarray:
        return self.extract_embeddings_batch([face_image], normalize=normalize)[0]

    def extract_embeddings_batch(self, face_images: List[np.ndarray], normalize: bool = True,
                                 batch_size: int = 32) -> np.ndarray:
        """``batch_size`` is accepted for signature parity; the device forward is
        batch-invariant and chunks by the handle's max_batch instead."""
        if len(face_images) == 0:
            return np.array([])
        out = self.embed_tensor(self.to_device_crops(face_images), normalize=normalize)
        return out.cpu().numpy()

    def to_device_crops(self, face_images: List[np.ndarray]) -> torch.Tensor:
        """Host HxWx3 crops -> uint8 [N,112,112,3] on the device: 112x112 crops uploaded as they
        are, any other size uploaded and resized there (cv2.resize INTER_LINEAR restatement,
        face_embedder.py:94-96), one launch per distinct size."""
        for f in face_images:
            self._check_shape(f)
        if all(f.shape[:2] == self.input_size for f in face_images):
            host = np.ascontiguousarray(np.stack([self._as_u8(f) for f in face_images]))
            rgb = torch.from_numpy(host).to(self.device, non_blocking=False)
        else:
            # cv2.resize branch (face_embedder.py:94-96) on the device, one launch per crop size
            rgb = torch.empty((len(face_images),) + self.input_size + (3,), dtype=torch.uint8, device=self.device)
            by_size = {}
            for i, f in enumerate(face_images):
                by_size.setdefault(f.shape[:2], []).append(i)
            for size, rows in by_size.items():
                src = torch.from_numpy(np.ascontiguousarray(np.stack([self._as_u8(face_images[i]) for i in rows])))
                src = src.to(self.device)
                if size == self.input_size:
                    rgb[rows] = src
                else:
                    tmp = torch.empty((len(rows),) + self.input_size + (3,), dtype=torch.uint8, device=self.device)
                    self.model.resize_crops(src, tmp)
                    rgb[rows] = tmp
        return rgb

    def compute_similarity(self, embedding1: np.ndarray, embedding2: np.ndarray) -> float:
        e1 = embedding1 / (np.linalg.norm(embedding1) + 1e-8)
        e2 = embedding2 / (np.linalg.norm(embedding2) + 1e-8)
        return np.dot(e1, e2)

    def compute_similarity_batch(self, embedding: np.ndarray, gallery_embeddings: np.ndarray) -> np.ndarray:
        e = embedding / (np.linalg.norm(embedding) + 1e-8)
        g = gallery_embeddings / (np.linalg.norm(gallery_embeddings, axis=1, keepdims=True) + 1e-8)
        return np.dot(g, e)

    def aggregate_embeddings(self, embeddings: np.ndarray, method: str = "mean") -> np.ndarray:
        if len(embeddings) == 0:
            raise ValueError("Cannot aggregate empty embeddings")
        if len(embeddings) == 1:
            return embeddings[0]
        if method == "mean":
            agg = np.mean(embeddings, axis=0)
        elif method == "median":
            agg = np.median(embeddings, axis=0)
        elif method == "weighted_mean":
            w = np.mean(np.dot(embeddings, embeddings.T), axis=1)
            agg = np.sum(embeddings * (w / np.sum(w))[:, np.newaxis], axis=0)
        else:
            raise ValueError(f"Unknown aggregation method: {method}")
        return agg / (np.linalg.norm(agg) + 1e-8)

    # -- device-resident API (no host round trip) ----------------------------
    def embed_tensor(self, rgb: torch.Tensor, normalize: bool = True,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 [N,112,112,3] RGB on the handle's device -> float32 [N,512] on device."""
        if rgb.device != self.device or rgb.dtype != torch.uint8 or rgb.dim() != 4 or rgb.shape[3] != 3:
            raise ValueError("expected a uint8 [N,112,112,3] tensor on " + str(self.device))
        rgb = rgb.contiguous()
        if out is None:
            out = torch.empty((rgb.shape[0], 512), dtype=torch.float32, device=self.device)
        self.model.embed(rgb, out, normalize)
        return out

    def _check_shape(self, face_image: np.ndarray) -> None:
        if face_image.ndim != 3 or face_image.shape[2] != 3:
            raise ValueError(f"expected an HxWx3 RGB crop, got shape {face_image.shape}")
        if min(face_image.shape[:2]) < 1 or max(face_image.shape[:2]) > 8192:
            raise ValueError(f"crop size {face_image.shape[:2]} out of range [1, 8192]")

    _as_u8 = staticmethod(lambda face_image: as_uint8_crop(face_image))


def as_uint8_crop(face_image: np.ndarray, input_size=INPUT_SIZE) -> np.ndarray:
    """The device path computes on uint8 pixels (a 256-entry LUT of the reference's float64
    normalisation, face_embedder.py:99-100).  A non-uint8 crop is accepted only when it is
    already ``input_size`` (112x112) and its values are integers in [0, 255]: it then converts
    exactly and the result is the reference's.  Any other size is refused: the reference
    resizes a float or 16-bit crop in that dtype (cv2.resize on the original array,
    face_embedder.py:94-96), with no 8-bit fixed-point rounding, which the uint8 device resize
    does not restate.  Fractional or out-of-range values are refused too (the LUT covers bytes)."""
    a = np.asarray(face_image)
    if a.dtype == np.uint8:
        return a
    if tuple(a.shape[:2]) != tuple(input_size):
        raise ValueError(f"non-uint8 crops ({a.dtype}) must already be {input_size[0]}x{input_size[1]}: the reference "
                         f"resizes them in {a.dtype} (cv2.resize), which the uint8 device resize does not restate")
    if a.dtype.kind in "biuf" and np.all(np.isfinite(a)) and np.all((a >= 0) & (a <= 255) & (a == np.floor(a))):
        return a.astype(np.uint8)
    raise ValueError(f"crops must be uint8 (or integer-valued in [0, 255]); got {a.dtype} with other values")
