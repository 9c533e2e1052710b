"""Batched frame-level recognition: the serving caller of the hot path.

The reference server recognises one face per request at batch 1 with a PNG
round trip in between (``face_recognition_server.py:314-347``, ``:586-739``).
Here one call takes a frame and its detections and runs, on the GPU, with the
frame uploaded once:

    align all faces (fr_align_faces)  ->  blur scores (fr_blur_scores)  ->
    quality gate (host scalars, face_recognition.py:123-158)  ->
    embed + match every valid face in one fr_embed_match  ->  top-k per face

Detections come from any detector with the reference ``FaceDetector.detect``
contract (``face_recognition.py:31-48``); SCRFD itself is not rebuilt yet.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .face_embedder import FaceEmbedder
from .face_recognition import FaceAligner, FaceQualityFilter
from .gallery_manager import GalleryManager, _slice_len


class RecognitionPipeline:
    def __init__(self, embedder: FaceEmbedder, gallery: GalleryManager,
                 quality_filter_config: Optional[Dict] = None, similarity_threshold: float = 0.4):
        self.embedder = embedder
        self.gallery = gallery
        self.gallery.attach_handle(embedder.model)
        dev = embedder.device
        self.aligner = FaceAligner(output_size=112, device=dev)
        self.quality = FaceQualityFilter(**(quality_filter_config or {}), device=dev)
        self.similarity_threshold = similarity_threshold

    def recognize(self, frame_rgb, detections: Sequence[Dict], top_k: int = 3) -> List[Dict]:
        """frame: uint8 [H,W,3] RGB (host array or device tensor); detections: reference dicts.

        Returns one dict per detection: quality metrics, ``is_valid`` and, for valid
        faces, ``matches`` = [(student_id, name, score)] and ``recognized`` (top-1
        score >= similarity_threshold, face_recognition_server.py:983-986).
        """
        dev = self.embedder.device
        if len(detections) == 0:
            return []
        frame = frame_rgb if isinstance(frame_rgb, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(frame_rgb, dtype=np.uint8))
        frame = frame.to(dev).contiguous()
        crops = self.aligner.align_batch(frame, np.stack([np.asarray(d["landmarks"], np.float32)
                                                          for d in detections]))
        blur = self.quality.compute_blur_scores(crops) if self.quality.check_blur else None
        out, valid = [], []
        for i, d in enumerate(detections):
            ok, q = self.quality.is_valid(d, None, None if blur is None else float(blur[i]))
            out.append({"bbox": d.get("bbox"), "det_score": d["det_score"], "quality_metrics": q,
                        "is_valid": ok, "matches": [], "recognized": False})
            if ok:
                valid.append(i)
        g = self.gallery
        k = _slice_len(len(g.students), top_k)
        if not valid or k == 0:
            return out
        h = g._sync_device()
        sel = crops[torch.tensor(valid, device=dev)].contiguous()
        idx = torch.empty((len(valid), k), dtype=torch.int32, device=dev)
        score = torch.empty((len(valid), k), dtype=torch.float32, device=dev)
        h.embed_match(sel, k, idx, score)
        idx, score = idx.cpu().numpy(), score.cpu().numpy()
        for row, i in enumerate(valid):
            m = [(g._ids[j], g.students[g._ids[j]].name, float(s)) for j, s in zip(idx[row], score[row])]
            out[i]["matches"] = m
            out[i]["recognized"] = bool(m) and m[0][2] >= self.similarity_threshold
        return out
