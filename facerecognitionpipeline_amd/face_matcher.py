"""``FaceMatcher.match_single_face`` — one embed + match unit (face_matcher.py:52-58).

Only the hot-path unit is mirrored: track consensus,
visualisation and the CLI stay out of scope.  ``match_faces`` is the batched
form: every crop of a frame (or every due track) in one ``fr_embed_match``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .face_embedder import FaceEmbedder
from .gallery_manager import GalleryManager, _slice_len


class FaceMatcher:
    def __init__(self, gallery_path: Optional[str] = None, similarity_threshold: float = 0.5,
                 aggregation_method: str = "majority_vote", model_type: str = "adaface",
                 architecture: str = "ir_101", model_path: Optional[str] = None, device=None,
                 embedder: Optional[FaceEmbedder] = None, gallery: Optional[GalleryManager] = None):
        self.similarity_threshold = similarity_threshold
        self.aggregation_method = aggregation_method
        self.model_type = model_type
        self.architecture = architecture
        self.embedder = embedder or FaceEmbedder(architecture=architecture, model_path=model_path,
                                                 model_type=model_type, device=device)
        self.gallery = gallery or GalleryManager(gallery_path=gallery_path, device=self.embedder.device)
        self.gallery.attach_handle(self.embedder.model)

    def match_single_face(self, face_image: np.ndarray, top_k: int = 5) -> List[Tuple[str, str, float]]:
        embedding = self.embedder.extract_embedding(face_image, normalize=True)
        return self.gallery.search(embedding, top_k=top_k)

    def match_faces(self, face_images: Sequence[np.ndarray], top_k: int = 5) -> List[List[Tuple[str, str, float]]]:
        """Batched match_single_face: one device embed+match for all crops."""
        if len(face_images) == 0:
            return []
        rgb = self.embedder.to_device_crops(list(face_images))  # validates; resizes non-112 crops
        return self.gallery.match_resolved(len(face_images), top_k,
                                           lambda h, k, idx, score: h.embed_match(rgb, k, idx, score))
