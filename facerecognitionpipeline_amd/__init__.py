"""MI355X-native (gfx950) face embed + match hot path.

Drop-in for the reference's ``FaceEmbedder`` / ``GalleryManager.search`` /
``FaceMatcher.match_single_face`` seams, backed by hand-written HIP kernels in
``libfrhip.so`` (C ABI: ``include/frhip.h``).  Import is cheap: the GPU
library loads on first use and raises if it is missing — there is no CPU
fallback.
"""
from .arch import block_specs, flop_per_face, state_dict_schema  # noqa: F401

__all__ = ["FaceEmbedder", "GalleryManager", "FaceMatcher", "block_specs", "flop_per_face", "state_dict_schema"]


def __getattr__(name):
    if name == "FaceEmbedder":
        from .face_embedder import FaceEmbedder
        return FaceEmbedder
    if name == "GalleryManager":
        from .gallery_manager import GalleryManager
        return GalleryManager
    if name == "FaceMatcher":
        from .face_matcher import FaceMatcher
        return FaceMatcher
    raise AttributeError(name)
