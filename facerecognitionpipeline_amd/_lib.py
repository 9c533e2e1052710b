"""ctypes binding of libfrhip.so (the C ABI of include/frhip.h).

The library is loaded AFTER ``import torch`` so that it binds to the same HIP
runtime instance (SONAME libamdhip64.so.7) PyTorch-ROCm already loaded: device
pointers and streams are then shared with torch tensors.  There is no CPU
fallback anywhere: if the library is missing or no GPU is present, every
entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

# FRHIP_LIB: another build of the library (tools' A/B of two builds in one tree); default: in-tree
LIB_PATH = os.environ.get("FRHIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfrhip.so")

FR_OK = 0
FR_ERR_INVALID_ARGUMENT = -1
FR_ERR_MISSING_PARAM = -2
FR_ERR_HIP = -3
FR_ERR_STATE = -4
FR_ERR_UNSUPPORTED = -5

_P = ctypes.c_void_p
_I = ctypes.c_int
_SIGNATURES = {
    "fr_create": (_I, [ctypes.c_char_p, ctypes.c_char_p, _I, _I, ctypes.POINTER(_P)]),
    "fr_destroy": (_I, [_P]),
    "fr_set_param": (_I, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    "fr_finalize": (_I, [_P]),
    "fr_embed": (_I, [_P, _P, _I, _I, _I, _P, _I, _P]),
    "fr_embed_host": (_I, [_P, _P, _I, _I, _I, _P, _I]),
    "fr_resize_crops": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "fr_gallery_set": (_I, [_P, _P, _I, _I, _I, _P]),
    "fr_gallery_size": (_I, [_P, ctypes.POINTER(_I)]),
    "fr_gallery_write_rows": (_I, [_P, _I, _I, _P, _I, _P]),
    "fr_gallery_delete_rows": (_I, [_P, _I, _I, _P]),
    "fr_gallery_read": (_I, [_P, _I, _I, _P, _I, _P]),
    "fr_build_templates": (_I, [_P, _P, _P, _I, _I, ctypes.c_float, _P, _P, _P]),
    "fr_match_topk": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "fr_match_topk_host": (_I, [_P, _P, _I, _I, _P, _P]),
    "fr_embed_match": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "fr_align_faces": (_I, [_P, _P, _I, _I, _P, _I, _I, _P, _P, _P]),
    "fr_warp_affine": (_I, [_P, _P, _I, _I, _P, _I, _I, _P, _P]),
    "fr_blur_scores": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "fr_detect": (_I, [_P, _P, _I, _I, _I, ctypes.c_float, _I, _P, _P, _P]),
    "fr_set_precision": (_I, [_P, _I]),
    "fr_set_conv_algorithm": (_I, [_P, _I]),
    "fr_set_graph_batch": (_I, [_P, _I]),
    "fr_set_lanes": (_I, [_P, _I, _I]),
    "fr_graph_count": (_I, [_P, ctypes.POINTER(ctypes.c_int)]),
    "fr_get_lanes": (_I, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "fr_profile_enable": (_I, [_P, _I]),
    "fr_profile_kernel": (_I, [_P, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "fr_profile_read": (_I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "fr_last_error": (ctypes.c_char_p, [_P]),
    "fr_version": (ctypes.c_char_p, []),
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


class FrHipError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libfrhip.so once; raise loudly if it is not built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise FrHipError(f"{LIB_PATH} is not built: run `python -m facerecognitionpipeline_amd.build` "
                                 "(the HIP path has no CPU fallback)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int, handle=None) -> None:
    """Map a status code to the reference's exception types (SURVEY.md §8(b) Errors)."""
    if rc == FR_OK:
        return
    msg = load().fr_last_error(handle)
    msg = msg.decode() if msg else f"frhip error {rc}"
    if rc == FR_ERR_INVALID_ARGUMENT:
        raise ValueError(msg)
    if rc == FR_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise FrHipError(msg)


def ptr(t) -> Optional[int]:
    """Raw data pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class Handle:
    """Owns one ``fr_handle``: a model (after ``load_state_dict``) and/or a gallery."""

    def __init__(self, architecture: str, model_type: str, device: torch.device, max_batch: int = 256):
        if device.type != "cuda":
            raise RuntimeError("facerecognitionpipeline_amd runs on a HIP device only (no CPU fallback); "
                               f"got device={device}")
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device available: the MI355X hot path has no CPU fallback")
        self.device = device
        self._lib = load()
        h = _P()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.gallery_tag = None  # (owner, version) of the rows in HBM; see GalleryManager._sync_device
        check(self._lib.fr_create(architecture.encode(), model_type.encode(), idx, int(max_batch), ctypes.byref(h)))
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None) and self._lib is not None:
            self._lib.fr_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # -- model -------------------------------------------------------------
    def load_state_dict(self, state_dict) -> None:
        import numpy as np
        for k, v in state_dict.items():
            a = np.ascontiguousarray(np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v),
                                     dtype=np.float32)
            check(self._lib.fr_set_param(self.h, k.encode(), a.ctypes.data, a.size), self.h)
        check(self._lib.fr_finalize(self.h), self.h)

    def embed(self, rgb: torch.Tensor, out: torch.Tensor, normalize: bool = True) -> None:
        n = rgb.shape[0]
        check(self._lib.fr_embed(self.h, ptr(rgb), n, rgb.shape[1], rgb.shape[2], ptr(out), int(normalize),
                                 stream_of(self.device)), self.h)

    def resize_crops(self, src: torch.Tensor, out: torch.Tensor) -> None:
        """cv2.resize(INTER_LINEAR) of uint8 [n,H,W,3] device crops into out [n,112,112,3]."""
        check(self._lib.fr_resize_crops(self.h, ptr(src), src.shape[0], src.shape[1], src.shape[2], ptr(out),
                                        stream_of(self.device)), self.h)

    # -- gallery -----------------------------------------------------------
    def gallery_set(self, E: torch.Tensor, tag=None) -> None:
        G = E.shape[0] if E.numel() else 0
        D = E.shape[1] if E.dim() == 2 else 512
        check(self._lib.fr_gallery_set(self.h, ptr(E) if G else None, G, D, 1, stream_of(self.device)), self.h)
        self.gallery_tag = tag

    def gallery_replace(self, E: torch.Tensor) -> None:
        """Replace the rows with a device [G,512] matrix built from the current ones (a delta
        replay's compaction; the gallery tag is left to the caller)."""
        E = E.contiguous()
        G = E.shape[0]
        check(self._lib.fr_gallery_set(self.h, ptr(E) if G else None, G, 512, 1, stream_of(self.device)), self.h)

    def gallery_size(self) -> int:
        g = ctypes.c_int()
        check(self._lib.fr_gallery_size(self.h, ctypes.byref(g)), self.h)
        return g.value

    def gallery_write_rows(self, row0: int, E: torch.Tensor) -> None:
        """Rows [row0, row0 + len(E)) := E (device f32 [n,512]); may extend the gallery."""
        E = E.to(device=self.device, dtype=torch.float32).contiguous()
        check(self._lib.fr_gallery_write_rows(self.h, int(row0), E.shape[0], ptr(E), 1, stream_of(self.device)),
              self.h)

    def gallery_delete_rows(self, row0: int, n: int = 1) -> None:
        check(self._lib.fr_gallery_delete_rows(self.h, int(row0), int(n), stream_of(self.device)), self.h)

    def gallery_read(self) -> torch.Tensor:
        G = self.gallery_size()
        out = torch.empty((G, 512), dtype=torch.float32, device=self.device)
        check(self._lib.fr_gallery_read(self.h, 0, G, ptr(out) if G else None, 1, stream_of(self.device)), self.h)
        return out

    def build_templates(self, emb: torch.Tensor, offsets, method: str = "mean", min_similarity: float = 0.70):
        """Templates of len(offsets)-1 students whose samples are CSR rows of ``emb`` [total,512]
        -> (templates f32 [S,512], kept int32 [S]) on the device."""
        import numpy as np
        methods = {"mean": 0, "median": 1, "weighted_mean": 2}
        m = methods.get(method, 0)  # the reference falls back to mean for unknown methods
        off = np.ascontiguousarray(offsets, dtype=np.int32)
        S = off.shape[0] - 1
        emb = emb.to(device=self.device, dtype=torch.float32).contiguous()
        tpl = torch.empty((max(S, 0), 512), dtype=torch.float32, device=self.device)
        kept = torch.empty((max(S, 0),), dtype=torch.int32, device=self.device)
        check(self._lib.fr_build_templates(self.h, ptr(emb), off.ctypes.data, S, m, float(min_similarity), ptr(tpl),
                                           ptr(kept), stream_of(self.device)), self.h)
        return tpl, kept

    def match(self, Q: torch.Tensor, k: int, idx: torch.Tensor, score: torch.Tensor) -> None:
        check(self._lib.fr_match_topk(self.h, ptr(Q), Q.shape[0], int(k), ptr(idx), ptr(score),
                                      stream_of(self.device)), self.h)

    def embed_match(self, rgb: torch.Tensor, k: int, idx: torch.Tensor, score: torch.Tensor,
                    emb: Optional[torch.Tensor] = None) -> None:
        check(self._lib.fr_embed_match(self.h, ptr(rgb), rgb.shape[0], int(k), ptr(idx), ptr(score), ptr(emb),
                                       stream_of(self.device)), self.h)

    # -- alignment / quality ----------------------------------------------
    def align_faces(self, frame: torch.Tensor, landmarks, out_size: int, out: torch.Tensor):
        """frame: uint8 [H,W,3] on device; landmarks: host float32 [n,5,2] -> out [n,S,S,3]; returns tforms."""
        import numpy as np
        lm = np.ascontiguousarray(landmarks, dtype=np.float32)
        n = lm.shape[0]
        tf = np.empty((n, 2, 3), dtype=np.float64)
        check(self._lib.fr_align_faces(self.h, ptr(frame), frame.shape[0], frame.shape[1], lm.ctypes.data, n,
                                       int(out_size), ptr(out), tf.ctypes.data, stream_of(self.device)), self.h)
        return tf

    def warp_affine(self, frame: torch.Tensor, tforms, out_size: int, out: torch.Tensor) -> None:
        import numpy as np
        tf = np.ascontiguousarray(tforms, dtype=np.float64)
        check(self._lib.fr_warp_affine(self.h, ptr(frame), frame.shape[0], frame.shape[1], tf.ctypes.data,
                                       tf.shape[0], int(out_size), ptr(out), stream_of(self.device)), self.h)

    def blur_scores(self, crops: torch.Tensor):
        """uint8 [n,H,W] (gray) or [n,H,W,C] (C = 3 / 4, RGB(A)) on the device -> float64 [n]."""
        import numpy as np
        if crops.dtype != torch.uint8 or crops.dim() not in (3, 4):
            raise ValueError("expected uint8 [n,H,W] or [n,H,W,C] images")
        n = crops.shape[0]
        c = 1 if crops.dim() == 3 else crops.shape[3]
        out = np.empty(n, dtype=np.float64)
        check(self._lib.fr_blur_scores(self.h, ptr(crops), n, crops.shape[1], crops.shape[2], c, out.ctypes.data,
                                       stream_of(self.device)), self.h)
        return out

    # -- detector (arch "scrfd_10g") ---------------------------------------
    def detect(self, frames: torch.Tensor, det_thresh: float = 0.5, max_faces: int = 256):
        """frames: uint8 [n,H,W,3] RGB on the device -> (dets f32 [n,max_faces,15], counts int32 [n]);
        row i < min(counts[f], max_faces) of frame f = x1 y1 x2 y2 score, 5 x (x, y)."""
        import numpy as np
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
            raise ValueError("expected uint8 [n,H,W,3] RGB frames")
        frames = frames.to(self.device).contiguous()
        n = frames.shape[0]
        dets = np.zeros((n, max_faces, 15), dtype=np.float32)
        counts = np.zeros(n, dtype=np.int32)
        check(self._lib.fr_detect(self.h, ptr(frames), n, frames.shape[1], frames.shape[2], float(det_thresh),
                                  int(max_faces), dets.ctypes.data, counts.ctypes.data, stream_of(self.device)),
              self.h)
        return dets, counts

    def set_precision(self, mode: str) -> None:
        modes = {"fp32": 0, "f32": 0, "bf16x3": 1}
        if mode not in modes:
            raise ValueError(f"precision must be one of {sorted(modes)}")
        check(self._lib.fr_set_precision(self.h, modes[mode]), self.h)

    def set_conv_algorithm(self, algo: str) -> None:
        algos = {"direct": 0, "winograd": 1, "winograd4": 2}
        if algo not in algos:
            raise ValueError(f"conv_algorithm must be one of {sorted(algos)}")
        check(self._lib.fr_set_conv_algorithm(self.h, algos[algo]), self.h)

    def set_graph_batch(self, max_n: int) -> None:
        """Replay forwards of n <= max_n crops as captured hipGraphs (0 disables)."""
        check(self._lib.fr_set_graph_batch(self.h, int(max_n)), self.h)

    def set_lanes(self, min_n: int, max_lanes: int = 2) -> None:
        """Run a forward of n crops as min(max_lanes, n // min_n) concurrent parts (0: one lane)."""
        check(self._lib.fr_set_lanes(self.h, int(min_n), int(max_lanes)), self.h)

    def get_lanes(self) -> dict:
        """The lane setting in force; ``fell_back`` is True when a failed workspace allocation
        turned lanes off (until the next ``set_lanes``)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.fr_get_lanes(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), self.h)
        return {"min_n": a.value, "max_lanes": b.value, "fell_back": bool(c.value)}

    def graph_count(self) -> int:
        c = ctypes.c_int()
        check(self._lib.fr_graph_count(self.h, ctypes.byref(c)), self.h)
        return c.value

    # -- profiling ---------------------------------------------------------
    def profile_enable(self, on: bool = True) -> None:
        check(self._lib.fr_profile_enable(self.h, int(on)), self.h)

    def profile_read(self) -> dict:
        cms, cfl, tms = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        cn = ctypes.c_int64()
        check(self._lib.fr_profile_read(self.h, ctypes.byref(cms), ctypes.byref(cfl), ctypes.byref(cn),
                                        ctypes.byref(tms)), self.h)
        out = {"conv_ms": cms.value, "conv_flop": cfl.value, "conv_launches": cn.value, "total_ms": tms.value}
        for kind, name in ((0, "other"), (1, "direct"), (2, "winograd")):
            ms, fl, ex = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            n = ctypes.c_int64()
            check(self._lib.fr_profile_kernel(self.h, kind, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(ex),
                                              ctypes.byref(n)), self.h)
            out[name] = {"ms": ms.value, "flop": fl.value, "exec_flop": ex.value, "launches": n.value}
        return out
