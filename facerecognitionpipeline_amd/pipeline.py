"""Batched frame-level recognition: the serving caller of the hot path.

The reference server recognises one face per request at batch 1 with a PNG
round trip in between (``face_recognition_server.py:314-347``, ``:586-739``).
Here one call takes a frame and its detections and runs, on the GPU, with the
frame uploaded once:

    align all faces (fr_align_faces)  ->  blur scores (fr_blur_scores)  ->
    quality gate (host scalars, face_recognition.py:123-158)  ->
    embed + match every valid face in one fr_embed_match  ->  top-k per face

Detections come from any detector with the reference ``FaceDetector.detect``
contract (``face_recognition.py:31-48``), the GPU SCRFD ``FaceDetector`` included.
``MatchBatcher`` batches concurrent single-face requests the same way.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .face_embedder import FaceEmbedder, as_uint8_crop
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
        if not valid:
            return out
        sel = crops[torch.tensor(valid, device=dev)].contiguous()
        res = self.gallery.match_resolved(len(valid), top_k, lambda h, k, idx, score: h.embed_match(sel, k, idx, score))
        for row, i in enumerate(valid):
            m = res[row]
            out[i]["matches"] = m
            out[i]["recognized"] = bool(m) and m[0][2] >= self.similarity_threshold
        return out


class MatchBatcher:
    """Dynamic batching of concurrent ``match_single_face`` calls.

    The reference server handles each request on its own Flask thread
    (``threaded=True``, ``face_recognition_server.py:1102``) and every one of them
    runs a batch-1 embed + search (``:321-323`` -> ``face_matcher.py:52-58``).  Here
    those threads call :meth:`match_single_face` (or :meth:`submit`) and one worker
    thread gathers whatever is pending -- up to ``max_batch`` crops, waiting at most
    ``max_wait_ms`` after the first -- into ONE ``FaceMatcher.match_faces`` call, i.e.
    one ``fr_embed_match`` (a replayed hipGraph when the batch is small).  Each
    caller gets what ``match_single_face`` would return, to fp32 summation order: the
    forward is batch-invariant within 1e-6 per embedding element (the stream-K schedule
    cuts a batch-size-dependent set of tiles along K), and the top-k kernel is exact
    with the same tie order, so the first ``top_k`` of a larger k are the top-``top_k``.

    Errors keep the reference behaviour per request: a crop of the wrong shape raises
    ``ValueError`` in the calling thread before it is queued; a failure of the batched
    call is raised in every caller of that batch.
    """

    def __init__(self, matcher, max_batch: int = 64, max_wait_ms: float = 2.0):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.matcher = matcher
        self.max_batch = int(max_batch)
        self.max_wait = max(0.0, float(max_wait_ms)) / 1000.0
        self.batches: List[int] = []  # size of every batch run (for tests and monitoring)
        self._q: "queue.Queue[Optional[Tuple[np.ndarray, int, Future]]]" = queue.Queue()
        self._closed = False
        self._lock = threading.Lock()
        self._worker = threading.Thread(target=self._run, name="frhip-match-batcher", daemon=True)
        self._worker.start()

    def submit(self, face_image: np.ndarray, top_k: int = 5) -> Future:
        self.matcher.embedder._check_shape(face_image)
        fut: Future = Future()
        item = (np.ascontiguousarray(as_uint8_crop(face_image)), int(top_k), fut)
        with self._lock:
            if self._closed:
                raise RuntimeError("MatchBatcher is closed")
            self._q.put(item)
        return fut

    def match_single_face(self, face_image: np.ndarray, top_k: int = 5) -> List[Tuple[str, str, float]]:
        return self.submit(face_image, top_k).result()

    def close(self) -> None:
        """Finish every queued request, then stop the worker."""
        with self._lock:
            if self._closed:
                return
            self._closed = True
            self._q.put(None)
        self._worker.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _run(self) -> None:
        stop = False
        while not stop:
            item = self._q.get()
            if item is None:
                break
            batch = [item]
            deadline = time.monotonic() + self.max_wait
            while len(batch) < self.max_batch:
                try:
                    nxt = self._q.get(timeout=max(0.0, deadline - time.monotonic()))
                except queue.Empty:
                    break
                if nxt is None:
                    stop = True
                    break
                batch.append(nxt)
            self._serve(batch)

    def _serve(self, batch) -> None:
        self.batches.append(len(batch))
        try:
            n_rows = len(self.matcher.gallery.students)
            ks = [_slice_len(n_rows, k) for _, k, _ in batch]
            kmax = max(ks)
            if kmax == 0:
                res = [[] for _ in batch]
            else:
                res = self.matcher.match_faces([f for f, _, _ in batch], top_k=kmax)
        except BaseException as e:  # every caller of this batch sees the failure
            for _, _, fut in batch:
                fut.set_exception(e)
            return
        for (_, _, fut), r, k in zip(batch, res, ks):
            fut.set_result(r[:k])
