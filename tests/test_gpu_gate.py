"""GPU FaceProcessor vs the REFERENCE FaceProcessor.process_numpy / FaceQualityFilter (face_recognition.py:77-216).

tests/golden/gate.npz was written by tools/make_golden.py gate: the reference module itself, with
insightface stubbed (its FaceAnalysis is never built; a fixed-detection detector stands in) and
cv2's calls delegated to the restatements in oracle/align_ref.py.  This repo's FaceProcessor runs
the same detections through the device similarity fit + warpAffine and the device blur kernel;
every result must agree exactly: which detections come back, in which order, is_valid, every
quality metric (value and numpy type), the aligned crop's bytes and its dimensionality.  Pinned:
the gate order, the pose arithmetic, the blur variance's summation order, the sort and the
return_all / [results[0]] semantics.  Unpinned: cv2's own numerics (absent here).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from tests._gate_inputs import QUALITY_CONFIGS, S, detections, frame, frame_gray

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _same(got: dict, want: dict):
    assert list(got) == list(want)
    for k, w in want.items():
        assert type(got[k]).__name__ == w["t"], (k, type(got[k]), w["t"])
        assert float(got[k]) == w["v"], (k, float(got[k]), w["v"])


class FixedDetector:
    def __init__(self, dets):
        self.dets = dets

    def detect(self, image):
        return [{"bbox": d["bbox"].copy(), "landmarks": d["landmarks"].copy(), "det_score": d["det_score"],
                 "pose": None, "age": None, "gender": None} for d in self.dets]


def test_process_numpy_matches_reference_module(golden_dir):
    from facerecognitionpipeline_amd.face_recognition import FaceProcessor
    g = np.load(os.path.join(golden_dir, "gate.npz"))
    f = frame()
    assert _sha(f) == str(g["frame_sha256"])
    dets = detections()
    frames = {"rgb": f, "gray": frame_gray(f)}
    for rec in json.loads(str(g["records"])):
        fp = FaceProcessor(output_size=S, detector=FixedDetector(dets),
                           quality_filter_config=QUALITY_CONFIGS[rec["config"]], device="cuda:0")
        img = frames[rec["frame"]]
        # per detection: the host-API align (one face) and is_valid on its crop (device blur)
        for d, want in zip(dets, rec["per_face"]):
            # the reference's own calls: a 2-D gray frame gives a 2-D crop, blur-scored as 2-D
            crop = fp.aligner.align(img, d["landmarks"])
            assert crop.ndim == img.ndim
            assert _sha(crop) == want["crop_sha256"]
            ok, m = fp.quality_filter.is_valid(d, crop)
            assert ok == want["is_valid"]
            _same(m, want["metrics"])
        for ra in (False, True):
            got = fp.process_numpy(img, return_all=ra)
            want = rec["process_numpy"][str(ra)]
            assert len(got) == len(want)
            for r, w in zip(got, want):
                assert np.array_equal(r["landmarks"], dets[w["det"]]["landmarks"])
                assert r["is_valid"] == w["is_valid"] and r["det_score"] == w["det_score"]
                _same(r["quality_metrics"], w["metrics"])
                assert _sha(r["aligned_face"]) == w["crop_sha256"] and r["aligned_face"].ndim == w["crop_ndim"]
                assert sorted(r) == w["keys"]


def test_process_image_matches_reference_module(golden_dir, tmp_path):
    """FaceProcessor.process_image (face_recognition.py:174-182) on the gate frame written as PNG vs
    the reference's process_image on the same file (tools/make_golden.py image): same detections
    back, same order, is_valid, crop bytes and blur scores; and equal to process_numpy on the
    decoded array."""
    from PIL import Image
    from facerecognitionpipeline_amd.face_recognition import FaceProcessor, load_image_rgb
    g = json.loads(str(np.load(os.path.join(golden_dir, "image.npz"))["process_image"]))
    f = frame()
    png = str(tmp_path / "gate_frame.png")
    Image.fromarray(f, "RGB").save(png)
    assert np.array_equal(load_image_rgb(png), f)
    fp = FaceProcessor(output_size=S, detector=FixedDetector(detections()), device="cuda:0")
    for ra in (False, True):
        got = fp.process_image(png, return_all=ra)
        want = g[str(ra)]
        assert len(got) == len(want)
        for r, w in zip(got, want):
            assert np.array_equal(r["landmarks"], detections()[w["det"]]["landmarks"])
            assert r["is_valid"] == w["is_valid"] and _sha(r["aligned_face"]) == w["crop_sha256"]
            assert float(r["quality_metrics"].get("blur_score", -1.0)) == w["blur"]
        same = fp.process_numpy(f, return_all=ra)
        assert [_sha(r["aligned_face"]) for r in same] == [_sha(r["aligned_face"]) for r in got]
