"""CPU: FaceQualityFilter's pose arithmetic and gate order vs the REFERENCE module itself.

tests/golden/gate.npz holds what the reference ``FaceQualityFilter.compute_pose_angles`` /
``is_valid`` (face_recognition.py:101-158) returned on the fixed detections of
tests/_gate_inputs.py (tools/make_golden.py gate: the reference module imported with insightface
stubbed and cv2 delegated to oracle/align_ref.py).  Here the gate runs with the reference's own
blur values handed in, so everything but the device blur kernel is checked without a GPU:
metric values bitwise, their numpy types, the early exits.  tests/test_gpu_gate.py runs the whole
GPU FaceProcessor on the same inputs.
"""
import json
import os

import numpy as np
import pytest

from tests._gate_inputs import QUALITY_CONFIGS, detections


@pytest.fixture(scope="module")
def records(golden_dir):
    return json.loads(str(np.load(os.path.join(golden_dir, "gate.npz"))["records"]))


def _same(got: dict, want: dict):
    assert list(got) == list(want)  # same keys in the same (insertion) order: the same early exit
    for k, w in want.items():
        assert type(got[k]).__name__ == w["t"], (k, type(got[k]), w["t"])
        assert float(got[k]) == w["v"], (k, float(got[k]), w["v"])


def test_pose_angles_and_gate_match_reference(records):
    from facerecognitionpipeline_amd.face_recognition import FaceQualityFilter
    dets = detections()
    for rec in records:
        qf = FaceQualityFilter(**QUALITY_CONFIGS[rec["config"]])
        for d, want in zip(dets, rec["per_face"]):
            _same(qf.compute_pose_angles(d["landmarks"]), want["pose"])
            blur = want["metrics"].get("blur_score")
            ok, m = qf.is_valid(d, None, None if blur is None else blur["v"])
            assert ok == want["is_valid"]
            _same(m, want["metrics"])


def test_process_image_loader_decodes_committed_pngs(golden_dir):
    """FaceProcessor.process_image's decode (face_recognition.py:177-180: cv2.imread IMREAD_COLOR +
    COLOR_BGR2RGB): lossless PNGs decode to exactly the arrays they were written from -- RGB as is,
    8-bit gray expanded to 3 equal channels, RGBA without its alpha (tools/make_golden.py image)."""
    import hashlib
    from facerecognitionpipeline_amd.face_recognition import load_image_rgb
    want = json.loads(str(np.load(os.path.join(golden_dir, "image.npz"))["decoded_sha256"]))
    assert sorted(want) == ["image_gray.png", "image_rgb.png", "image_rgba.png"]
    for name, sha in want.items():
        a = load_image_rgb(os.path.join(golden_dir, name))
        assert a.dtype == np.uint8 and a.shape == (48, 64, 3) and a.flags["C_CONTIGUOUS"]
        assert hashlib.sha256(a.tobytes()).hexdigest() == sha, name


def test_process_image_unreadable_raises_like_reference(golden_dir, tmp_path):
    """cv2.imread returns None for a missing or undecodable file; the reference then raises
    ValueError("Could not load image: <path>") (face_recognition.py:177-179)."""
    from facerecognitionpipeline_amd.face_recognition import FaceProcessor

    class NoDetector:
        def detect(self, image):  # pragma: no cover -- never reached
            raise AssertionError("process_numpy must not run")

    fp = FaceProcessor(detector=NoDetector(), device="cpu")
    msg = str(np.load(os.path.join(golden_dir, "image.npz"))["missing_error"])
    missing = str(tmp_path / "missing.png")
    with pytest.raises(ValueError) as e:
        fp.process_image(missing)
    assert str(e.value) == msg.replace("<dir>", str(tmp_path))
    bad = tmp_path / "not_an_image.png"
    bad.write_bytes(b"not a png")
    with pytest.raises(ValueError, match="Could not load image"):
        fp.process_image(str(bad))
