"""Seeded inputs of the quality-gate / ``process_numpy`` fixture (``tests/golden/gate.npz``).

``tools/make_golden.py gate`` runs the REFERENCE ``FaceQualityFilter`` and
``FaceProcessor.process_numpy`` (face_recognition.py:77-216) on these inputs;
``tests/test_gpu_gate.py`` runs this repo's GPU ``FaceProcessor`` on the same
ones.  The frame mixes smooth regions (Laplacian variance far below the
default blur threshold of 100), noise patches of graded amplitude (variances
around the threshold) and full-range noise; the detections straddle every gate
of ``is_valid`` (det score, face size, yaw / pitch / roll, blur) including the
exact det-score and face-size thresholds.
"""
import numpy as np

SEED = 0xFACE0A7E
H, W = 540, 960
S = 112


def frame() -> np.ndarray:
    r = np.random.Generator(np.random.PCG64(SEED))
    yy, xx = np.mgrid[0:H, 0:W]
    f = np.stack([(yy // 3 + xx // 5) % 256, (xx // 4 + 30) % 256, (yy // 2 + 60) % 256], -1).astype(np.int64)
    # graded noise patches: amplitude a -> Laplacian variance ~ 20 a^2 / 3 after gray conversion
    patches = [(20, 20, 200, 200, 128), (20, 260, 180, 180, 2), (20, 480, 180, 180, 7), (20, 700, 180, 220, 8),
               (260, 20, 200, 200, 9), (260, 260, 220, 220, 10), (300, 520, 200, 400, 128)]
    for y0, x0, h, w, a in patches:
        base = 128 if a < 128 else 0
        f[y0:y0 + h, x0:x0 + w] = base + r.integers(-a if a < 128 else 0, a + 1 if a < 128 else 256, (h, w, 3))
    return np.clip(f, 0, 255).astype(np.uint8)


def frame_gray(f: np.ndarray) -> np.ndarray:
    """The grayscale variant of the frame (a 2-D uint8 image, cv2's RGB2GRAY fixed point)."""
    x = f.astype(np.int64)
    return ((x[..., 0] * 4899 + x[..., 1] * 9617 + x[..., 2] * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def _landmarks(cx, cy, scale, roll=0.0, nose_dx=0.0, nose_dy=0.0):
    t = np.array([[0.34, 0.46], [0.66, 0.46], [0.50, 0.61], [0.37, 0.74], [0.63, 0.74]]) * S - S / 2
    t[2] += (nose_dx, nose_dy)
    c, s = np.cos(roll), np.sin(roll)
    p = t @ (scale * np.array([[c, -s], [s, c]])).T + (cx, cy)
    return p.astype(np.float32)


def detections():
    """Fixed detections in the reference detector's dict format (face_recognition.py:39-46):
    bbox int32 x1 y1 x2 y2, landmarks float32 (5, 2), det_score float."""
    r = np.random.Generator(np.random.PCG64(SEED + 1))
    specs = [  # (cx, cy, scale, roll, nose_dx, nose_dy, det_score, bbox_size or None)
        (120, 120, 1.2, 0.05, 0.0, 0.0, 0.93, None),     # noise: valid
        (350, 110, 1.1, -0.1, 1.0, 0.0, 0.88, None),     # amplitude 2: blur below 100
        (570, 110, 1.1, 0.0, 0.0, 1.0, 0.91, None),      # amplitude 7
        (810, 110, 1.1, 0.2, -2.0, 0.0, 0.85, None),     # amplitude 8
        (120, 360, 1.3, 0.0, 0.0, 0.0, 0.97, None),      # amplitude 9
        (370, 370, 1.4, -0.3, 0.0, 0.0, 0.8, None),      # amplitude 10
        (620, 400, 1.0, 0.0, 0.0, 0.0, 0.6, 60),         # exactly at the det-score and size gates: valid
        (760, 400, 1.0, 0.0, 0.0, 0.0, 0.5999, None),    # det score just under 0.6
        (860, 420, 1.0, 0.0, 0.0, 0.0, 0.9, 59),         # one pixel under the size gate
        (700, 460, 1.2, 0.0, 40.0, 0.0, 0.9, None),      # yaw beyond 45
        (560, 470, 1.2, 0.0, 0.0, 20.0, 0.9, None),      # pitch beyond 30
        (820, 480, 1.2, 0.62, 0.0, 0.0, 0.9, None),      # roll beyond 30 degrees
        (200, 200, 0.8, 0.1, 3.0, -3.0, 0.95, None),     # noise, small face
        (480, 250, 1.0, 0.0, 0.0, 0.0, 0.7, None),       # smooth background: blur ~ 0
        (940, 520, 1.5, 0.0, 0.0, 0.0, 0.99, None),      # crosses the frame border
    ]
    out = []
    for cx, cy, sc, roll, ndx, ndy, score, size in specs:
        lm = _landmarks(cx, cy, sc, roll, ndx, ndy) + r.normal(0, 0.4, (5, 2)).astype(np.float32)
        lo, hi = lm.min(0), lm.max(0)
        if size is None:
            bb = np.array([lo[0] - 18, lo[1] - 30, hi[0] + 18, hi[1] + 14]).astype(np.int32)
        else:
            x0, y0 = int(lo[0]) - 5, int(lo[1]) - 5
            bb = np.array([x0, y0, x0 + size, y0 + size + 7], np.int32)
        out.append({"bbox": bb, "landmarks": lm.astype(np.float32), "det_score": float(score)})
    return out


QUALITY_CONFIGS = [
    {},                                                                     # FaceQualityFilter defaults
    {"min_det_score": 0.5, "min_face_size": 40, "max_yaw": 30, "max_pitch": 20, "max_roll": 20,
     "check_blur": True, "blur_threshold": 50},
    {"check_blur": False},
]
