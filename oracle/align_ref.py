"""Restatement of the reference's alignment + quality arithmetic — ORACLE, test-only.

PARITY UNPINNED: the reference calls OpenCV (``cv2.estimateAffinePartial2D``,
``cv2.warpAffine``, ``cv2.cvtColor``, ``cv2.Laplacian``; face_recognition.py:
64-74, 94-99), and OpenCV (unpinned, ``client_environment.yml:14``) is absent
from this image; the reference holds no aligned-crop fixtures (frames are
gitignored).  This module restates OpenCV 4.x's published algorithms from its
source semantics; tests pin the HIP kernels to THIS restatement bit for bit.

* ``fit_similarity``: estimateAffinePartial2D(from, to) with default RANSAC
  (threshold 3 px, refine on inliers).  When every point is an inlier of the
  least-squares similarity (the normal case for 5 face landmarks) OpenCV's
  Levenberg-Marquardt refinement converges to that least-squares solution,
  which is what is returned here.  Otherwise the max-consensus 2-point model
  over all 10 pairs decides the inliers (OpenCV's random sample order can pick
  a different equal-size set: unpinned).
* ``invert_affine``: warpAffine's double-precision inverse (imgwarp.cpp).
* ``warp_affine_linear``: warpAffine INTER_LINEAR, BORDER_CONSTANT 0, uint8:
  AB_BITS=10 fixed-point map (cvRound = round-half-even), INTER_BITS=5 sub-pixel
  table, 15-bit bilinear weights (exact products (32-a)(32-b)*32), rounding
  shift, saturate.
* ``rgb_to_gray``: COLOR_RGB2GRAY fixed point (R 4899, G 9617, B 1868, >>14).
* ``laplacian_var``: Laplacian(gray, CV_64F) ksize=1 kernel [0 1 0;1 -4 1;0 1 0],
  BORDER_REFLECT_101, then numpy ``.var()``.
* ``pose_angles``: FaceQualityFilter.compute_pose_angles (face_recognition.py:101-121).
"""
from __future__ import annotations

import itertools
from typing import Dict

import numpy as np

AB_BITS = 10
AB_SCALE = 1 << AB_BITS
INTER_BITS = 5
INTER_TAB = 1 << INTER_BITS
ROUND_DELTA = AB_SCALE // INTER_TAB // 2


def reference_template(output_size: int = 112) -> np.ndarray:
    """FaceAligner.template (face_recognition.py:52-60), float32."""
    S = output_size
    return np.array([[0.34 * S, 0.46 * S], [0.66 * S, 0.46 * S], [0.50 * S, 0.61 * S],
                     [0.37 * S, 0.74 * S], [0.63 * S, 0.74 * S]], dtype=np.float32)


def _ls_similarity(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Least-squares [a -b tx; b a ty] mapping src -> dst, closed form, float64.

    Written as explicit sequential sums so the C++ path (frhip_runtime.cpp:
    fit_similarity) performs the identical IEEE operation sequence.
    """
    n = src.shape[0]
    sx = sy = dx = dy = 0.0
    for i in range(n):
        sx += float(src[i, 0]); sy += float(src[i, 1]); dx += float(dst[i, 0]); dy += float(dst[i, 1])
    sx /= n; sy /= n; dx /= n; dy /= n
    num_a = num_b = den = 0.0
    for i in range(n):
        px, py = float(src[i, 0]) - sx, float(src[i, 1]) - sy
        qx, qy = float(dst[i, 0]) - dx, float(dst[i, 1]) - dy
        num_a += px * qx + py * qy
        num_b += px * qy - py * qx
        den += px * px + py * py
    a = num_a / den if den != 0 else 0.0
    b = num_b / den if den != 0 else 0.0
    tx = dx - (a * sx - b * sy)
    ty = dy - (b * sx + a * sy)
    return np.array([[a, -b, tx], [b, a, ty]], dtype=np.float64)


def _residuals(M: np.ndarray, src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    p = src @ M[:, :2].T + M[:, 2]
    return np.sqrt(((p - dst) ** 2).sum(1))


def fit_similarity(src_pts: np.ndarray, dst_pts: np.ndarray, thresh: float = 3.0) -> np.ndarray:
    """estimateAffinePartial2D(src, dst)[0] as float64 2x3 (see module doc)."""
    src = np.asarray(src_pts, dtype=np.float32).astype(np.float64)
    dst = np.asarray(dst_pts, dtype=np.float32).astype(np.float64)
    M = _ls_similarity(src, dst)
    if (_residuals(M, src, dst) < thresh).all():
        return M
    best, best_n = None, -1
    for i, j in itertools.combinations(range(len(src)), 2):
        Mi = _ls_similarity(src[[i, j]], dst[[i, j]])
        n_in = int((_residuals(Mi, src, dst) < thresh).sum())
        if n_in > best_n:
            best, best_n = Mi, n_in
    inl = _residuals(best, src, dst) < thresh
    return _ls_similarity(src[inl], dst[inl]) if inl.sum() >= 2 else best


def invert_affine(M: np.ndarray) -> np.ndarray:
    """warpAffine's inverse of a forward 2x3 map (double precision, imgwarp.cpp)."""
    m = [float(v) for v in np.asarray(M, dtype=np.float64).reshape(-1)]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = m[4] * D, m[0] * D
    m[0] = A11
    m[1] *= -D
    m[3] *= -D
    m[4] = A22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return np.array(m, dtype=np.float64).reshape(2, 3)


def _cvround(x: np.ndarray) -> np.ndarray:
    return np.rint(x).astype(np.int64)


def warp_affine_linear(img: np.ndarray, M_fwd: np.ndarray, size: int) -> np.ndarray:
    """cv2.warpAffine(img, M, (size, size), INTER_LINEAR, BORDER_CONSTANT, 0) for uint8 HxWxC."""
    Mi = invert_affine(M_fwd)
    H, W, C = img.shape
    xs = np.arange(size)
    ys = np.arange(size)
    adelta = _cvround(Mi[0, 0] * xs * AB_SCALE)
    bdelta = _cvround(Mi[1, 0] * xs * AB_SCALE)
    X0 = _cvround((Mi[0, 1] * ys + Mi[0, 2]) * AB_SCALE) + ROUND_DELTA
    Y0 = _cvround((Mi[1, 1] * ys + Mi[1, 2]) * AB_SCALE) + ROUND_DELTA
    X = (X0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx, fx = X >> INTER_BITS, X & (INTER_TAB - 1)
    sy, fy = Y >> INTER_BITS, Y & (INTER_TAB - 1)
    # 15-bit weights: (32-fx)(32-fy)*32 etc. (exact, sum 32768)
    w00 = (INTER_TAB - fx) * (INTER_TAB - fy) * 32
    w01 = fx * (INTER_TAB - fy) * 32
    w10 = (INTER_TAB - fx) * fy * 32
    w11 = fx * fy * 32
    src = img.astype(np.int64)

    def px(yy, xx):
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        v = src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]
        return np.where(ok[..., None], v, 0)

    acc = (px(sy, sx) * w00[..., None] + px(sy, sx + 1) * w01[..., None] +
           px(sy + 1, sx) * w10[..., None] + px(sy + 1, sx + 1) * w11[..., None])
    out = (acc + (1 << 14)) >> 15
    # fully outside (no tap inside the image) -> border value 0 (same as the weighted sum of zeros)
    return np.clip(out, 0, 255).astype(np.uint8)


def rgb_to_gray(img: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(img, COLOR_RGB2GRAY) for uint8 (fixed point, 14-bit)."""
    x = img.astype(np.int64)
    return ((x[..., 0] * 4899 + x[..., 1] * 9617 + x[..., 2] * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def laplacian_var(gray: np.ndarray) -> float:
    """cv2.Laplacian(gray, CV_64F).var() (ksize=1, BORDER_REFLECT_101)."""
    g = gray.astype(np.float64)
    p = np.pad(g, 1, mode="reflect")  # numpy 'reflect' == OpenCV BORDER_REFLECT_101
    lap = p[:-2, 1:-1] + p[2:, 1:-1] + p[1:-1, :-2] + p[1:-1, 2:] - 4.0 * g
    return float(lap.var())


def blur_score(face_rgb: np.ndarray) -> float:
    """FaceQualityFilter.compute_blur_score (face_recognition.py:94-99)."""
    gray = rgb_to_gray(face_rgb) if face_rgb.ndim == 3 else face_rgb
    return laplacian_var(gray)


def pose_angles(landmarks: np.ndarray) -> Dict[str, float]:
    """FaceQualityFilter.compute_pose_angles (face_recognition.py:101-121)."""
    le, re, nose, lm, rm = [np.asarray(p) for p in landmarks]
    eye_c = (le + re) / 2
    d = re - le
    roll = np.degrees(np.arctan2(d[1], d[0]))
    yaw = np.degrees(np.arcsin(np.clip((nose[0] - eye_c[0]) / np.linalg.norm(d), -1, 1))) * 2
    mouth_c = (lm + rm) / 2
    pitch = ((nose[1] - eye_c[1]) / (mouth_c[1] - eye_c[1]) - 0.5) * 60
    return {"yaw": yaw, "pitch": pitch, "roll": roll}
