"""Restatement of the reference's alignment + quality arithmetic — ORACLE, test-only.

PARITY UNPINNED: the reference calls OpenCV (``cv2.estimateAffinePartial2D``,
``cv2.warpAffine``, ``cv2.cvtColor``, ``cv2.Laplacian``; face_recognition.py:
64-74, 94-99), and OpenCV (unpinned, ``client_environment.yml:14``) is absent
from this image; the reference holds no aligned-crop fixtures (frames are
gitignored).  This module restates OpenCV 4.x's published algorithms from its
source semantics; tests pin the HIP kernels to THIS restatement bit for bit.

* ``fit_similarity``: estimateAffinePartial2D(from, to) with its defaults
  (RANSAC, threshold 3 px, 2000 iterations, confidence 0.99, 10 refine
  iterations), restating OpenCV's calib3d ``ptsetreg.cpp`` step for step:
  ``RANSACPointSetRegistrator::run`` with ``cv::RNG((uint64)-1)`` (the
  multiply-with-carry generator of core ``rand.cpp``), 2-point subsets drawn by
  ``getSubset`` (distinct indices, ``rng.uniform(0, count)``),
  ``AffinePartial2DEstimatorCallback::runKernel`` (closed-form 2-point
  similarity in double), ``computeError`` / ``findInliers`` in float32
  (``err <= (float)(thr*thr)``), the adaptive ``RANSACUpdateNumIters``; then
  the inliers (in input order) refined by the Levenberg-Marquardt solver of
  ``levmarq.cpp`` (OpenCV 3.x-4.5 ``LMSolverImpl::run``: lambda 1, Rlo 0.25,
  Rhi 0.75, eps FLT_EPSILON) on ``AffinePartial2DRefineCallback`` (parameters
  a, b, tx, ty).  Two deliberate deviations, both below double rounding: the
  damped normal equations are solved by Gaussian elimination with partial
  pivoting instead of ``DECOMP_EIG``, and sums run in index order.  (OpenCV
  4.7+ rewrote the LM solver; on this linear model every variant converges to
  the inliers' least-squares optimum.)  The C++ fit behind ``fr_align_faces``
  (frhip_runtime.cpp) performs the same IEEE operation sequence.
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

import math
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


_RNG_COEFF = 4164903690  # CV_RNG_COEFF (core/rand.cpp)
_M64 = (1 << 64) - 1
_DBL_MIN = 2.2250738585072014e-308
_DBL_EPSILON = 2.220446049250313e-16
_FLT_EPSILON = 1.1920928955078125e-07


class CvRNG:
    """cv::RNG: 64-bit multiply-with-carry; ``next`` returns the low 32 bits (core/rand.cpp)."""

    def __init__(self, state: int):
        state &= _M64
        self.state = state if state else 0xFFFFFFFF

    def next(self) -> int:
        s = self.state
        self.state = ((s & 0xFFFFFFFF) * _RNG_COEFF + (s >> 32)) & _M64
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        """RNG::uniform(int a, int b): a + next() % (b - a) in unsigned arithmetic."""
        return a if a == b else self.next() % (b - a) + a


def _kernel2(f, t):
    """AffinePartial2DEstimatorCallback::runKernel: exact similarity through 2 point pairs (double)."""
    (x1, y1), (x2, y2) = f
    (X1, Y1), (X2, Y2) = t
    den = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2)
    d = 1.0 / den if den != 0 else math.inf
    S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2))
    S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return [S0, -S1, S2, S1, S0, S3]


def _find_inliers(M, src32, dst32, thresh):
    """Affine2DEstimatorCallback::computeError (float32 model and arithmetic) + findInliers."""
    F = [np.float32(v) for v in M]
    t = np.float32(thresh * thresh)
    mask = []
    for (fx, fy), (tx, ty) in zip(src32, dst32):
        a = F[0] * fx + F[1] * fy + F[2] - tx
        b = F[3] * fx + F[4] * fy + F[5] - ty
        mask.append(bool(a * a + b * b <= t))
    return sum(mask), mask


def _update_num_iters(p: float, ep: float, model_points: int, max_iters: int) -> int:
    """RANSACUpdateNumIters (ptsetreg.cpp); (1 - ep)^2 as one product, as the compiled pow does."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, _DBL_MIN)
    q = 1.0 - ep
    denom = 1.0 - q * q if model_points == 2 else 1.0 - math.pow(q, model_points)
    if denom < _DBL_MIN:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(round(num / denom))  # cvRound: half to even


def _solve(A, b):
    """Gaussian elimination with partial pivoting (n <= 4); a zero pivot leaves its unknown 0."""
    n = len(b)
    M = [list(A[i]) + [b[i]] for i in range(n)]
    for c in range(n):
        p = c
        for r in range(c + 1, n):
            if abs(M[r][c]) > abs(M[p][c]):
                p = r
        M[c], M[p] = M[p], M[c]
        if M[c][c] == 0.0:
            continue
        for r in range(c + 1, n):
            f = M[r][c] / M[c][c]
            for k in range(c, n + 1):
                M[r][k] = M[r][k] - f * M[c][k]
    x = [0.0] * n
    for c in range(n - 1, -1, -1):
        if M[c][c] == 0.0:
            continue
        s = M[c][n]
        for k in range(c + 1, n):
            s = s - M[c][k] * x[k]
        x[c] = s / M[c][c]
    return x


def _refine_compute(h, src, dst, want_j):
    """AffinePartial2DRefineCallback::compute: residuals (and Jacobian) of h = (a, b, tx, ty)."""
    r, J = [], []
    for (Mx, My), (mx, my) in zip(src, dst):
        xi = h[0] * Mx - h[1] * My + h[2]
        yi = h[1] * Mx + h[0] * My + h[3]
        r += [xi - mx, yi - my]
        if want_j:
            J += [[Mx, -My, 1.0, 0.0], [My, Mx, 0.0, 1.0]]
    return r, J


def _normal(J, r):
    n = len(J)
    A = [[0.0] * 4 for _ in range(4)]
    v = [0.0] * 4
    for i in range(4):
        for j in range(4):
            s = 0.0
            for k in range(n):
                s += J[k][i] * J[k][j]
            A[i][j] = s
        s = 0.0
        for k in range(n):
            s += J[k][i] * r[k]
        v[i] = s
    return A, v


def _sq(r):
    s = 0.0
    for e in r:
        s += e * e
    return s


def _dot(a, b):
    s = 0.0
    for x, y in zip(a, b):
        s += x * y
    return s


def _lm_refine(h, src, dst, max_iters: int = 10, eps: float = _FLT_EPSILON):
    """LMSolverImpl::run (levmarq.cpp, OpenCV 3.x-4.5) on the partial-affine refine callback."""
    x = list(h)
    r, J = _refine_compute(x, src, dst, True)
    S = _sq(r)
    A, v = _normal(J, r)
    D = [A[i][i] for i in range(4)]
    Rlo, Rhi = 0.25, 0.75
    lam, lc = 1.0, 0.75
    it = 0
    while True:
        Ap = [[A[i][j] + (lam * D[i] if i == j else 0.0) for j in range(4)] for i in range(4)]
        d = _solve(Ap, v)
        xd = [x[i] - d[i] for i in range(4)]
        rd, _ = _refine_compute(xd, src, dst, False)
        Sd = _sq(rd)
        temp = [-_dot(A[i], d) + 2.0 * v[i] for i in range(4)]  # gemm(A, d, -1, v, 2)
        dS = _dot(d, temp)
        R = (S - Sd) / (dS if abs(dS) > _DBL_EPSILON else 1.0)
        if R > Rhi:
            lam *= 0.5
            if lam < lc:
                lam = 0.0
        elif R < Rlo:
            t = _dot(d, v)
            nu = (Sd - S) / (t if abs(t) > _DBL_EPSILON else 1.0) + 2.0
            nu = min(max(nu, 2.0), 10.0)
            if lam == 0.0:
                maxval = _DBL_EPSILON
                for i in range(4):
                    e = [1.0 if k == i else 0.0 for k in range(4)]
                    maxval = max(maxval, abs(_solve(A, e)[i]))
                lam = lc = 1.0 / maxval
                nu *= 0.5
            lam *= nu
        if Sd < S:
            S = Sd
            x = xd
            r, J = _refine_compute(x, src, dst, True)
            A, v = _normal(J, r)
        it += 1
        if not (it < max_iters and max(abs(e) for e in d) >= eps and max(abs(e) for e in r) >= eps):
            break
    return x


def fit_similarity(src_pts: np.ndarray, dst_pts: np.ndarray, thresh: float = 3.0, confidence: float = 0.99,
                   max_iters: int = 2000, refine_iters: int = 10) -> np.ndarray:
    """estimateAffinePartial2D(src, dst)[0] as float64 2x3 (see module doc); NaN-filled when it fails (None in cv2)."""
    src32 = [(np.float32(x), np.float32(y)) for x, y in np.asarray(src_pts, dtype=np.float32).reshape(-1, 2)]
    dst32 = [(np.float32(x), np.float32(y)) for x, y in np.asarray(dst_pts, dtype=np.float32).reshape(-1, 2)]
    src = [(float(x), float(y)) for x, y in src32]
    dst = [(float(x), float(y)) for x, y in dst32]
    count = len(src)
    fail = np.full((2, 3), np.nan)
    if count < 2 or len(dst) != count:
        return fail
    if count == 2:
        best, mask, good = _kernel2(src, dst), [True, True], 2
    else:
        rng = CvRNG(_M64)
        niters, good, best, mask = max(max_iters, 1), 0, None, None
        it = 0
        while it < niters:
            i0 = rng.uniform(0, count)
            i1 = rng.uniform(0, count)
            while i1 == i0:
                i1 = rng.uniform(0, count)
            M = _kernel2([src[i0], src[i1]], [dst[i0], dst[i1]])
            g, m = _find_inliers(M, src32, dst32, thresh)
            if g > max(good, 1):
                best, mask, good = M, m, g
                niters = _update_num_iters(confidence, (count - g) / count, 2, niters)
            it += 1
        if good <= 0:
            return fail
        if refine_iters:
            si = [p for p, k in zip(src, mask) if k]
            di = [p for p, k in zip(dst, mask) if k]
            h = _lm_refine([best[0], best[3], best[2], best[5]], si, di, refine_iters)
            best = [h[0], -h[1], h[2], h[1], h[0], h[3]]
    return np.array(best, dtype=np.float64).reshape(2, 3)


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


def warp_maps(M_fwd: np.ndarray, size: int):
    """warpAffine's fixed-point source map of every output pixel: X, Y in 1/32-pixel units
    (INTER_BITS sub-pixel); two forward maps give identical uint8 warps wherever these agree."""
    Mi = invert_affine(M_fwd)
    xs = np.arange(size)
    ys = np.arange(size)
    adelta = _cvround(Mi[0, 0] * xs * AB_SCALE)
    bdelta = _cvround(Mi[1, 0] * xs * AB_SCALE)
    X0 = _cvround((Mi[0, 1] * ys + Mi[0, 2]) * AB_SCALE) + ROUND_DELTA
    Y0 = _cvround((Mi[1, 1] * ys + Mi[1, 2]) * AB_SCALE) + ROUND_DELTA
    X = (X0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    return X, Y


def warp_affine_linear(img: np.ndarray, M_fwd: np.ndarray, size: int) -> np.ndarray:
    """cv2.warpAffine(img, M, (size, size), INTER_LINEAR, BORDER_CONSTANT, 0) for uint8 HxWxC."""
    H, W, C = img.shape
    X, Y = warp_maps(M_fwd, size)
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
