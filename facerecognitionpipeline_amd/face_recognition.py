"""Drop-in ``FaceAligner`` / ``FaceQualityFilter`` / ``FaceProcessor`` (face_recognition.py:50-216).

Alignment (cv2.estimateAffinePartial2D + cv2.warpAffine, face_recognition.py:64-74)
and the blur score (cv2.Laplacian variance, :94-99) run on the GPU through
``fr_align_faces`` / ``fr_warp_affine`` / ``fr_blur_scores``, so a frame uploaded
once yields crops that stay in HBM for ``FaceEmbedder.embed_tensor``.  Pose
angles and the threshold logic are scalar host code, as in the reference.

``FaceDetector`` replaces insightface ``FaceAnalysis('buffalo_l')`` (SCRFD
det_10g, :19-48) with the SCRFD-10G network on the GPU (``fr_detect``:
letterbox, MFMA conv pyramid, anchor decode, NMS).  No weights exist offline,
so it runs seeded synthetic weights unless ``model_path`` / ``state_dict``
gives a state dict in ``detector_arch`` keys; ``FaceProcessor`` also accepts
any detector object with the reference's
``detect(image_rgb) -> [{'bbox','landmarks','det_score',...}]`` contract.

Parity of the OpenCV arithmetic is UNPINNED (cv2 absent); the kernels are
pinned bit-exactly to the restatement in ``oracle/align_ref.py``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _lib


def reference_template(output_size: int) -> np.ndarray:
    S = output_size
    return np.array([[0.34 * S, 0.46 * S], [0.66 * S, 0.46 * S], [0.50 * S, 0.61 * S],
                     [0.37 * S, 0.74 * S], [0.63 * S, 0.74 * S]], dtype=np.float32)


class _DeviceOps:
    """One lightweight handle for the alignment / quality kernels (no model weights)."""

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        self._h: Optional[_lib.Handle] = None

    @property
    def handle(self) -> "_lib.Handle":
        if self._h is None:
            self._h = _lib.Handle("ir_50", "adaface", self.device, max_batch=1)
        return self._h


class FaceAligner:
    def __init__(self, output_size: int = 112, device=None):
        self.output_size = output_size
        self.template = reference_template(output_size)
        self._ops = _DeviceOps(device)

    def align(self, image: np.ndarray, landmarks: np.ndarray, method: str = "similarity") -> np.ndarray:
        """Host image in, host crop out (reference signature).  A 2-D gray image gives a 2-D crop,
        as cv2.warpAffine does (each channel of the warp is the single-channel warp)."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        gray = img.ndim == 2
        if gray:
            img = np.repeat(img[:, :, None], 3, axis=2)
        frame = torch.from_numpy(img).to(self._ops.device)
        out = self.align_batch(frame, np.asarray(landmarks, np.float32)[None], method)[0].cpu().numpy()
        return np.ascontiguousarray(out[..., 0]) if gray else out

    def align_batch(self, frame: torch.Tensor, landmarks: np.ndarray, method: str = "similarity") -> torch.Tensor:
        """Device form: uint8 [H,W,3] frame on the GPU, float32 [n,5,2] landmarks -> uint8 [n,S,S,3] on the GPU."""
        if frame.dtype != torch.uint8 or frame.dim() != 3 or frame.shape[2] != 3:
            raise ValueError("expected a uint8 [H,W,3] RGB frame tensor")
        lm = np.ascontiguousarray(landmarks, dtype=np.float32).reshape(-1, 5, 2)
        S = self.output_size
        out = torch.empty((lm.shape[0], S, S, 3), dtype=torch.uint8, device=self._ops.device)
        frame = frame.to(self._ops.device).contiguous()
        if method == "similarity":
            self._ops.handle.align_faces(frame, lm, S, out)
        else:
            tf = np.stack([affine_from_3_points(x[:3], self.template[:3]) for x in lm])
            self._ops.handle.warp_affine(frame, tf, S, out)
        return out


def affine_from_3_points(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """cv2.getAffineTransform(src[:3], dst[:3]) (exact 3-point solve, float64)."""
    s = np.asarray(src, np.float32).astype(np.float64)
    d = np.asarray(dst, np.float32).astype(np.float64)
    A = np.zeros((6, 6))
    b = np.zeros(6)
    for i in range(3):
        A[2 * i, :3] = [s[i, 0], s[i, 1], 1.0]
        A[2 * i + 1, 3:] = [s[i, 0], s[i, 1], 1.0]
        b[2 * i], b[2 * i + 1] = d[i, 0], d[i, 1]
    return np.linalg.solve(A, b).reshape(2, 3)


class FaceQualityFilter:
    def __init__(self, min_det_score=0.6, min_face_size=60, max_yaw=45, max_pitch=30, max_roll=30,
                 check_blur=True, blur_threshold=100, device=None):
        self.min_det_score = min_det_score
        self.min_face_size = min_face_size
        self.max_yaw = max_yaw
        self.max_pitch = max_pitch
        self.max_roll = max_roll
        self.check_blur = check_blur
        self.blur_threshold = blur_threshold
        self._ops = _DeviceOps(device)

    def compute_blur_score(self, face_image) -> float:
        """cv2.Laplacian(gray, CV_64F).var() of one image (face_recognition.py:94-99): a 3-D
        [H,W,3] (or [H,W,4]) RGB image goes through RGB2GRAY, a 2-D one is the gray image.  Any
        size.  Returns np.float64, like ndarray.var() in the reference."""
        t = face_image if isinstance(face_image, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(face_image, np.uint8))
        if t.dim() not in (2, 3):
            raise ValueError(f"expected an HxW or HxWxC image, got {tuple(t.shape)}")
        return np.float64(self.compute_blur_scores(t.unsqueeze(0))[0])

    def compute_blur_scores(self, crops) -> np.ndarray:
        """A batch of one size (host array or device tensor): uint8 [n,H,W,3|4] RGB(A) or
        [n,H,W] gray -> float64 [n]."""
        t = crops if isinstance(crops, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(crops, np.uint8))
        if t.dtype != torch.uint8:
            t = t.to(torch.uint8)
        if t.dim() not in (3, 4) or (t.dim() == 4 and t.shape[3] not in (1, 3, 4)):
            raise ValueError(f"expected uint8 [n,H,W] gray or [n,H,W,3] RGB images, got {tuple(t.shape)}")
        if t.dim() == 4 and t.shape[3] == 1:
            t = t[..., 0]
        return self._ops.handle.blur_scores(t.to(self._ops.device).contiguous())

    def compute_pose_angles(self, landmarks: np.ndarray) -> Dict[str, float]:
        le, re, nose, lm, rm = [np.asarray(p) for p in landmarks]
        eye_c = (le + re) / 2
        d = re - le
        roll = np.degrees(np.arctan2(d[1], d[0]))
        yaw = np.degrees(np.arcsin(np.clip((nose[0] - eye_c[0]) / np.linalg.norm(d), -1, 1))) * 2
        mouth_c = (lm + rm) / 2
        pitch = ((nose[1] - eye_c[1]) / (mouth_c[1] - eye_c[1]) - 0.5) * 60
        return {"yaw": yaw, "pitch": pitch, "roll": roll}

    def is_valid(self, face_dict: Dict, face_image=None, blur_score: Optional[float] = None) -> Tuple[bool, Dict]:
        m: Dict = {"det_score": face_dict["det_score"]}
        if m["det_score"] < self.min_det_score:
            return False, m
        x0, y0, x1, y1 = face_dict["bbox"][:4]
        m["face_size"] = min(x1 - x0, y1 - y0)
        if m["face_size"] < self.min_face_size:
            return False, m
        pose = self.compute_pose_angles(face_dict["landmarks"])
        m.update(pose)
        if abs(pose["yaw"]) > self.max_yaw or abs(pose["pitch"]) > self.max_pitch or abs(pose["roll"]) > self.max_roll:
            return False, m
        if self.check_blur and (face_image is not None or blur_score is not None):
            m["blur_score"] = np.float64(blur_score) if blur_score is not None else self.compute_blur_score(face_image)
            if m["blur_score"] < self.blur_threshold:
                return False, m
        return True, m


def load_image_rgb(path: str) -> Optional[np.ndarray]:
    """cv2.cvtColor(cv2.imread(path), COLOR_BGR2RGB) through PIL: uint8 [H,W,3] RGB, or None when
    the file is missing or not a decodable image (cv2.imread returns None there).  imread's
    default IMREAD_COLOR makes every image 3-channel: gray and palette images are expanded, an
    alpha channel is dropped.  (8-bit images; imread's 16-bit down-conversion is not restated.)"""
    try:
        from PIL import Image
        with Image.open(path) as im:
            im.load()
            return np.array(im.convert("RGB"), dtype=np.uint8)  # a writable copy
    except (OSError, ValueError, SyntaxError):
        return None


class FaceDetector:
    """``FaceDetector`` (face_recognition.py:19-48) on the GPU: SCRFD-10G at ``det_size``,
    ``det_thresh``, NMS IoU 0.4; ``providers`` is accepted for signature parity."""

    def __init__(self, det_size=(640, 640), det_thresh=0.5, providers=None, model_path: Optional[str] = None,
                 state_dict=None, device=None, max_frames: int = 16, max_faces: int = 256):
        from .detector_arch import synthetic_detector_state_dict
        if tuple(det_size) != (640, 640):
            raise NotImplementedError("the MI355X detector is built for det_size=(640, 640) (the reference's setting)")
        self.det_size = tuple(det_size)
        self.det_thresh = float(det_thresh)
        self.max_faces = int(max_faces)
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        if state_dict is None:
            if model_path is not None:
                sd = torch.load(model_path, map_location="cpu", weights_only=True)
                state_dict = sd.get("state_dict", sd) if isinstance(sd, dict) else sd
            else:
                state_dict = synthetic_detector_state_dict()
        self.model = _lib.Handle("scrfd_10g", "scrfd", self.device, max_batch=max_frames)
        self.model.load_state_dict({k: v for k, v in state_dict.items()})

    @staticmethod
    def _to_rgb(image: np.ndarray) -> np.ndarray:
        if image.ndim == 2:  # cv2.COLOR_GRAY2BGR replicates the channel (face_recognition.py:32-33)
            image = np.repeat(image[:, :, None], 3, axis=2)
        if image.ndim != 3 or image.shape[2] != 3:
            raise ValueError(f"expected an HxW or HxWx3 image, got {image.shape}")
        return np.ascontiguousarray(image, dtype=np.uint8)

    @staticmethod
    def _faces(dets: np.ndarray, count: int) -> List[Dict]:
        out = []
        for i in range(count):
            d = dets[i]
            out.append({"bbox": d[:4].astype(np.int32), "landmarks": d[5:15].reshape(5, 2).astype(np.float32),
                        "det_score": float(d[4]), "pose": None, "age": None, "gender": None})
        return out

    def detect(self, image: np.ndarray) -> List[Dict]:
        """RGB (or gray) uint8 image -> [{'bbox' int32 x1y1x2y2, 'landmarks' f32 (5,2), 'det_score', ...}]
        in descending score order, like face_recognition.py:31-48."""
        frame = torch.from_numpy(self._to_rgb(image)).to(self.device)
        return self.detect_batch(frame[None])[0]

    def detect_batch(self, frames: torch.Tensor) -> List[List[Dict]]:
        """Device form: uint8 [n,H,W,3] RGB frames (one size) -> per-frame face lists."""
        dets, counts = self.model.detect(frames, self.det_thresh, self.max_faces)
        return [self._faces(dets[f], min(int(counts[f]), self.max_faces)) for f in range(dets.shape[0])]


class FaceProcessor:
    """detect -> align -> quality (face_recognition.py:160-216) with device alignment and blur."""

    def __init__(self, output_size=224, det_size=(640, 640), det_thresh=0.5,
                 quality_filter_config: Optional[Dict] = None, providers=None, detector=None, device=None):
        self.detector = detector if detector is not None else FaceDetector(det_size, det_thresh, providers,
                                                                           device=device)
        self.aligner = FaceAligner(output_size=output_size, device=device)
        self.quality_filter = FaceQualityFilter(**(quality_filter_config or {}), device=device)

    def process_image(self, image_path: str, return_all: bool = False) -> List[Dict]:
        """face_recognition.py:174-182: read the file, convert to RGB, process_numpy.  The file is
        decoded by PIL (cv2 is not in the image): lossless formats (PNG, BMP, TIFF) decode to the
        same bytes cv2.imread gives; JPEG decoders may differ in rounding, so JPEG parity with
        cv2.imread is unpinned.  Like cv2.imread, a file that cannot be read raises ValueError."""
        image_rgb = load_image_rgb(image_path)
        if image_rgb is None:
            raise ValueError(f"Could not load image: {image_path}")
        return self.process_numpy(image_rgb, return_all)

    def process_numpy(self, image_rgb: np.ndarray, return_all: bool = False) -> List[Dict]:
        faces = self.detector.detect(image_rgb)
        if len(faces) == 0:
            return []
        # a grayscale frame is warped as three equal channels: each channel of the warp is the
        # reference's single-channel warpAffine (face_recognition.py:72-74), and RGB2GRAY of
        # (g, g, g) is g, so the blur score is the reference's on the 2-D crop (:94-99); the
        # aligned face is handed back 2-D, as the reference's is
        gray = np.ndim(image_rgb) == 2
        frame = torch.from_numpy(FaceDetector._to_rgb(image_rgb)).to(self.aligner._ops.device)
        crops = self.aligner.align_batch(frame, np.stack([f["landmarks"] for f in faces]))
        blur = self.quality_filter.compute_blur_scores(crops) if self.quality_filter.check_blur else None
        host = crops.cpu().numpy()
        if gray:
            host = np.ascontiguousarray(host[..., 0])
        results = []
        for i, face in enumerate(faces):
            ok, q = self.quality_filter.is_valid(face, None, None if blur is None else float(blur[i]))
            if ok or return_all:
                results.append({"aligned_face": host[i], "bbox": face["bbox"], "landmarks": face["landmarks"],
                                "det_score": face["det_score"], "quality_metrics": q, "is_valid": ok})
        results.sort(key=lambda x: x["det_score"] * x["quality_metrics"].get("blur_score", 1000), reverse=True)
        if not return_all and results:
            return [results[0]]
        return results
