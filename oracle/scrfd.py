"""Restatement of the reference's face detector path (A14) — ORACLE, test-only.

``FaceDetector.detect`` (``face_recognition.py:31-48``) calls insightface
``FaceAnalysis('buffalo_l').get`` (``:20-29``), whose detector is SCRFD
``det_10g.onnx`` run by onnxruntime at ``det_size=(640,640)``.  insightface,
onnxruntime and the model pack are all absent (and must not be fetched), so
parity is UNPINNED: this module restates, from their published sources,

* ``insightface.model_zoo.scrfd.SCRFD.detect / forward / nms`` (letterbox with
  ``cv2.resize``, ``cv2.dnn.blobFromImage(1/128, mean 127.5, swapRB)``, per-stride
  anchor decode ``distance2bbox`` / ``distance2kps``, score-sorted greedy NMS at
  IoU 0.4) in numpy float32, the way the Python code computes it;
* ``cv2.resize(INTER_LINEAR)`` on uint8 as OpenCV's fixed-point resizer does it
  (11-bit coefficients; the SSE2 vertical pass rounds as
  ``(((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16) + 2) >> 2`` and its scalar tail as
  ``(S0*b0 + S1*b1 + 2^21) >> 22``);
* the SCRFD-10G-BNKPS network (insightface ``detection/scrfd`` config
  ``scrfd_10g_bnkps``: ResNetV1e backbone, BasicBlock stages (3,4,2,3) of widths
  (56,88,88,224), deep stem 28/28/56, avg-pool downsample shortcuts; PAFPN to 56
  channels over strides 8/16/32; per-stride heads of 3 x (conv3x3 80 + BN + ReLU)
  then cls(2) / bbox(8) / kps(20) conv3x3; 2 anchors per location) as a
  PyTorch-CPU fp32 module.  The ONNX graph itself is not available to check the
  restatement against; weights are seeded synthetic.

Only tests/ and bench.py's CPU baseline use this module.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch
from torch import nn
import torch.nn.functional as F

STRIDES = (8, 16, 32)
NUM_ANCHORS = 2
INPUT_MEAN, INPUT_STD = 127.5, 128.0
NMS_THRESH = 0.4

STAGE_BLOCKS = (3, 4, 2, 3)
STAGE_PLANES = (56, 88, 88, 224)
STEM = 56
NECK = 56
HEAD = 80


# --------------------------------------------------------------------------- network
def _bn(c):
    return nn.BatchNorm2d(c, eps=1e-5)


class ConvBN(nn.Module):
    def __init__(self, cin, cout, k, s, p):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, s, p, bias=False)
        self.bn = _bn(cout)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)))


class BasicBlock(nn.Module):
    """mmdet BasicBlock: stride on conv1; ReLU after the residual add."""

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = _bn(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = _bn(cout)
        self.downsample = None
        if stride != 1 or cin != cout:  # ResNetV1e avg_down: AvgPool(stride) -> conv1x1 -> BN
            self.downsample = nn.Sequential(
                nn.AvgPool2d(stride, stride, ceil_mode=True, count_include_pad=False) if stride > 1 else nn.Identity(),
                nn.Conv2d(cin, cout, 1, 1, bias=False), _bn(cout))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(out)) + idt)


class Conv(nn.Module):
    def __init__(self, cin, cout, k, s=1, p=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, s, p, bias=True)

    def forward(self, x):
        return self.conv(x)


class SCRFD10G(nn.Module):
    def __init__(self):
        super().__init__()
        bb = nn.Module()
        bb.stem = nn.Sequential(ConvBN(3, STEM // 2, 3, 2, 1), ConvBN(STEM // 2, STEM // 2, 3, 1, 1),
                                ConvBN(STEM // 2, STEM, 3, 1, 1))
        cin = STEM
        for i, (n, c) in enumerate(zip(STAGE_BLOCKS, STAGE_PLANES)):
            s = 1 if i == 0 else 2
            setattr(bb, f"layer{i + 1}", nn.Sequential(*[BasicBlock(cin if u == 0 else c, c, s if u == 0 else 1)
                                                        for u in range(n)]))
            cin = c
        self.backbone = bb
        neck = nn.Module()
        ins = STAGE_PLANES[1:]
        neck.lateral_convs = nn.ModuleList([Conv(c, NECK, 1) for c in ins])
        neck.fpn_convs = nn.ModuleList([Conv(NECK, NECK, 3, 1, 1) for _ in ins])
        neck.downsample_convs = nn.ModuleList([Conv(NECK, NECK, 3, 2, 1) for _ in ins[1:]])
        neck.pafpn_convs = nn.ModuleList([Conv(NECK, NECK, 3, 1, 1) for _ in ins[1:]])
        self.neck = neck
        head = nn.Module()
        head.towers = nn.ModuleList([nn.Sequential(ConvBN(NECK, HEAD, 3, 1, 1), ConvBN(HEAD, HEAD, 3, 1, 1),
                                                   ConvBN(HEAD, HEAD, 3, 1, 1)) for _ in STRIDES])
        head.cls = nn.ModuleList([nn.Conv2d(HEAD, NUM_ANCHORS, 3, 1, 1) for _ in STRIDES])
        head.reg = nn.ModuleList([nn.Conv2d(HEAD, NUM_ANCHORS * 4, 3, 1, 1) for _ in STRIDES])
        head.kps = nn.ModuleList([nn.Conv2d(HEAD, NUM_ANCHORS * 10, 3, 1, 1) for _ in STRIDES])
        self.bbox_head = head

    def forward(self, x) -> List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        bb = self.backbone
        x = F.max_pool2d(bb.stem(x), 3, 2, 1)
        feats = []
        for i in range(4):
            x = getattr(bb, f"layer{i + 1}")(x)
            if i >= 1:
                feats.append(x)
        nk = self.neck
        lat = [c(f) for c, f in zip(nk.lateral_convs, feats)]
        for i in range(len(lat) - 1, 0, -1):
            lat[i - 1] = lat[i - 1] + F.interpolate(lat[i], size=lat[i - 1].shape[2:], mode="nearest")
        inter = [c(l) for c, l in zip(nk.fpn_convs, lat)]
        for i in range(len(inter) - 1):
            inter[i + 1] = inter[i + 1] + nk.downsample_convs[i](inter[i])
        outs = [inter[0]] + [nk.pafpn_convs[i - 1](inter[i]) for i in range(1, len(inter))]
        hd = self.bbox_head
        res = []
        for lv, f in enumerate(outs):
            t = hd.towers[lv](f)
            res.append((torch.sigmoid(hd.cls[lv](t)), hd.reg[lv](t), hd.kps[lv](t)))
        return res


def load_oracle(state_dict) -> SCRFD10G:
    m = SCRFD10G()
    m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()})
    return m.eval()


# --------------------------------------------------------------------------- cv2.resize
def _coeffs(dsize: int, ssize: int):
    """Source index and 11-bit weights per output coordinate (cv::resize, INTER_LINEAR)."""
    scale = 1.0 / (float(dsize) / ssize)
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    hi = s >= ssize - 1
    f[hi], s[hi] = 0, ssize - 1
    a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, ssize - 1), a0, a1


def resize_linear_u8(img: np.ndarray, dw: int, dh: int) -> np.ndarray:
    H, W, C = img.shape
    xs0, xs1, a0, a1 = _coeffs(dw, W)
    ys0, ys1, b0, b1 = _coeffs(dh, H)
    src = img.astype(np.int64)
    D = src[:, xs0, :] * a0[None, :, None] + src[:, xs1, :] * a1[None, :, None]   # [H, dw, C] = value x 2048
    D = D.reshape(H, dw * C)
    S0, S1 = D[ys0], D[ys1]
    B0, B1 = b0[:, None], b1[:, None]
    simd = ((S0 >> 4) * B0 >> 16) + ((S1 >> 4) * B1 >> 16)
    simd = (simd + 2) >> 2
    scal = (S0 * B0 + S1 * B1 + (1 << 21)) >> 22
    width = dw * C
    x = 0
    while x <= width - 16:
        x += 16
    while x < width - 8:
        x += 8
    out = np.where(np.arange(width)[None, :] < x, simd, scal)
    return np.clip(out, 0, 255).astype(np.uint8).reshape(dh, dw, C)


def letterbox_geometry(h: int, w: int, det_w: int = 640, det_h: int = 640) -> Tuple[int, int, float]:
    """scrfd.py detect(): new size and det_scale for an h x w image."""
    im_ratio = float(h) / w
    model_ratio = float(det_h) / det_w
    if im_ratio > model_ratio:
        new_h = det_h
        new_w = int(new_h / im_ratio)
    else:
        new_w = det_w
        new_h = int(new_w * im_ratio)
    return new_w, new_h, float(new_h) / h


def letterbox(img: np.ndarray, det_w: int = 640, det_h: int = 640) -> Tuple[np.ndarray, float]:
    new_w, new_h, det_scale = letterbox_geometry(img.shape[0], img.shape[1], det_w, det_h)
    out = np.zeros((det_h, det_w, 3), np.uint8)
    out[:new_h, :new_w] = resize_linear_u8(img, new_w, new_h)
    return out, det_scale


def blob(det_img_rgb: np.ndarray) -> torch.Tensor:
    """blobFromImage(bgr, 1/128, mean 127.5, swapRB=True) of the BGR image = the RGB image."""
    x = (det_img_rgb.astype(np.float32) - np.float32(INPUT_MEAN)) * np.float32(1.0 / INPUT_STD)
    return torch.from_numpy(np.ascontiguousarray(x.transpose(2, 0, 1)))[None]


# --------------------------------------------------------------------------- post-processing
def head_outputs_to_lists(heads) -> Tuple[List[np.ndarray], List[np.ndarray], List[np.ndarray]]:
    """NCHW head maps -> the ONNX output layout: per stride [(H*W*A), 1|4|10]."""
    sc, bb, kp = [], [], []
    for cls, reg, kps in heads:
        sc.append(cls[0].permute(1, 2, 0).reshape(-1, 1).numpy())
        bb.append(reg[0].permute(1, 2, 0).reshape(-1, 4).numpy())
        kp.append(kps[0].permute(1, 2, 0).reshape(-1, 10).numpy())
    return sc, bb, kp


def decode(scores_l, bbox_l, kps_l, threshold: float, input_h: int = 640, input_w: int = 640):
    """SCRFD.forward after session.run: threshold, anchor centres, distance2bbox/kps."""
    scores_list, bboxes_list, kpss_list = [], [], []
    for idx, stride in enumerate(STRIDES):
        scores = scores_l[idx]
        bbox_preds = bbox_l[idx] * np.float32(stride)
        kps_preds = kps_l[idx] * np.float32(stride)
        height, width = input_h // stride, input_w // stride
        centers = np.stack(np.mgrid[:height, :width][::-1], axis=-1).astype(np.float32)
        centers = (centers * stride).reshape((-1, 2))
        centers = np.stack([centers] * NUM_ANCHORS, axis=1).reshape((-1, 2))
        pos = np.where(scores >= threshold)[0]
        x1 = centers[:, 0] - bbox_preds[:, 0]
        y1 = centers[:, 1] - bbox_preds[:, 1]
        x2 = centers[:, 0] + bbox_preds[:, 2]
        y2 = centers[:, 1] + bbox_preds[:, 3]
        bboxes = np.stack([x1, y1, x2, y2], axis=-1)
        kpss = np.stack([centers[:, i % 2] + kps_preds[:, i] for i in range(10)], axis=-1).reshape(-1, 5, 2)
        scores_list.append(scores[pos])
        bboxes_list.append(bboxes[pos])
        kpss_list.append(kpss[pos])
    return scores_list, bboxes_list, kpss_list


def nms(dets: np.ndarray, thresh: float = NMS_THRESH) -> List[int]:
    x1, y1, x2, y2, scores = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3], dets[:, 4]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    order = scores.argsort(kind="stable")[::-1]
    keep = []
    while order.size > 0:
        i = order[0]
        keep.append(i)
        xx1 = np.maximum(x1[i], x1[order[1:]])
        yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]])
        yy2 = np.minimum(y2[i], y2[order[1:]])
        w = np.maximum(np.float32(0.0), xx2 - xx1 + 1)
        h = np.maximum(np.float32(0.0), yy2 - yy1 + 1)
        inter = w * h
        ovr = inter / (areas[i] + areas[order[1:]] - inter)
        inds = np.where(ovr <= np.float32(thresh))[0]
        order = order[inds + 1]
    return keep


def detect_from_heads(scores_l, bbox_l, kps_l, det_scale: float, threshold: float = 0.5,
                      input_h: int = 640, input_w: int = 640) -> Tuple[np.ndarray, np.ndarray]:
    """SCRFD.detect after forward: concat, score sort, / det_scale, NMS -> det [n,5], kpss [n,5,2].

    Ties: insightface's ``argsort()[::-1]`` is unstable; the restatement (and the GPU
    path) order equal scores by ascending anchor index (stable sort, reversed, puts the
    higher index first -- so the key is (score desc, index asc) via a lexsort)."""
    s_l, b_l, k_l = decode(scores_l, bbox_l, kps_l, threshold, input_h, input_w)
    scores = np.vstack(s_l) if s_l else np.zeros((0, 1), np.float32)
    ravel = scores.ravel()
    idx = np.arange(ravel.shape[0])
    order = np.lexsort((idx, -ravel.astype(np.float64)))
    bboxes = (np.vstack(b_l) / np.float32(det_scale)).astype(np.float32)
    kpss = (np.vstack(k_l) / np.float32(det_scale)).astype(np.float32)
    pre_det = np.hstack((bboxes, scores)).astype(np.float32, copy=False)[order, :]
    keep = _nms_sorted(pre_det)
    return pre_det[keep, :], kpss[order][keep]


def _nms_sorted(dets: np.ndarray, thresh: float = NMS_THRESH) -> List[int]:
    """``nms`` on rows already in priority order (the re-sort inside insightface's nms
    is the identity on them, ties aside)."""
    x1, y1, x2, y2 = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    order = np.arange(dets.shape[0])
    keep = []
    while order.size > 0:
        i = order[0]
        keep.append(i)
        xx1 = np.maximum(x1[i], x1[order[1:]])
        yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]])
        yy2 = np.minimum(y2[i], y2[order[1:]])
        w = np.maximum(np.float32(0.0), xx2 - xx1 + 1)
        h = np.maximum(np.float32(0.0), yy2 - yy1 + 1)
        inter = w * h
        ovr = inter / (areas[i] + areas[order[1:]] - inter)
        order = order[np.where(ovr <= np.float32(thresh))[0] + 1]
    return keep


def detect(model: SCRFD10G, img_rgb: np.ndarray, threshold: float = 0.5, det_size=(640, 640)) -> List[Dict]:
    """FaceDetector.detect (face_recognition.py:31-48) with the restated SCRFD."""
    det_img, det_scale = letterbox(img_rgb, det_size[0], det_size[1])
    with torch.no_grad():
        heads = model(blob(det_img))
    s, b, k = head_outputs_to_lists(heads)
    det, kpss = detect_from_heads(s, b, k, det_scale, threshold, det_size[1], det_size[0])
    return [{"bbox": det[i, :4].astype(np.int32), "landmarks": kpss[i].astype(np.float32),
             "det_score": float(det[i, 4]), "pose": None, "age": None, "gender": None}
            for i in range(det.shape[0])]
