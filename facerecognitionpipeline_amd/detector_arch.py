"""SCRFD-10G detector description: state-dict schema and seeded synthetic weights.

The reference detects with insightface ``FaceAnalysis('buffalo_l')`` -> SCRFD
``det_10g.onnx`` (``face_recognition.py:19-48``).  That model pack is not in
the image and must not be fetched, so the network is the published
SCRFD-10G-BNKPS configuration restated (oracle/scrfd.py is the
test-side PyTorch module with the same keys): 4.23 M parameters and 13.34
GMAC at 640x640, which match the model zoo's figures (4.23 M, 10.18 GFLOPs at
VGA 640x480).  ``fr_set_param`` accepts exactly these keys.
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import List, Tuple

import numpy as np

STAGE_BLOCKS = (3, 4, 2, 3)
STAGE_PLANES = (56, 88, 88, 224)
STEM, NECK, HEAD = 56, 56, 80
STRIDES = (8, 16, 32)
DETECTOR_WEIGHT_SEED = 20251227
# A seeded random network's score maps are nearly flat, so the synthetic head is scaled to
# put ~150 anchors of a 1080p frame above det_thresh 0.5 (then ~75 boxes of 100-400 px survive
# NMS): cls weights x30 with per-level biases, bbox distances biased to 2 strides.  Enough to
# exercise decode + NMS, far below the 4096-candidate cap.  (SCRFD's own head init uses
# bias_init_with_prob(0.01) = -4.595.)
SYNTHETIC_CLS_GAIN = 30.0
SYNTHETIC_CLS_BIAS = (0.0, -0.8, -2.0)
SYNTHETIC_REG_BIAS = 2.0


def _bn(p: str, c: int) -> List[Tuple[str, tuple]]:
    return [(p + ".weight", (c,)), (p + ".bias", (c,)), (p + ".running_mean", (c,)), (p + ".running_var", (c,)),
            (p + ".num_batches_tracked", ())]


def detector_state_dict_schema() -> "OrderedDict[str, tuple]":
    s: List[Tuple[str, tuple]] = []
    stem = [(3, STEM // 2), (STEM // 2, STEM // 2), (STEM // 2, STEM)]
    for i, (ci, co) in enumerate(stem):
        s += [(f"backbone.stem.{i}.conv.weight", (co, ci, 3, 3))] + _bn(f"backbone.stem.{i}.bn", co)
    cin = STEM
    for st, (n, c) in enumerate(zip(STAGE_BLOCKS, STAGE_PLANES)):
        for u in range(n):
            ci = cin if u == 0 else c
            p = f"backbone.layer{st + 1}.{u}."
            s += [(p + "conv1.weight", (c, ci, 3, 3))] + _bn(p + "bn1", c)
            s += [(p + "conv2.weight", (c, c, 3, 3))] + _bn(p + "bn2", c)
            if u == 0 and (st > 0 or ci != c):
                s += [(p + "downsample.1.weight", (c, ci, 1, 1))] + _bn(p + "downsample.2", c)
        cin = c
    ins = STAGE_PLANES[1:]
    for i, c in enumerate(ins):
        s += [(f"neck.lateral_convs.{i}.conv.weight", (NECK, c, 1, 1)), (f"neck.lateral_convs.{i}.conv.bias", (NECK,))]
    for i in range(len(ins)):
        s += [(f"neck.fpn_convs.{i}.conv.weight", (NECK, NECK, 3, 3)), (f"neck.fpn_convs.{i}.conv.bias", (NECK,))]
    for name in ("downsample_convs", "pafpn_convs"):
        for i in range(len(ins) - 1):
            s += [(f"neck.{name}.{i}.conv.weight", (NECK, NECK, 3, 3)), (f"neck.{name}.{i}.conv.bias", (NECK,))]
    for lv in range(len(STRIDES)):
        for j in range(3):
            p = f"bbox_head.towers.{lv}.{j}"
            s += [(p + ".conv.weight", (HEAD, NECK if j == 0 else HEAD, 3, 3))] + _bn(p + ".bn", HEAD)
    for name, c in (("cls", 2), ("reg", 8), ("kps", 20)):
        for lv in range(len(STRIDES)):
            s += [(f"bbox_head.{name}.{lv}.weight", (c, HEAD, 3, 3)), (f"bbox_head.{name}.{lv}.bias", (c,))]
    return OrderedDict(s)


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(key.encode())])))


def synthetic_detector_state_dict(seed: int = DETECTOR_WEIGHT_SEED) -> "OrderedDict[str, np.ndarray]":
    """conv: U(+-1/sqrt(fan_in)) (cls convs x SYNTHETIC_CLS_GAIN); BN: gamma U(0.9,1.1),
    beta N(0,0.02^2), mean N(0,0.1^2), var U(0.5,1.5); cls / reg biases as above, other
    biases U(+-1/sqrt(fan_in))."""
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    schema = detector_state_dict_schema()
    for key, shape in schema.items():
        r = _rng(seed, key)
        leaf = key.rsplit(".", 1)[1]
        if leaf == "num_batches_tracked":
            sd[key] = np.array(0, dtype=np.int64)
            continue
        if len(shape) == 4:
            bound = 1.0 / np.sqrt(np.prod(shape[1:]))
            v = r.uniform(-bound, bound, size=shape)
            if key.startswith("bbox_head.cls."):
                v = v * SYNTHETIC_CLS_GAIN
        elif key.startswith("bbox_head.cls.") and leaf == "bias":
            v = np.full(shape, SYNTHETIC_CLS_BIAS[int(key.split(".")[2])])
        elif key.startswith("bbox_head.reg.") and leaf == "bias":
            v = np.full(shape, SYNTHETIC_REG_BIAS)
        elif (key.startswith("neck.") or key.startswith("bbox_head.")) and leaf == "bias" and ".bn." not in key:
            w = schema[key[:-4] + "weight"]
            bound = 1.0 / np.sqrt(np.prod(w[1:]))
            v = r.uniform(-bound, bound, size=shape)
        elif leaf == "weight":
            v = r.uniform(0.9, 1.1, size=shape)
        elif leaf == "bias":
            v = r.normal(0.0, 0.02, size=shape)
        elif leaf == "running_mean":
            v = r.normal(0.0, 0.1, size=shape)
        elif leaf == "running_var":
            v = r.uniform(0.5, 1.5, size=shape)
        else:  # pragma: no cover
            raise KeyError(key)
        sd[key] = v.astype(np.float32)
    return sd


def detector_macs(det_w: int = 640, det_h: int = 640) -> int:
    """Multiply-accumulates of one letterboxed frame (unpadded channels)."""
    macs = 0
    h, w = det_h // 2, det_w // 2
    for ci, co in [(3, STEM // 2), (STEM // 2, STEM // 2), (STEM // 2, STEM)]:
        macs += h * w * ci * co * 9
    h, w = h // 2, w // 2
    cin = STEM
    dims = []
    for st, (n, c) in enumerate(zip(STAGE_BLOCKS, STAGE_PLANES)):
        for u in range(n):
            s = 2 if (u == 0 and st > 0) else 1
            ci = cin if u == 0 else c
            ho, wo = h // s, w // s
            macs += ho * wo * c * ci * 9 + ho * wo * c * c * 9
            if u == 0 and (st > 0 or ci != c):
                macs += ho * wo * c * ci
            h, w = ho, wo
        cin = c
        dims.append((h, w))
    lv = dims[1:]
    for (hh, ww), c in zip(lv, STAGE_PLANES[1:]):
        macs += hh * ww * NECK * c + hh * ww * NECK * NECK * 9                        # lateral + fpn
    for (hh, ww) in lv[1:]:
        macs += 2 * hh * ww * NECK * NECK * 9                                         # downsample + pafpn
    for (hh, ww) in lv:
        macs += hh * ww * 9 * (NECK * HEAD + 2 * HEAD * HEAD + HEAD * 30)              # towers + heads
    return macs
