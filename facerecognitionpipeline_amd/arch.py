"""AdaFace IR backbone description: block list and state-dict schema.

The reference builds the network with ``net.build_model(architecture)``
(``face_embedder.py:49``) and loads a checkpoint whose ``state_dict`` keys are
``model.``-prefixed (``face_embedder.py:51-53``).  The upstream module is
absent from the reference; this file is the single
place the MI355X build describes it: which BasicBlockIR units exist, what the
state-dict keys/shapes are, and therefore what ``fr_set_param`` accepts.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

ARCHITECTURES = {
    "ir_18": (2, 2, 2, 2),
    "ir_34": (3, 4, 6, 3),
    "ir_50": (3, 4, 14, 3),
    "ir_101": (3, 13, 30, 3),
}
STAGE_WIDTHS = (64, 128, 256, 512)
EMBED_DIM = 512
INPUT_SIZE = (112, 112)


def block_specs(architecture: str) -> List[Tuple[int, int, int]]:
    """(in_channel, depth, stride) per BasicBlockIR unit (upstream ``get_blocks``)."""
    if architecture not in ARCHITECTURES:
        raise ValueError(f"Unknown architecture: {architecture}. "
                         f"Available: {['ir_50', 'ir_101']}")
    specs, in_ch = [], 64
    for units, depth in zip(ARCHITECTURES[architecture], STAGE_WIDTHS):
        specs.append((in_ch, depth, 2))
        specs.extend((depth, depth, 1) for _ in range(units - 1))
        in_ch = depth
    return specs


def _bn(prefix: str, c: int, affine: bool = True) -> List[Tuple[str, tuple]]:
    out = []
    if affine:
        out += [(prefix + ".weight", (c,)), (prefix + ".bias", (c,))]
    out += [(prefix + ".running_mean", (c,)), (prefix + ".running_var", (c,)),
            (prefix + ".num_batches_tracked", ())]
    return out


def state_dict_schema(architecture: str) -> "OrderedDict[str, tuple]":
    """Every AdaFace state-dict key (no ``model.`` prefix) -> shape."""
    s: List[Tuple[str, tuple]] = [("input_layer.0.weight", (64, 3, 3, 3))]
    s += _bn("input_layer.1", 64)
    s += [("input_layer.2.weight", (64,))]
    s += _bn("output_layer.0", 512)
    s += [("output_layer.3.weight", (EMBED_DIM, 512 * 7 * 7)), ("output_layer.3.bias", (EMBED_DIM,))]
    s += _bn("output_layer.4", EMBED_DIM, affine=False)
    for i, (cin, d, _stride) in enumerate(block_specs(architecture)):
        p = f"body.{i}."
        if cin != d:
            s += [(p + "shortcut_layer.0.weight", (d, cin, 1, 1))]
            s += _bn(p + "shortcut_layer.1", d)
        s += _bn(p + "res_layer.0", cin)
        s += [(p + "res_layer.1.weight", (d, cin, 3, 3))]
        s += _bn(p + "res_layer.2", d)
        s += [(p + "res_layer.3.weight", (d,))]
        s += [(p + "res_layer.4.weight", (d, d, 3, 3))]
        s += _bn(p + "res_layer.5", d)
    return OrderedDict(s)


def arcface_state_dict_schema(architecture: str) -> "OrderedDict[str, tuple]":
    """Every insightface ``arcface_torch`` IResNet key -> shape (ArcFace branch,
    ``face_embedder.py:64-88``; the ONNX exports come from this module).  Same unit
    counts as AdaFace; every stage's first unit has a conv1x1+BN ``downsample``."""
    s: List[Tuple[str, tuple]] = [("conv1.weight", (64, 3, 3, 3))]
    s += _bn("bn1", 64)
    s += [("prelu.weight", (64,))]
    specs = block_specs(architecture)
    stage, unit = 0, 0
    for i, (cin, d, stride) in enumerate(specs):
        if stride == 2 and i > 0:
            stage, unit = stage + 1, 0
        p = f"layer{stage + 1}.{unit}."
        s += _bn(p + "bn1", cin)
        s += [(p + "conv1.weight", (d, cin, 3, 3))]
        s += _bn(p + "bn2", d)
        s += [(p + "prelu.weight", (d,))]
        s += [(p + "conv2.weight", (d, d, 3, 3))]
        s += _bn(p + "bn3", d)
        if stride == 2:
            s += [(p + "downsample.0.weight", (d, cin, 1, 1))]
            s += _bn(p + "downsample.1", d)
        unit += 1
    s += _bn("bn2", 512)
    s += [("fc.weight", (EMBED_DIM, 512 * 7 * 7)), ("fc.bias", (EMBED_DIM,))]
    s += _bn("features", EMBED_DIM)
    return OrderedDict(s)


def schema_for(architecture: str, model_type: str = "adaface") -> "OrderedDict[str, tuple]":
    if model_type == "adaface":
        return state_dict_schema(architecture)
    if model_type == "arcface":
        return arcface_state_dict_schema(architecture)
    raise ValueError(f"Unknown model_type: {model_type}. Must be 'adaface' or 'arcface'")


def conv_macs_per_face(architecture: str, match_gallery: int = 0, model_type: str = "adaface") -> Dict[str, int]:
    """Multiply-accumulates per 112x112 face (forward-hook count of SURVEY.md §2).
    ArcFace adds the stage-1 conv1x1 downsample (AdaFace uses MaxPool2d(1,2) there)."""
    macs3 = 64 * 3 * 9 * 112 * 112  # stem
    macs1, hw = 0, 112
    for cin, d, stride in block_specs(architecture):
        macs3 += d * cin * 9 * hw * hw          # conv1 at input resolution
        ho = hw // stride
        macs3 += d * d * 9 * ho * ho            # conv2 carries the stride
        if cin != d or (model_type == "arcface" and stride == 2):
            macs1 += d * cin * ho * ho
        hw = ho
    fc = 512 * 49 * EMBED_DIM
    return {"conv3x3": macs3, "conv1x1": macs1, "fc": fc,
            "match": match_gallery * EMBED_DIM,
            "total": macs3 + macs1 + fc + match_gallery * EMBED_DIM}


def flop_per_face(architecture: str, match_gallery: int = 0, model_type: str = "adaface") -> float:
    return 2.0 * conv_macs_per_face(architecture, match_gallery, model_type)["total"]
