"""Test infrastructure: write an insightface ``arcface_torch`` IResNet as an ONNX model
(protobuf wire format by hand: no onnx package here), in the two forms ``torch.onnx.export``
produces -- every BatchNormalization its own node (``fused=False``), or the BN after each Conv
folded into the Conv's weight and bias (``fused=True``, what eval-mode export does) -- so the
importer (facerecognitionpipeline_amd/onnx_import.py) can be checked against the state dict
the graph was written from.  Node order follows iresnet.py's forward (downsample after bn3)."""
from __future__ import annotations

import struct

import numpy as np

from facerecognitionpipeline_amd.arch import ARCHITECTURES, STAGE_WIDTHS

EPS = 1e-5


def _varint(x: int) -> bytes:
    x &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fn: int, wt: int) -> bytes:
    return _varint(fn << 3 | wt)


def _len(fn: int, payload: bytes) -> bytes:
    return _key(fn, 2) + _varint(len(payload)) + payload


def _int(fn: int, v: int) -> bytes:
    return _key(fn, 0) + _varint(v)


def _str(fn: int, s: str) -> bytes:
    return _len(fn, s.encode())


def tensor(name: str, a: np.ndarray, raw: bool = True) -> bytes:
    a = np.asarray(a, dtype=np.float32)
    out = b"".join(_int(1, d) for d in a.shape) + _int(2, 1) + _str(8, name)
    if raw:
        out += _len(9, a.astype("<f4").tobytes())
    else:
        out += _len(4, struct.pack(f"<{a.size}f", *a.ravel().tolist()))
    return out


def _attr_int(name: str, v: int) -> bytes:
    return _len(5, _str(1, name) + _int(3, v) + _int(20, 2))


def _attr_ints(name: str, vs) -> bytes:
    return _len(5, _str(1, name) + b"".join(_int(8, v) for v in vs) + _int(20, 7))


def _attr_float(name: str, v: float) -> bytes:
    return _len(5, _str(1, name) + _key(2, 5) + struct.pack("<f", v) + _int(20, 1))


def node(op: str, ins, outs, name: str = "", attrs: bytes = b"") -> bytes:
    return _len(1, b"".join(_str(1, i) for i in ins) + b"".join(_str(2, o) for o in outs) + _str(3, name) +
                _str(4, op) + attrs)


def _value_info(name: str) -> bytes:
    return _str(1, name)


class _G:
    def __init__(self, sd, fused: bool, raw: bool, wrap: str = ""):
        self.sd, self.fused, self.raw, self.wrap = sd, fused, raw, wrap
        self.nodes, self.inits, self.k = [], [], 0

    def t(self) -> str:
        self.k += 1
        return f"t{self.k}"

    def init(self, a) -> str:
        nm = f"w{len(self.inits)}"
        self.inits.append(tensor(nm, a, self.raw))
        if not self.wrap:
            return nm
        # weights fed through Identity / Cast(to=FLOAT) nodes, as some torch.onnx exports do for
        # shared or deduplicated parameters: "identity" wraps every one once; "mixed" rotates
        # Identity, Cast and a two-Identity chain
        forms = (("Identity",),) if self.wrap == "identity" else (("Identity",), ("Cast",), ("Identity", "Identity"))
        cur = nm
        for j, op in enumerate(forms[(len(self.inits) - 1) % len(forms)]):
            out = f"{nm}_{op.lower()}{j}"
            self.nodes.append(node(op, [cur], [out], out, _attr_int("to", 1) if op == "Cast" else b""))
            cur = out
        return cur

    def bn(self, x: str, key: str) -> str:
        y = self.t()
        ins = [x] + [self.init(self.sd[f"{key}.{n}"]) for n in ("weight", "bias", "running_mean", "running_var")]
        self.nodes.append(node("BatchNormalization", ins, [y], key, _attr_float("epsilon", EPS)))
        return y

    def conv_bn(self, x: str, wkey: str, bnkey: str, stride: int) -> str:
        w = np.asarray(self.sd[wkey], np.float32)
        k = w.shape[-1]
        attrs = (_attr_ints("kernel_shape", [k, k]) + _attr_ints("strides", [stride, stride]) +
                 _attr_ints("pads", [(k - 1) // 2] * 4) + _attr_ints("dilations", [1, 1]) + _attr_int("group", 1))
        y = self.t()
        if self.fused:  # what eval-mode export does: W' = W * g / sqrt(v + eps), b' = b - m * g / sqrt(v + eps)
            g, b, m, v = (np.asarray(self.sd[f"{bnkey}.{n}"], np.float64)
                          for n in ("weight", "bias", "running_mean", "running_var"))
            s = g / np.sqrt(v + EPS)
            wf = (w.astype(np.float64) * s[:, None, None, None]).astype(np.float32)
            bf = (b - m * s).astype(np.float32)
            self.nodes.append(node("Conv", [x, self.init(wf), self.init(bf)], [y], wkey, attrs))
            return y
        self.nodes.append(node("Conv", [x, self.init(w)], [y], wkey, attrs))
        return self.bn(y, bnkey)

    def prelu(self, x: str, key: str) -> str:
        y = self.t()
        a = np.asarray(self.sd[key], np.float32)
        self.nodes.append(node("PRelu", [x, self.init(a.reshape(-1, 1, 1))], [y], key))
        return y


def iresnet_onnx(sd, architecture: str, fused: bool = True, raw: bool = True, fc: str = "gemm",
                 features_folded: bool = False, wrap: str = "") -> bytes:
    """ModelProto bytes of the IResNet of state dict ``sd`` (arcface_torch keys).  ``fc``: "gemm"
    (Gemm, transB=1) or "matmul" (MatMul on the transposed weight + Add, another exporter form);
    ``features_folded``: the BatchNorm1d after the FC folded into its weight and bias; ``wrap``:
    "identity" / "mixed" feed the weights through Identity / Cast nodes (_G.init)."""
    g = _G(sd, fused, raw, wrap)
    x = g.conv_bn("data", "conv1.weight", "bn1", 1)
    x = g.prelu(x, "prelu.weight")
    for s, (units, _depth) in enumerate(zip(ARCHITECTURES[architecture], STAGE_WIDTHS)):
        for u in range(units):
            p = f"layer{s + 1}.{u}."
            stride = 2 if u == 0 else 1
            m = g.bn(x, p + "bn1")
            m = g.conv_bn(m, p + "conv1.weight", p + "bn2", 1)
            m = g.prelu(m, p + "prelu.weight")
            m = g.conv_bn(m, p + "conv2.weight", p + "bn3", stride)
            idt = g.conv_bn(x, p + "downsample.0.weight", p + "downsample.1", stride) if u == 0 else x
            y = g.t()
            g.nodes.append(node("Add", [m, idt], [y], p + "add"))
            x = y
    x = g.bn(x, "bn2")
    f = g.t()
    g.nodes.append(node("Flatten", [x], [f], "flatten", _attr_int("axis", 1)))
    d = g.t()
    g.nodes.append(node("Dropout", [f], [d], "dropout"))
    fw = np.asarray(sd["fc.weight"], np.float64)
    fb = np.asarray(sd["fc.bias"], np.float64)
    if features_folded:
        gm, bt, mu, var = (np.asarray(sd[f"features.{n}"], np.float64)
                           for n in ("weight", "bias", "running_mean", "running_var"))
        sc = gm / np.sqrt(var + EPS)
        fw, fb = fw * sc[:, None], (fb - mu) * sc + bt
    fw, fb = fw.astype(np.float32), fb.astype(np.float32)
    y = g.t()
    if fc == "gemm":
        g.nodes.append(node("Gemm", [d, g.init(fw), g.init(fb)], [y], "fc",
                            _attr_float("alpha", 1.0) + _attr_float("beta", 1.0) + _attr_int("transB", 1)))
    else:
        mm = g.t()
        g.nodes.append(node("MatMul", [d, g.init(np.ascontiguousarray(fw.T))], [mm], "fc.matmul"))
        g.nodes.append(node("Add", [mm, g.init(fb)], [y], "fc.add"))
    out = y if features_folded else g.bn(y, "features")
    graph = (b"".join(g.nodes) + _str(2, "iresnet") + b"".join(_len(5, t) for t in g.inits) +
             _len(11, _value_info("data")) + _len(12, _value_info(out)))
    return _int(1, 8) + _len(8, _str(1, "") + _int(2, 13)) + _len(7, graph)
