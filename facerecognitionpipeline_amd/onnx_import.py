"""ArcFace ``.onnx`` weights -> the IResNet state dict the HIP runtime takes.

The reference's ArcFace branch opens the ONNX export of insightface ``arcface_torch``
IResNet-50/100 with ``onnxruntime.InferenceSession`` (``face_embedder.py:64-88``) and runs it
(``:124-130``).  Neither onnx nor onnxruntime is a dependency here: this module reads the ONNX
protobuf wire format directly (ModelProto -> GraphProto -> NodeProto / TensorProto, field
numbers of the public ``onnx.proto``), walks the graph's dataflow from its input and maps it
onto the ``arcface_torch`` state-dict keys (``conv1``, ``bn1``, ``prelu``,
``layerS.U.{bn1,conv1,bn2,prelu,conv2,bn3,downsample.0,downsample.1}``, ``bn2``, ``fc``,
``features``) that ``schema_arcface`` in the runtime expects.

Both export forms are accepted:
  * unfused: every ``BatchNormalization`` is its own node;
  * fused (``torch.onnx.export`` in eval mode folds a BN that follows a Conv into the Conv's
    weights and bias): a conv with a bias and no BN after it becomes the conv weight plus an
    identity BatchNorm whose shift is the bias (scale exactly 1: ``running_var`` chosen so
    that ``var + 1e-5f == 1.0f``), which the runtime folds back to ``y = conv + bias``.
A node the IResNet graph does not contain (or a BN epsilon other than 1e-5) raises
``NotImplementedError`` naming it.  Parity against insightface's published ``.onnx`` files is
UNPINNED (no model files offline): the importer is tested on graphs written from seeded weights
in both forms (tests/test_onnx_import.py).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

EPS = 1e-5

# ---- protobuf wire format ---------------------------------------------------------------


def _varint(buf, i: int) -> Tuple[int, int]:
    v = shift = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v, i
        shift += 7


def _fields(buf):
    """(field number, wire type, value) of one message; length-delimited values are memoryviews"""
    mv = memoryview(buf)
    i, n = 0, len(mv)
    while i < n:
        key, i = _varint(mv, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(mv, i)
        elif wt == 1:
            v, i = mv[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(mv, i)
            v, i = mv[i:i + ln], i + ln
        elif wt == 5:
            v, i = mv[i:i + 4], i + 4
        else:
            raise ValueError(f"ONNX file: unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _packed_varints(v) -> List[int]:
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def _signed(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


# TensorProto: dims 1, data_type 2, float_data 4, int64_data 7, name 8, raw_data 9, data_location 14
def _tensor(buf) -> Tuple[str, np.ndarray]:
    dims: List[int] = []
    dtype, name, raw = 1, "", None
    floats: List[float] = []
    ints: List[int] = []
    for fn, wt, v in _fields(buf):
        if fn == 1:
            dims += [_signed(x) for x in (_packed_varints(v) if wt == 2 else [v])]
        elif fn == 2:
            dtype = v
        elif fn == 4:
            floats += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [struct.unpack("<f", v)[0]]
        elif fn == 7:
            ints += [_signed(x) for x in (_packed_varints(v) if wt == 2 else [v])]
        elif fn == 8:
            name = bytes(v).decode()
        elif fn == 9:
            raw = v
        elif fn == 14 and v == 1:
            raise NotImplementedError(f"ONNX tensor {name or '?'}: external data files are not supported")
    np_dt = {1: np.float32, 7: np.int64}.get(dtype)
    if np_dt is None:
        raise NotImplementedError(f"ONNX tensor {name}: data type {dtype} (only float32 / int64)")
    if raw is not None:
        arr = np.frombuffer(bytes(raw), dtype=np.dtype(np_dt).newbyteorder("<")).astype(np_dt)
    else:
        arr = np.asarray(floats if np_dt is np.float32 else ints, dtype=np_dt)
    return name, arr.reshape(dims) if dims else arr.reshape(())


# AttributeProto: name 1, f 2, i 3, t 5, floats 7, ints 8
def _attribute(buf):
    name, val = "", None
    for fn, wt, v in _fields(buf):
        if fn == 1:
            name = bytes(v).decode()
        elif fn == 2:
            val = struct.unpack("<f", v)[0]
        elif fn == 3:
            val = _signed(v)
        elif fn == 5:
            val = _tensor(v)[1]
        elif fn == 8:
            val = (val or []) + [_signed(x) for x in (_packed_varints(v) if wt == 2 else [v])]
        elif fn == 7:
            val = (val or []) + (list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2
                                 else [struct.unpack("<f", v)[0]])
    return name, val


class Node:
    __slots__ = ("op", "inputs", "outputs", "attrs", "name")

    def __init__(self, op, inputs, outputs, attrs, name):
        self.op, self.inputs, self.outputs, self.attrs, self.name = op, inputs, outputs, attrs, name

    def __repr__(self):
        return f"{self.op}({self.name or ','.join(self.outputs)})"


# NodeProto: input 1, output 2, name 3, op_type 4, attribute 5
def _node(buf) -> Node:
    ins, outs, attrs, name, op = [], [], {}, "", ""
    for fn, _wt, v in _fields(buf):
        if fn == 1:
            ins.append(bytes(v).decode())
        elif fn == 2:
            outs.append(bytes(v).decode())
        elif fn == 3:
            name = bytes(v).decode()
        elif fn == 4:
            op = bytes(v).decode()
        elif fn == 5:
            k, val = _attribute(v)
            attrs[k] = val
    return Node(op, ins, outs, attrs, name)


def read_graph(path: str):
    """(nodes, initializers by name, graph input names, graph output names) of an ONNX model"""
    with open(path, "rb") as f:
        data = f.read()
    graph = None
    for fn, _wt, v in _fields(data):  # ModelProto: graph 7
        if fn == 7:
            graph = v
    if graph is None:
        raise ValueError(f"{path}: no graph in the ONNX model")
    nodes, inits, g_in, g_out = [], {}, [], []
    for fn, _wt, v in _fields(graph):  # GraphProto: node 1, initializer 5, input 11, output 12
        if fn == 1:
            nodes.append(_node(v))
        elif fn == 5:
            k, arr = _tensor(v)
            inits[k] = arr
        elif fn in (11, 12):
            nm = ""
            for f2, _w2, v2 in _fields(v):  # ValueInfoProto: name 1
                if f2 == 1:
                    nm = bytes(v2).decode()
            (g_in if fn == 11 else g_out).append(nm)
    for n in nodes:  # Constant nodes are initializers too
        if n.op == "Constant" and "value" in n.attrs:
            inits[n.outputs[0]] = n.attrs["value"]
    return nodes, inits, [i for i in g_in if i not in inits], g_out


# ---- IResNet graph -> state dict --------------------------------------------------------


def _identity_var() -> np.float32:
    """running_var v with float32(v) + float32(1e-5) == 1.0f exactly (BN scale exactly 1)"""
    v = np.float32(1.0) - np.float32(EPS)
    for _ in range(8):
        s = np.float32(v) + np.float32(EPS)
        if s == np.float32(1.0):
            return np.float32(v)
        v = np.nextafter(v, np.float32(2.0) if s < 1 else np.float32(0.0), dtype=np.float32)
    raise AssertionError("no identity running_var")  # pragma: no cover


class _Walker:
    PASS = ("Identity", "Dropout")

    def __init__(self, nodes, inits):
        self.inits = inits
        self.consumers: Dict[str, List[Node]] = {}
        # Identity / Cast nodes by output: some exporters feed (shared or deduplicated) weights
        # through them instead of naming the initializer directly (init() follows the chain)
        self.producer: Dict[str, Node] = {n.outputs[0]: n for n in nodes
                                          if n.op in ("Identity", "Cast") and n.inputs and n.outputs}
        for n in nodes:
            if n.op == "Constant":
                continue
            for t in n.inputs:
                if t and t not in inits:
                    self.consumers.setdefault(t, []).append(n)
        self.sd: Dict[str, np.ndarray] = {}

    def only(self, t: str, what: str) -> Node:
        c = self.consumers.get(t, [])
        while len(c) == 1 and c[0].op in self.PASS:
            t = c[0].outputs[0]
            c = self.consumers.get(t, [])
        if len(c) != 1:
            raise NotImplementedError(f"ONNX IResNet: expected one {what} after tensor {t!r}, found {c}")
        return c[0]

    def init(self, node: Node, k: int) -> np.ndarray:
        if k >= len(node.inputs) or not node.inputs[k]:
            return None
        name = node.inputs[k]
        hops = 0
        while name not in self.inits and name in self.producer and hops < 64:
            p = self.producer[name]
            if p.op == "Cast" and p.attrs.get("to", 1) != 1:  # TensorProto.FLOAT
                raise NotImplementedError(f"ONNX IResNet: {node} input {name!r} is a Cast to type {p.attrs.get('to')}")
            name, hops = p.inputs[0], hops + 1
        if name not in self.inits:
            raise NotImplementedError(f"ONNX IResNet: {node} input {node.inputs[k]!r} is not an initializer "
                                      "(nor an Identity / Cast chain from one)")
        return np.asarray(self.inits[name], dtype=np.float32)

    def expect(self, node: Node, op: str) -> Node:
        if node.op != op:
            raise NotImplementedError(f"ONNX IResNet: expected {op}, found {node}")
        return node

    def bn(self, node: Node, key: str, c: int):
        eps = node.attrs.get("epsilon", 1e-5)
        if abs(eps - EPS) > 1e-9:
            raise NotImplementedError(f"ONNX IResNet: {node} has epsilon {eps} (the runtime folds BN with 1e-5)")
        names = ("weight", "bias", "running_mean", "running_var")
        for k, nm in enumerate(names):
            v = self.init(node, k + 1)
            if v is None or v.size != c:
                raise NotImplementedError(f"ONNX IResNet: {node} {nm} has {None if v is None else v.size} values, "
                                          f"expected {c}")
            self.sd[f"{key}.{nm}"] = v.reshape(c)

    def identity_bn(self, key: str, bias: Optional[np.ndarray], c: int):
        self.sd[f"{key}.weight"] = np.ones(c, np.float32)
        self.sd[f"{key}.bias"] = (np.zeros(c, np.float32) if bias is None else bias.reshape(c).astype(np.float32))
        self.sd[f"{key}.running_mean"] = np.zeros(c, np.float32)
        self.sd[f"{key}.running_var"] = np.full(c, _identity_var(), np.float32)

    def conv(self, node: Node, key: str, k: int, stride: int, cin: int, cout: int) -> Optional[np.ndarray]:
        self.expect(node, "Conv")
        w = self.init(node, 1)
        a = node.attrs
        pad = (k - 1) // 2
        if (w is None or w.shape != (cout, cin, k, k) or a.get("group", 1) != 1 or
                list(a.get("strides", [1, 1])) != [stride, stride] or
                list(a.get("pads", [0, 0, 0, 0])) != [pad] * 4 or list(a.get("dilations", [1, 1])) != [1, 1]):
            raise NotImplementedError(f"ONNX IResNet: {node} is not Conv{k}x{k}({cin}->{cout}, stride {stride}, "
                                      f"pad {pad}): weight {None if w is None else w.shape}, attributes {a}")
        self.sd[key] = w
        return self.init(node, 2)

    def conv_bn(self, t: str, wkey: str, bnkey: str, k: int, stride: int, cin: int, cout: int) -> str:
        """Conv (+ BatchNormalization, or its bias when the export folded the BN in) from tensor t"""
        node = self.only(t, f"Conv ({wkey})")
        bias = self.conv(node, wkey, k, stride, cin, cout)
        out = node.outputs[0]
        nxt = self.consumers.get(out, [])
        if len(nxt) == 1 and nxt[0].op == "BatchNormalization":
            if bias is not None and np.any(bias != 0):
                raise NotImplementedError(f"ONNX IResNet: {node} has a bias and a BatchNormalization after it")
            self.bn(nxt[0], bnkey, cout)
            return nxt[0].outputs[0]
        self.identity_bn(bnkey, bias, cout)
        return out

    def prelu(self, t: str, key: str, c: int) -> str:
        node = self.expect(self.only(t, "PRelu"), "PRelu")
        s = self.init(node, 1)
        if s is None or s.size != c:
            raise NotImplementedError(f"ONNX IResNet: {node} slope has {None if s is None else s.size} values, "
                                      f"expected {c}")
        self.sd[key] = s.reshape(c)
        return node.outputs[0]


def arcface_state_dict_from_onnx(path: str, architecture: str) -> Dict[str, np.ndarray]:
    """IResNet state dict (``arcface_torch`` keys) of an ArcFace ONNX export of ``architecture``."""
    from .arch import ARCHITECTURES, STAGE_WIDTHS
    if architecture not in ARCHITECTURES:
        raise ValueError(f"Unknown architecture: {architecture}")
    nodes, inits, g_in, _g_out = read_graph(path)
    if len(g_in) != 1:
        raise NotImplementedError(f"ONNX IResNet: expected one graph input, found {g_in}")
    wk = _Walker(nodes, inits)
    # stem: conv1 (3x3, 3 -> 64) -> bn1 -> prelu
    t = wk.conv_bn(g_in[0], "conv1.weight", "bn1", 3, 1, 3, 64)
    t = wk.prelu(t, "prelu.weight", 64)
    cin = 64
    for s, (units, depth) in enumerate(zip(ARCHITECTURES[architecture], STAGE_WIDTHS)):
        for u in range(units):
            p = f"layer{s + 1}.{u}."
            stride = 2 if u == 0 else 1
            cons = [c for c in wk.consumers.get(t, [])]
            bn1 = [c for c in cons if c.op == "BatchNormalization"]
            if len(bn1) != 1:
                raise NotImplementedError(f"ONNX IResNet: unit {p[:-1]}: expected its bn1 after {t!r}, found {cons}")
            wk.bn(bn1[0], p + "bn1", cin)
            m = wk.conv_bn(bn1[0].outputs[0], p + "conv1.weight", p + "bn2", 3, 1, cin, depth)
            m = wk.prelu(m, p + "prelu.weight", depth)
            m = wk.conv_bn(m, p + "conv2.weight", p + "bn3", 3, stride, depth, depth)
            add = wk.expect(wk.only(m, "Add"), "Add")
            other = [i for i in add.inputs if i != m]
            if len(other) != 1:
                raise NotImplementedError(f"ONNX IResNet: unit {p[:-1]}: {add} inputs {add.inputs}")
            if u == 0:  # downsample = Conv1x1(cin, depth, stride 2) -> BN, from the unit input
                convs = [c for c in cons if c.op == "Conv"]
                if len(convs) != 1:
                    raise NotImplementedError(f"ONNX IResNet: unit {p[:-1]}: expected a downsample Conv of {t!r}")
                wk.consumers[t] = [convs[0]]
                sc = wk.conv_bn(t, p + "downsample.0.weight", p + "downsample.1", 1, stride, cin, depth)
                if sc != other[0]:
                    raise NotImplementedError(f"ONNX IResNet: unit {p[:-1]}: the Add does not take the downsample")
            elif other[0] != t:
                raise NotImplementedError(f"ONNX IResNet: unit {p[:-1]}: the Add does not take the unit input")
            t, cin = add.outputs[0], depth
    # head: bn2 (2d) -> flatten -> fc (Gemm, or MatMul + Add) -> features (BN1d)
    bn2 = wk.expect(wk.only(t, "BatchNormalization"), "BatchNormalization")
    wk.bn(bn2, "bn2", 512)
    fl = wk.only(bn2.outputs[0], "Flatten")
    if fl.op not in ("Flatten", "Reshape"):
        raise NotImplementedError(f"ONNX IResNet: expected Flatten after bn2, found {fl}")
    fc = wk.only(fl.outputs[0], "Gemm")
    if fc.op == "Gemm":
        w, b = wk.init(fc, 1), wk.init(fc, 2)
        a = fc.attrs
        if a.get("transA", 0) or a.get("alpha", 1.0) != 1.0 or a.get("beta", 1.0) != 1.0:
            raise NotImplementedError(f"ONNX IResNet: {fc} attributes {a}")
        if not a.get("transB", 0):
            w = None if w is None else w.T
        out = fc.outputs[0]
    elif fc.op == "MatMul":
        w = wk.init(fc, 1)
        w = None if w is None else w.T
        add = wk.expect(wk.only(fc.outputs[0], "Add"), "Add")
        bname = [i for i in add.inputs if i in inits]
        b = np.asarray(inits[bname[0]], np.float32) if bname else None
        out = add.outputs[0]
    else:
        raise NotImplementedError(f"ONNX IResNet: expected Gemm after Flatten, found {fc}")
    if w is None or w.shape != (512, 512 * 49) or b is None or b.size != 512:
        raise NotImplementedError(f"ONNX IResNet: fc weight {None if w is None else w.shape}, bias "
                                  f"{None if b is None else b.size}: expected (512, 25088) and 512")
    wk.sd["fc.weight"] = np.ascontiguousarray(w, dtype=np.float32)
    wk.sd["fc.bias"] = b.reshape(512).astype(np.float32)
    feats = wk.consumers.get(out, [])
    if len(feats) == 1 and feats[0].op == "BatchNormalization":
        wk.bn(feats[0], "features", 512)
    else:  # features BN folded into the Gemm by the exporter
        wk.identity_bn("features", None, 512)
    return wk.sd
