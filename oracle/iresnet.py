"""Restatement of insightface ``arcface_torch`` IResNet (ArcFace branch) — ORACLE, test-only.

The reference's ``model_type='arcface'`` branch runs an ONNX export of
insightface's iresnet50/100 through onnxruntime (``face_embedder.py:64-88``):
``preprocess`` gives ``(bgr - 127.5) / 127.5`` in float64 then float32
(``:105-110``), ``InferenceSession.run`` returns the raw 512-d feature
(``:124-130``, ``:163-174``) and ``normalize=True`` divides by ``||e|| + 1e-8``
(``:133-134``, ``:177-180``).  Neither onnxruntime nor the ``.onnx`` files exist
here, so this module restates the published PyTorch definition the exports come
from (deepinsight/insightface ``recognition/arcface_torch/backbones/iresnet.py``,
not vendored, no version pin) with the same state-dict keys:

    conv1 = Conv3x3(3,64,s1,p1,nobias) -> bn1 = BN2d(64) -> prelu = PReLU(64)
    layer{1..4}[u] = IBasicBlock(inplanes, planes, stride)
        bn1(in) -> conv1 3x3 s1 -> bn2 -> prelu -> conv2 3x3 stride -> bn3
        downsample = Conv1x1(inplanes, planes, stride) -> BN2d   (first unit of
                     every stage: stride 2 everywhere, so stage 1 too, unlike
                     AdaFace's MaxPool2d(1,2) there)
        out = res + identity/downsample
    bn2 = BN2d(512) -> flatten (NCHW) -> dropout(p=0) -> fc = Linear(25088,512)
    features = BN1d(512, affine=True);  no L2 inside the model.

All BatchNorms use eps=1e-5.  Parity against the ONNX files is UNPINNED (no
onnxruntime, no model files): this restatement is checked only for its shape
contract (tests/test_cpu_oracle.py) and is the checker of the GPU ArcFace path.
"""
from __future__ import annotations

import torch
from torch import nn

# units per stage: iresnet50 / iresnet100 (arcface_torch get_model('r50' / 'r100'))
STAGE_UNITS = {
    "ir_18": (2, 2, 2, 2),
    "ir_34": (3, 4, 6, 3),
    "ir_50": (3, 4, 14, 3),
    "ir_101": (3, 13, 30, 3),
}
STAGE_WIDTHS = (64, 128, 256, 512)


class IBasicBlock(nn.Module):
    def __init__(self, inplanes: int, planes: int, stride: int, downsample: bool):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(inplanes, eps=1e-05)
        self.conv1 = nn.Conv2d(inplanes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes, eps=1e-05)
        self.prelu = nn.PReLU(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes, eps=1e-05)
        self.downsample = (nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False),
                                         nn.BatchNorm2d(planes, eps=1e-05)) if downsample else None)

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.bn3(self.conv2(self.prelu(self.bn2(self.conv1(self.bn1(x))))))
        return out + identity


class IResNet(nn.Module):
    def __init__(self, architecture: str):
        super().__init__()
        if architecture not in STAGE_UNITS:
            raise ValueError(f"Unknown architecture: {architecture}")
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64, eps=1e-05)
        self.prelu = nn.PReLU(64)
        inplanes = 64
        for s, (units, planes) in enumerate(zip(STAGE_UNITS[architecture], STAGE_WIDTHS)):
            blocks = [IBasicBlock(inplanes, planes, 2, True)]
            blocks += [IBasicBlock(planes, planes, 1, False) for _ in range(units - 1)]
            setattr(self, f"layer{s + 1}", nn.Sequential(*blocks))
            inplanes = planes
        self.bn2 = nn.BatchNorm2d(512, eps=1e-05)
        self.dropout = nn.Dropout(p=0.0)
        self.fc = nn.Linear(512 * 7 * 7, 512)
        self.features = nn.BatchNorm1d(512, eps=1e-05)

    def forward(self, x):
        x = self.prelu(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.bn2(x), 1)
        return self.features(self.fc(self.dropout(x)))


def load_oracle(architecture: str, state_dict) -> IResNet:
    m = IResNet(architecture)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict.items()})
    return m.eval()


def preprocess(face_image):
    """``face_embedder.py:105-110``: BGR, (x - 127.5) / 127.5 in float64, CHW, float32."""
    import numpy as np
    bgr = face_image[:, :, ::-1]
    bgr = (bgr - 127.5) / 127.5
    return np.expand_dims(bgr.transpose(2, 0, 1), axis=0).astype(np.float32)


def extract_embeddings_batch(model, face_images, normalize: bool = True, batch_size: int = 32):
    """``face_embedder.py:163-182`` with the ORT session replaced by the restated module."""
    import numpy as np
    if len(face_images) == 0:
        return np.array([])
    outs = []
    with torch.no_grad():
        for i in range(0, len(face_images), batch_size):
            batch = np.vstack([preprocess(f) for f in face_images[i:i + batch_size]])
            outs.append(model(torch.from_numpy(batch)).numpy())
    e = np.vstack(outs)
    if normalize:
        e = e / (np.linalg.norm(e, axis=1, keepdims=True) + 1e-8)
    return e
