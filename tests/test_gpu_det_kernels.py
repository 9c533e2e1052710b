"""Detector kernels tested alone against PyTorch CPU ops of the same shape.

maxpool3_kernel (detect.hip): SCRFD's stem MaxPool2d(3, 2, 1) (scrfd.py's network, the pool after
the stem convs), NHWC f32, row strips of MP_R output rows per thread.  A max is exact, so the
result must equal torch's bitwise at every shape: odd and even sizes, a strip cut by the last
output row, maps smaller than a strip, negative inputs (the padding never wins).

The F(4x4) item shapes inside the detector network: with 8 frames the wide items run stage 2 and
the stride-8 head towers, the tall items the stem conv (more than one round of 64-cout items each),
and the forward must equal the 64-cout-items forward bitwise.
"""
import pytest
import torch
import torch.nn.functional as F

from tests import _frt

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H,W,C", [
    (32, 224, 320, 64),  # the C4 stem output (448 of 640 canvas rows at stride 2)
    (2, 320, 320, 64),   # a portrait frame's full canvas
    (3, 17, 23, 32),     # odd sizes: 9 x 12 outputs, the last strip one row long
    (1, 1, 1, 4),        # one pixel
    (5, 6, 2, 8),        # 3 output rows: a single, partial strip
    (4, 18, 9, 64),      # 9 output rows: two full strips and one row
])
def test_maxpool3_matches_torch(B, H, W, C):
    g = torch.Generator().manual_seed(B * 1000 + H + W + C)
    x = torch.randn(B, H, W, C, generator=g) - 0.5
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).contiguous()
    got = _frt.maxpool3(x.cuda())
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)


def test_detector_item_shapes_are_bitwise_the_64_cout_items():
    """The whole SCRFD-10G forward with the F(4x4) item shapes (wide items on its 80 / 88-channel
    layers, tall items on its stem conv and 30-channel outputs) against the same forward on 64-cout
    items only: every output is computed with the same products and sums, so the head maps are
    bitwise equal; and so are the detections."""
    import numpy as np
    from facerecognitionpipeline_amd.detector_arch import synthetic_detector_state_dict
    from facerecognitionpipeline_amd.face_recognition import FaceDetector
    det = FaceDetector(state_dict=synthetic_detector_state_dict(), max_frames=8)
    r = np.random.default_rng(11)
    frames = torch.from_numpy(r.integers(0, 256, (8, 1080, 1920, 3), dtype=np.uint8)).cuda()
    L = _frt.lib()
    try:
        L.frt_set_wino4_shapes(0)
        plain, _ = _frt.detector_forward(det.model, frames)
        plain = [x.clone() for x in plain]
        d0, c0 = det.model.detect(frames, 0.5, 256)
    finally:
        L.frt_set_wino4_shapes(1)
    shaped, _ = _frt.detector_forward(det.model, frames)
    d1, c1 = det.model.detect(frames, 0.5, 256)
    for a, b in zip(plain, shaped):
        assert torch.equal(a, b)
    assert np.array_equal(c0, c1) and np.array_equal(d0, d1)
