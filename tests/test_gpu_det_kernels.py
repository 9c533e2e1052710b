"""Detector kernels tested alone against PyTorch CPU ops of the same shape.

maxpool3_kernel (detect.hip): SCRFD's stem MaxPool2d(3, 2, 1) (scrfd.py's network, the pool after
the stem convs), NHWC f32, row strips of MP_R output rows per thread.  A max is exact, so the
result must equal torch's bitwise at every shape: odd and even sizes, a strip cut by the last
output row, maps smaller than a strip, negative inputs (the padding never wins).
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
