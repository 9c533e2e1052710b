"""A timed-out F(4x4) ring hand-off is reported, never passed off as a result.

wino4_kernel's LDS counter waits are bounded (a lost hand-off must not hang the GPU).  When a
wait expires the kernel stores an error code into the handle's host-pinned error word and the
runtime fails the call with FR_ERR_HIP.  frt_set_wino4_poll_limit(0) makes every wait that does
not find its step ready at once expire, which forces the path here; every global access of the
kernel is range-checked, so the forced run computes garbage without faulting.
"""
import ctypes

import numpy as np
import pytest
import torch

from facerecognitionpipeline_amd import _lib, weights as W
from tests import _frt

pytestmark = pytest.mark.gpu
N = 64  # a whole-item grid (MODE 0) at stages 1-2 and split-K (MODE 1) at stages 3-4


@pytest.fixture
def handle():
    h = _lib.Handle("ir_50", "adaface", torch.device("cuda", 0), max_batch=N)
    h.load_state_dict(W.synthetic_state_dict("ir_50"))
    yield h
    _frt.lib().frt_set_wino4_poll_limit(-1)
    h.close()


def _embed_host(h, crops):
    out = np.zeros((crops.shape[0], 512), np.float32)
    rc = h._lib.fr_embed_host(h.h, crops.ctypes.data, crops.shape[0], 112, 112, out.ctypes.data, 1)
    return rc, out


def test_handoff_timeout_fails_fr_embed_host(handle):
    crops = np.ascontiguousarray(W.synthetic_crops(N, W.CROP_SEED_GALLERY))
    rc, good = _embed_host(handle, crops)
    assert rc == _lib.FR_OK
    _frt.lib().frt_set_wino4_poll_limit(0)
    rc, _ = _embed_host(handle, crops)
    assert rc == _lib.FR_ERR_HIP
    assert b"hand-off timed out" in handle._lib.fr_last_error(handle.h)
    # the word is cleared once reported; with the default bound the results are right again
    _frt.lib().frt_set_wino4_poll_limit(-1)
    rc, again = _embed_host(handle, crops)
    assert rc == _lib.FR_OK
    assert np.array_equal(again, good)


def test_handoff_timeout_fails_next_async_call(handle):
    dev = torch.device("cuda", 0)
    rgb = torch.from_numpy(W.synthetic_crops(N, W.CROP_SEED_GALLERY)).to(dev)
    out = torch.empty((N, 512), device=dev)
    _frt.lib().frt_set_wino4_poll_limit(0)
    handle.embed(rgb, out)  # asynchronous: queued, returns FR_OK
    torch.cuda.synchronize()
    _frt.lib().frt_set_wino4_poll_limit(-1)
    with pytest.raises(_lib.FrHipError, match="hand-off timed out"):
        handle.embed(rgb, out)  # reports the completed faulty work at entry
    handle.embed(rgb, out)  # reported once: this call runs
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()


def test_handoff_timeout_fails_frt_conv(handle):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    B, H, C = 8, 14, 64
    x = torch.randn(B, H, H, C, generator=g).to(dev)
    w = (torch.randn(C, 3, 3, C, generator=g) * 0.05).to(dev)
    res = torch.randn(B, H, H, C, generator=g).to(dev)
    post = (torch.ones(C, device=dev), torch.zeros(C, device=dev))
    _frt.conv2d_winograd(x, w, B, H, H, C, C, post=post, res=res, epi=2, m=4)
    _frt.lib().frt_set_wino4_poll_limit(0)
    with pytest.raises(_lib.FrHipError, match="hand-off timed out"):
        _frt.conv2d_winograd(x, w, B, H, H, C, C, post=post, res=res, epi=2, m=4)
    _frt.lib().frt_set_wino4_poll_limit(-1)
    _frt.conv2d_winograd(x, w, B, H, H, C, C, post=post, res=res, epi=2, m=4)


@pytest.mark.parametrize("cout", [96, 32])  # wide items (wino4w_kernel), tall items (wino4t_kernel)
def test_handoff_timeout_fails_item_shape_kernels(handle, cout):
    """The wide / tall item kernels' waits are bounded and reported the same way."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    B, H, C = 8, 20, 64
    x = torch.randn(B, H, H, C, generator=g).to(dev)
    w = (torch.randn(cout, 3, 3, C, generator=g) * 0.05).to(dev)
    post = (torch.ones(cout, device=dev), torch.zeros(cout, device=dev))
    L = _frt.lib()
    try:
        L.frt_set_wino4_shapes(2)
        L.frt_set_wino4_split(0)
        good = _frt.conv2d_winograd(x, w, B, H, H, C, cout, post=post, epi=0, m=4)
        L.frt_set_wino4_poll_limit(0)
        with pytest.raises(_lib.FrHipError, match="hand-off timed out"):
            _frt.conv2d_winograd(x, w, B, H, H, C, cout, post=post, epi=0, m=4)
        L.frt_set_wino4_poll_limit(-1)
        again = _frt.conv2d_winograd(x, w, B, H, H, C, cout, post=post, epi=0, m=4)
        assert torch.equal(again, good)
    finally:
        L.frt_set_wino4_poll_limit(-1)
        L.frt_set_wino4_shapes(1)
        L.frt_set_wino4_split(1)
