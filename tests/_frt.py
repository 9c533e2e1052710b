"""ctypes binding of include/frhip_testing.h (kernel-level test entry points)."""
import ctypes

import torch

from facerecognitionpipeline_amd import _lib

_P = ctypes.c_void_p
_I = ctypes.c_int


def lib():
    L = _lib.load()
    if not getattr(L, "_frt_ready", False):
        L.frt_conv2d.restype = _I
        L.frt_conv2d.argtypes = [_P, _P, _P] + [_I] * 9 + [_P] * 6 + [_I] * 7 + [_P]
        L.frt_conv2d_winograd.restype = _I
        L.frt_conv2d_winograd.argtypes = [_P, _P, _P] + [_I] * 5 + [_P] * 6 + [_I, _P]
        L.frt_conv2d_winograd4.restype = _I
        L.frt_conv2d_winograd4.argtypes = [_P, _P, _P] + [_I] * 5 + [_P] * 6 + [_I, _P]
        L.frt_set_wino4_split.restype = _I
        L.frt_set_wino4_split.argtypes = [_I]
        L.frt_set_conv2sc_tile.restype = _I
        L.frt_set_conv2sc_tile.argtypes = [_I]
        L.frt_maxpool3.restype = _I
        L.frt_maxpool3.argtypes = [_P, _I, _I, _I, _I, _P, _P]
        L.frt_set_wino4_nbg.restype = _I
        L.frt_set_wino4_nbg.argtypes = [_I]
        L.frt_set_wino4_shapes.restype = _I
        L.frt_set_wino4_shapes.argtypes = [_I]
        L.frt_set_wino4_max_split.restype = _I
        L.frt_set_wino4_max_split.argtypes = [_I]
        L.frt_set_wino4_poll_limit.restype = _I
        L.frt_set_wino4_poll_limit.argtypes = [_I]
        L.frt_set_s2_band.restype = _I
        L.frt_set_s2_band.argtypes = [_I]
        L.frt_conv2d_s2band.restype = _I
        L.frt_conv2d_s2band.argtypes = [_P, _P, _P, _I, _I, _I, _P, _P, _P, _P]
        L.frt_set_fuse_shortcut.restype = _I
        L.frt_set_fuse_shortcut.argtypes = [_P, _I]
        L.frt_set_small_conv.restype = _I
        L.frt_set_small_conv.argtypes = [_P, _I]
        L.frt_set_small_conv_pre_epilogue.restype = _I
        L.frt_set_small_conv_pre_epilogue.argtypes = [_P, _I]
        L.frt_set_small_conv_blocked.restype = _I
        L.frt_set_small_conv_blocked.argtypes = [_P, _I]
        L.frt_set_small_conv_pixels.restype = _I
        L.frt_set_small_conv_pixels.argtypes = [_P, _I]
        L.frt_set_wino4_blocked.restype = _I
        L.frt_set_wino4_blocked.argtypes = [_P, _I]
        L.frt_conv2d_small.restype = _I
        L.frt_conv2d_small.argtypes = [_P, _P, _P, _P] + [_I] * 7 + [_P] * 6 + [_I, _P]
        L.frt_stem.restype = _I
        L.frt_stem.argtypes = [_P, _I, _P, _P, _P, _P, _P, _P, _P]
        L.frt_topk.restype = _I
        L.frt_topk.argtypes = [_P, _I, _I, _I, _P, _P, _P]
        L.frt_detector_forward.restype = _I
        L.frt_detector_forward.argtypes = [_P, _P, _I, _I, _I, _P, _P, _P]
        L.frt_set_detector_row_reduction.restype = _I
        L.frt_set_detector_row_reduction.argtypes = [_P, _I]
        L._frt_ready = True
    return L


def _p(t):
    return None if t is None else t.data_ptr()


def conv2d(x, w, B, H, W, cin, cout, kh, kw, stride, pad, pre=None, post=None, prelu=None, res=None,
           res_hw=(0, 0), epi=0, nsplit=1, tile=1, stream_k=0, precision=0):
    """x: NHWC cuda f32, w: [cout][kh][kw][cin] cuda f32.  Returns y (NHWC) or partial slabs."""
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    y = torch.full((nsplit, B, Ho, Wo, cout), float("nan"), device=x.device)
    ps, ph = (pre if pre is not None else (None, None))
    qs, qh = (post if post is not None else (None, None))
    rc = lib().frt_conv2d(_p(x), _p(w), _p(y), B, H, W, cin, cout, kh, kw, stride, pad, _p(ps), _p(ph), _p(qs),
                          _p(qh), _p(prelu), _p(res), res_hw[0], res_hw[1], epi, nsplit, tile, stream_k, precision,
                          torch.cuda.current_stream().cuda_stream)
    _lib.check(rc)
    return y if nsplit > 1 else y[0]


def conv2d_winograd(x, w, B, H, W, cin, cout, pre=None, post=None, prelu=None, res=None, epi=1, m=2):
    """Winograd F(mxm,3x3) stride-1 conv (m = 2 or 4);
    x NHWC cuda f32, w [cout][3][3][cin] cuda f32."""
    y = torch.full((B, H, W, cout), float("nan"), device=x.device)
    ps, ph = (pre if pre is not None else (None, None))
    qs, qh = post
    fn = lib().frt_conv2d_winograd4 if m == 4 else lib().frt_conv2d_winograd
    rc = fn(_p(x), _p(w), _p(y), B, H, W, cin, cout, _p(ps), _p(ph), _p(qs), _p(qh),
            _p(prelu), _p(res), epi, torch.cuda.current_stream().cuda_stream)
    _lib.check(rc)
    return y


def stem(img, lut, w27x64, sc, sh, al):
    B = img.shape[0]
    y = torch.full((B, 112, 112, 64), float("nan"), device=img.device)
    _lib.check(lib().frt_stem(_p(img), B, _p(lut), _p(w27x64), _p(sc), _p(sh), _p(al), _p(y),
                              torch.cuda.current_stream().cuda_stream))
    return y


def maxpool3(x):
    """MaxPool2d(3, 2, 1) of x [B][H][W][C] (NHWC cuda f32) on the detector's kernel."""
    B, H, W, C = x.shape
    y = torch.full((B, (H - 1) // 2 + 1, (W - 1) // 2 + 1, C), float("nan"), device=x.device)
    _lib.check(lib().frt_maxpool3(_p(x), B, H, W, C, _p(y), torch.cuda.current_stream().cuda_stream))
    return y


def topk(scores, k):
    n, G = scores.shape
    idx = torch.empty((n, k), dtype=torch.int32, device=scores.device)
    val = torch.empty((n, k), dtype=torch.float32, device=scores.device)
    _lib.check(lib().frt_topk(_p(scores), n, G, k, _p(idx), _p(val), torch.cuda.current_stream().cuda_stream))
    return idx, val


def detector_forward(handle, frames):
    """Letterbox + SCRFD network on the GPU -> ([3 level maps [n,h,w,32]], canvas [n,640,640,3])."""
    n, H, W = frames.shape[:3]
    sizes = [(640 // s, 640 // s) for s in (8, 16, 32)]
    heads = torch.empty(sum(n * h * w * 32 for h, w in sizes), dtype=torch.float32, device=frames.device)
    canvas = torch.empty((n, 640, 640, 3), dtype=torch.uint8, device=frames.device)
    rc = lib().frt_detector_forward(handle.h, _p(frames), n, H, W, _p(heads), _p(canvas),
                                    torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, handle.h)
    out, off = [], 0
    for h, w in sizes:
        out.append(heads[off:off + n * h * w * 32].view(n, h, w, 32))
        off += n * h * w * 32
    return out, canvas


def set_detector_row_reduction(handle, on):
    _lib.check(lib().frt_set_detector_row_reduction(handle.h, int(on)), handle.h)


def conv2d_s2band(x, w, B, H, W, post, res):
    """The stage-1 stride-2 band conv: x, res NHWC [B,H,W,64] cuda f32, w [64][3][3][64]."""
    y = torch.full((B, H // 2, W // 2, 64), float("nan"), device=x.device)
    rc = lib().frt_conv2d_s2band(_p(x), _p(w), _p(y), B, H, W, _p(post[0]), _p(post[1]), _p(res),
                                 torch.cuda.current_stream().cuda_stream)
    _lib.check(rc)
    return y


def conv2d_small(x, w, B, H, W, cin, cout, stride=1, x2=None, cin2=0, pre=None, post=None, prelu=None, res=None,
                 epi=0):
    """conv_small.hip's serving kernel: x NHWC cuda f32, w [cout][9*cin + cin2] cuda f32."""
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.full((B, Ho, Wo, cout), float("nan"), device=x.device)
    ps, ph = (pre if pre is not None else (None, None))
    qs, qh = post
    rc = lib().frt_conv2d_small(_p(x), _p(x2), _p(w), _p(y), B, H, W, cin, cin2, cout, stride, _p(ps), _p(ph),
                                _p(qs), _p(qh), _p(prelu), _p(res), epi, torch.cuda.current_stream().cuda_stream)
    _lib.check(rc)
    return y
