"""Kernel-level parity: each HIP kernel vs a PyTorch-CPU fp32 op of the same shape.

Tolerance: the conv kernel computes exact f32 products with f32 accumulation
(MFMA f32 = fmaf chain); only the summation order differs from PyTorch CPU, so
we allow |d| <= 1e-5 * max|ref| + 1e-6 (K <= 25088 terms).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests import _frt

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(*shape, generator=g) * (hi - lo) + lo


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _close(got, ref, rel=1e-5):
    ref = ref.float()
    tol = rel * ref.abs().max().item() + 1e-6
    d = (got.float() - ref).abs().max().item()
    assert d <= tol, f"max |diff| {d:.3e} > tol {tol:.3e}"


def _conv_case(B, H, cin, cout, k, stride, pad, epi, tile, use_pre, seed, nsplit=1):
    x = _rand(B, cin, H, H, seed=seed)
    w = _rand(cout, cin, k, k, seed=seed + 1) / (cin * k * k) ** 0.5
    pre_s, pre_b = _rand(cin, seed=seed + 2, lo=0.5, hi=1.5), _rand(cin, seed=seed + 3, lo=-0.2, hi=0.2)
    post_s, post_b = _rand(cout, seed=seed + 4, lo=0.5, hi=1.5), _rand(cout, seed=seed + 5, lo=-0.2, hi=0.2)
    al = _rand(cout, seed=seed + 6, lo=0.1, hi=0.4)
    xin = x * pre_s.view(1, -1, 1, 1) + pre_b.view(1, -1, 1, 1) if use_pre else x
    ref = F.conv2d(xin, w, stride=stride, padding=pad)
    Ho = ref.shape[2]
    res = None
    res_hw = (0, 0)
    if epi != 4:
        ref = ref * post_s.view(1, -1, 1, 1) + post_b.view(1, -1, 1, 1)
    if epi == 1:
        ref = torch.where(ref > 0, ref, ref * al.view(1, -1, 1, 1))
    if epi == 2:
        r = _rand(B, cout, Ho, Ho, seed=seed + 7)
        ref = ref + r
        res = _nhwc(r).to(DEV)
    if epi == 3:
        assert cin == cout and stride == 2
        ref = ref + x[:, :, ::2, ::2]
        res = _nhwc(x).to(DEV)
        res_hw = (H, H)
    wd = w.permute(0, 2, 3, 1).contiguous().to(DEV)
    got = _frt.conv2d(_nhwc(x).to(DEV), wd, B, H, H, cin, cout, k, k, stride, pad,
                      pre=(pre_s.to(DEV), pre_b.to(DEV)) if use_pre else None,
                      post=(post_s.to(DEV), post_b.to(DEV)) if epi != 4 else None,
                      prelu=al.to(DEV) if epi == 1 else None, res=res, res_hw=res_hw, epi=epi,
                      nsplit=nsplit, tile=tile)
    torch.cuda.synchronize()
    if nsplit > 1:
        got = got.sum(0)
    return got.cpu(), _nhwc(ref)


@pytest.mark.parametrize("tile", [0, 1])
def test_conv1_pre_bn_prelu(tile):
    # res_layer[0..3]: BN(in) -> conv3x3 s1 p1 -> BN -> PReLU; M = 2*14*14 = 392 (ragged tiles)
    got, ref = _conv_case(2, 14, 64, 64 if tile == 0 else 128, 3, 1, 1, epi=1, tile=tile, use_pre=True, seed=10)
    _close(got, ref)


def test_conv2_stride2_conv_shortcut_residual():
    # res_layer[4..5] stride 2 + residual from the conv1x1 shortcut tensor
    got, ref = _conv_case(3, 14, 128, 256, 3, 2, 1, epi=2, tile=1, use_pre=False, seed=20)
    _close(got, ref)


def test_conv2_stride2_maxpool_shortcut():
    # stage-1 unit-1: shortcut = MaxPool2d(1,2)(x), i.e. x[:, :, ::2, ::2]
    got, ref = _conv_case(2, 16, 64, 64, 3, 2, 1, epi=3, tile=0, use_pre=False, seed=30)
    _close(got, ref)


@pytest.mark.parametrize("B,H", [(2, 112), (3, 56), (1, 16), (17, 30)])
def test_conv2_stride2_maxpool_band_kernel(B, H):
    """The stage-1 stride-2 conv2 on its band kernel (conv_s2.hip): two output rows per workgroup,
    input rows staged in LDS for the 9 taps.  Against PyTorch CPU at the direct kernel's bar, incl.
    an odd output-row count (H = 30: a last band of one row) and an image of a single band."""
    seed = 80 + H
    x = _rand(B, 64, H, H, seed=seed)
    w = _rand(64, 64, 3, 3, seed=seed + 1) / (64 * 9) ** 0.5
    post_s, post_b = _rand(64, seed=seed + 4, lo=0.5, hi=1.5), _rand(64, seed=seed + 5, lo=-0.2, hi=0.2)
    ref = F.conv2d(x, w, stride=2, padding=1) * post_s.view(1, -1, 1, 1) + post_b.view(1, -1, 1, 1)
    ref = ref + x[:, :, ::2, ::2]
    xd = _nhwc(x).to(DEV)
    got = _frt.conv2d_s2band(xd, w.permute(0, 2, 3, 1).contiguous().to(DEV), B, H, H,
                             (post_s.to(DEV), post_b.to(DEV)), xd)
    torch.cuda.synchronize()
    _close(got.cpu(), _nhwc(ref))


@pytest.mark.parametrize("B,H,cin,cout,stride,cin2,epi,pre", [
    (1, 14, 256, 256, 1, 0, 1, True),     # IR stage-3 conv1 at batch 1: pre-BN + BN + PReLU
    (1, 14, 256, 256, 1, 0, 2, False),    # stage-3 conv2 + identity residual
    (2, 7, 512, 512, 1, 0, 2, False),     # stage 4, M = 98 (ragged last pixel block)
    (1, 56, 64, 64, 2, 0, 3, False),      # stage-1 unit-1 conv2: stride 2 + MaxPool2d(1,2) shortcut
    (1, 28, 128, 128, 2, 64, 0, False),   # stage-2 unit-1 conv2 + fused 1x1 s2 conv shortcut
    (3, 9, 32, 48, 1, 0, 1, True),        # odd sizes: 3 images of 9x9, Cout not a multiple of 128
])
def test_serving_conv_kernel(B, H, cin, cout, stride, cin2, epi, pre):
    """conv_small.hip's serving kernel (one workgroup per 16 pixels x 16 couts, whole K inside):
    against PyTorch CPU f32, incl. the fused shortcut (weights [cout][9 cin + cin2], the second
    input read at the output's stride) and ragged pixel blocks."""
    seed = 200 + H + cin + stride
    x = _rand(B, cin, H, H, seed=seed)
    w = _rand(cout, cin, 3, 3, seed=seed + 1) / (cin * 9) ** 0.5
    pre_s, pre_b = _rand(cin, seed=seed + 2, lo=0.5, hi=1.5), _rand(cin, seed=seed + 3, lo=-0.2, hi=0.2)
    post_s, post_b = _rand(cout, seed=seed + 4, lo=0.5, hi=1.5), _rand(cout, seed=seed + 5, lo=-0.2, hi=0.2)
    al = _rand(cout, seed=seed + 6, lo=0.1, hi=0.4)
    xin = x * pre_s.view(1, -1, 1, 1) + pre_b.view(1, -1, 1, 1) if pre else x
    acc = F.conv2d(xin, w, stride=stride, padding=1)
    Ho = acc.shape[2]
    wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)
    x2d = None
    if cin2:
        x2 = _rand(B, cin2, H, H, seed=seed + 8)
        w2 = _rand(cout, cin2, seed=seed + 9) / cin2 ** 0.5
        acc = acc + F.conv2d(x2, w2.view(cout, cin2, 1, 1), stride=stride)
        wk = torch.cat([wk, w2], 1)
        x2d = _nhwc(x2).to(DEV)
    ref = acc * post_s.view(1, -1, 1, 1) + post_b.view(1, -1, 1, 1)
    res = None
    if epi == 1:
        ref = torch.where(ref > 0, ref, ref * al.view(1, -1, 1, 1))
    if epi == 2:
        r = _rand(B, cout, Ho, Ho, seed=seed + 7)
        ref = ref + r
        res = _nhwc(r).to(DEV)
    if epi == 3:
        ref = ref + x[:, :, ::2, ::2]
        res = _nhwc(x).to(DEV)
    got = _frt.conv2d_small(_nhwc(x).to(DEV), wk.contiguous().to(DEV), B, H, H, cin, cout, stride=stride, x2=x2d,
                            cin2=cin2, pre=(pre_s.to(DEV), pre_b.to(DEV)) if pre else None,
                            post=(post_s.to(DEV), post_b.to(DEV)), prelu=al.to(DEV) if epi == 1 else None,
                            res=res, epi=epi)
    torch.cuda.synchronize()
    _close(got.cpu(), _nhwc(ref))


def test_conv2_identity_residual_tile0():
    got, ref = _conv_case(2, 12, 64, 64, 3, 1, 1, epi=2, tile=0, use_pre=False, seed=35)
    _close(got, ref)


def test_shortcut_conv1x1_stride2():
    got, ref = _conv_case(2, 14, 64, 128, 1, 2, 0, epi=0, tile=1, use_pre=False, seed=40)
    _close(got, ref)


def test_head_fc_as_7x7_conv_split_k():
    # output_layer: BN2d pre-affine + Linear(25088,512) == 7x7 valid conv; split-K over the 49 taps
    got, ref = _conv_case(5, 7, 512, 512, 7, 1, 0, epi=4, tile=1, use_pre=True, seed=50, nsplit=49)
    _close(got, ref)


def test_gemm_ragged_n_for_gallery_scores():
    # the matcher's S = Qn . E^T as a 1x1 conv over 1x1 images, N = G = 1000 (not a tile multiple)
    got, ref = _conv_case(7, 1, 512, 1000, 1, 1, 0, epi=4, tile=1, use_pre=False, seed=60)
    _close(got, ref)


def test_stem_matches_preprocess_and_input_layer():
    from oracle.reference_path import preprocess, preprocess_lut
    from facerecognitionpipeline_amd.weights import synthetic_crops
    imgs = synthetic_crops(3, seed=123)
    w = _rand(64, 3, 3, 3, seed=70) / 27 ** 0.5
    sc, sh = _rand(64, seed=71, lo=0.5, hi=1.5), _rand(64, seed=72, lo=-0.2, hi=0.2)
    al = _rand(64, seed=73, lo=0.1, hi=0.4)
    x = torch.cat([preprocess(i) for i in imgs])
    ref = F.conv2d(x, w, padding=1) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    ref = torch.where(ref > 0, ref, ref * al.view(1, -1, 1, 1))
    w27 = torch.empty(3, 3, 3, 64)
    for c in range(3):  # tensor channel c (BGR) is RGB channel 2-c
        w27[:, :, 2 - c, :] = w[:, c].permute(1, 2, 0)
    got = _frt.stem(torch.from_numpy(imgs).to(DEV), torch.from_numpy(preprocess_lut()).to(DEV),
                    w27.reshape(27, 64).contiguous().to(DEV), sc.to(DEV), sh.to(DEV), al.to(DEV))
    torch.cuda.synchronize()
    _close(got.cpu(), _nhwc(ref))


def test_preprocess_lut_is_bit_exact():
    from oracle.reference_path import preprocess, preprocess_lut
    img = np.arange(256, dtype=np.uint8).repeat(3 * 112 * 112 // 256 + 1)[: 112 * 112 * 3].reshape(112, 112, 3)
    t = preprocess(img)[0].numpy()           # reference float64 -> float32 path
    lut = preprocess_lut()
    assert np.array_equal(t, lut[img[:, :, ::-1].transpose(2, 0, 1)])


@pytest.mark.parametrize("G,k", [(1000, 5), (37, 3), (100_000, 5), (64, 64)])
def test_topk_matches_policy(G, k):
    from oracle.reference_path import topk_policy
    g = torch.Generator().manual_seed(G)
    s = torch.rand(9, G, generator=g)
    s[0, :] = 0.5            # all ties: highest indices first
    s[1, 3] = s[1, 7] = 2.0  # a tie at the top
    idx, val = _frt.topk(s.to(DEV), k)
    ri, rv = topk_policy(s.numpy(), k)
    assert np.array_equal(idx.cpu().numpy(), ri)
    assert np.array_equal(val.cpu().numpy(), rv)


@pytest.mark.parametrize("tile", list(range(10)))
def test_every_tile_config(tile):
    # ragged M (2*10*10 = 200) and N = 320 (not a multiple of 64/128/256) through each tile shape
    got, ref = _conv_case(2, 10, 64, 320, 3, 1, 1, epi=1, tile=tile, use_pre=True, seed=80 + tile)
    _close(got, ref)
    got, ref = _conv_case(2, 10, 96, 96, 3, 2, 1, epi=3, tile=tile, use_pre=False, seed=90 + tile)
    _close(got, ref)


def _conv_case_sk(B, H, cin, cout, k, stride, pad, epi, tile, use_pre, seed):
    got1, ref = _conv_case(B, H, cin, cout, k, stride, pad, epi, tile, use_pre, seed)  # grid mode
    import tests._frt as F_
    orig = F_.conv2d

    def sk(*a, **kw):
        kw["stream_k"] = 1
        return orig(*a, **kw)
    F_.conv2d = sk
    try:
        a, _ = _conv_case(B, H, cin, cout, k, stride, pad, epi, tile, use_pre, seed)
        b, _ = _conv_case(B, H, cin, cout, k, stride, pad, epi, tile, use_pre, seed)
    finally:
        F_.conv2d = orig
    return got1, a, b, ref


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 6, 7, 8, 9])
def test_stream_k_schedule_matches_and_is_deterministic(tile):
    # 8*28*28 = 6272 rows: fewer tiles than the persistent grid, so every tile is cut
    # across blocks and finished by the last arriver (slab sum in block order)
    grid, a, b, ref = _conv_case_sk(8, 28, 128, 256, 3, 1, 1, epi=1, tile=tile, use_pre=True, seed=100 + tile)
    _close(a, ref)
    assert torch.equal(a, b), "stream-K result depends on arrival order"
    # more tiles than blocks: whole-tile rounds + a stream-K tail; stride-2 residual epilogue
    grid, a, b, ref = _conv_case_sk(64, 28, 128, 128, 3, 2, 1, epi=2, tile=tile, use_pre=False, seed=110 + tile)
    _close(a, ref)
    assert torch.equal(a, b)


@pytest.mark.parametrize("tile", [1, 3, 4, 6, 7, 8])
@pytest.mark.parametrize("sk", [0, 1])
def test_bf16x3_split_precision(tile, sk):
    """Opt-in bf16x3 mode: x = hi + lo in bf16, three bf16 MFMAs per product, f32 accumulation.
    Per-product relative error <= ~2^-16, so the bar is 5e-5 * max|ref| (vs 1e-5 for f32)."""
    import tests._frt as F_
    orig = F_.conv2d

    def split(*a, **kw):
        kw["precision"] = 1
        kw["stream_k"] = sk
        return orig(*a, **kw)
    F_.conv2d = split
    try:
        got, ref = _conv_case(2, 14, 128, 256, 3, 1, 1, epi=1, tile=tile, use_pre=True, seed=200 + tile)
        _close(got, ref, rel=5e-5)
        got, ref = _conv_case(3, 14, 64, 64, 3, 2, 1, epi=3, tile=tile, use_pre=False, seed=210 + tile)
        _close(got, ref, rel=5e-5)
        got, ref = _conv_case(5, 7, 512, 512, 7, 1, 0, epi=4, tile=tile, use_pre=True, seed=220 + tile)
        _close(got, ref, rel=5e-5)
    finally:
        F_.conv2d = orig
