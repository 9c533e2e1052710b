"""Winograd F(2x2,3x3) / F(4x4,3x3) convs (FR_CONV_WINOGRAD / _WINOGRAD4, stride-1 3x3) vs PyTorch CPU.

Same f32 tolerance as the direct kernel (tests/test_gpu_kernels.py): |d| <= 1e-5 * max|ref| + 1e-6,
and 4e-5 for F(4x4): its transforms scale a patch by up to 5 per direction in and 8 per direction
out (B^T, A^T entries) before the cancellations, so each output carries ~10x the rounding of F(2x2)
(measured 1.3e-5 at Cin = 256).  The whole network stays within 1e-5 per embedding element (last test).
The transforms add a few f32 roundings per output (input: 2 adds, output: 4 adds, filter: rounded
once from double), well inside that bar; the network-level check compares whole embeddings.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tests import _frt
from tests.test_gpu_kernels import _close, _nhwc, _rand

pytestmark = pytest.mark.gpu
DEV = "cuda"
REL = {2: 1e-5, 4: 4e-5}  # per-conv relative tolerance by Winograd output tile (module docstring)


def _wino_case(B, H, cin, cout, epi, seed, W=None, m=2):
    W = W or H
    x = _rand(B, cin, H, W, seed=seed)
    w = _rand(cout, cin, 3, 3, seed=seed + 1) / (cin * 9) ** 0.5
    pre_s, pre_b = _rand(cin, seed=seed + 2, lo=0.5, hi=1.5), _rand(cin, seed=seed + 3, lo=-0.2, hi=0.2)
    post_s, post_b = _rand(cout, seed=seed + 4, lo=0.5, hi=1.5), _rand(cout, seed=seed + 5, lo=-0.2, hi=0.2)
    al = _rand(cout, seed=seed + 6, lo=0.1, hi=0.4)
    xin = x * pre_s.view(1, -1, 1, 1) + pre_b.view(1, -1, 1, 1) if epi == 1 else x
    ref = F.conv2d(xin, w, padding=1) * post_s.view(1, -1, 1, 1) + post_b.view(1, -1, 1, 1)
    res = None
    if epi == 1:
        ref = torch.where(ref > 0, ref, ref * al.view(1, -1, 1, 1))
    else:
        r = _rand(B, cout, H, W, seed=seed + 7)
        ref = ref + r
        res = _nhwc(r).to(DEV)
    got = _frt.conv2d_winograd(_nhwc(x).to(DEV), w.permute(0, 2, 3, 1).contiguous().to(DEV), B, H, W, cin, cout,
                               pre=(pre_s.to(DEV), pre_b.to(DEV)) if epi == 1 else None,
                               post=(post_s.to(DEV), post_b.to(DEV)),
                               prelu=al.to(DEV) if epi == 1 else None, res=res, epi=epi, m=m)
    torch.cuda.synchronize()
    return got.cpu(), _nhwc(ref)


@pytest.mark.parametrize("B,H,cin,cout", [
    (2, 14, 64, 64),     # NBW=2, ragged last block (2*49 = 98 tiles)
    (3, 9, 128, 96),     # odd H (edge tiles half outside), Cout % 64 != 0 -> NBW=1
    (4, 7, 512, 512),    # stage-4 shape: 4x4 tiles of a 7x7 map
    (1, 28, 256, 256),   # stage-3 width
    (2, 56, 64, 64),     # stage-1 shape
    (1, 112, 64, 64),    # stage-1 unit-1 conv1 at input resolution
    (1, 1, 32, 32),      # 1x1 map: a single tile, 3 of its 4 outputs outside
    (5, 14, 256, 256),   # F(4x4) canvas: 4 images per canvas row, last canvas row ragged
    (3, 15, 32, 64),     # F(4x4) canvas with an even period (16 = 4 tiles, no separator needed)
])
@pytest.mark.parametrize("epi", [1, 2])
@pytest.mark.parametrize("m", [2, 4])
def test_winograd_conv_matches_cpu(B, H, cin, cout, epi, m):
    got, ref = _wino_case(B, H, cin, cout, epi, seed=300 + H + cin + epi, m=m)
    _close(got, ref, rel=REL[m])


@pytest.mark.parametrize("m", [2, 4])
def test_winograd_non_square_map(m):
    got, ref = _wino_case(2, 10, 64, 128, 1, seed=400, W=13, m=m)
    _close(got, ref, rel=REL[m])


@pytest.mark.parametrize("B,H,cin,cout", [
    (96, 14, 256, 256),  # 344 workgroups > CUs: a full round plus a partial one
    (32, 112, 64, 64),   # 1568 workgroups, Cin = 64 (4 K-steps)
])
def test_winograd4_multi_round(B, H, cin, cout):
    got, ref = _wino_case(B, H, cin, cout, 2, seed=500 + H, m=4)
    _close(got, ref, rel=REL[4])


@pytest.mark.parametrize("B,H,W,cin,cout", [
    (256, 14, 14, 256, 256),  # IR-101 stage 3 at B = 256: 900 items
    (128, 28, 28, 128, 128),  # stage 2, one lane of the headline batch
    (64, 56, 56, 64, 64),     # stage 1 at 56 (4 K-steps per item)
    (256, 7, 7, 512, 512),    # stage 4: 8 cout blocks, 4x4 tiles of a 7x7 map
    (300, 15, 15, 32, 64),    # Cin = 32 (2 K-steps), even period 16, one cout block
    (400, 9, 9, 64, 128),     # odd map, separator rows and columns, part-filled last canvas row
    (1023, 8, 14, 32, 64),    # pre-BN: 4 | H but not W, a partial last canvas row (separator row added)
])
@pytest.mark.parametrize("epi", [1, 2])
def test_winograd4_whole_item_grids(B, H, W, cin, cout, epi):
    """Launches of whole items (at least one per CU, several rounds, a part-empty last round)
    match the CPU conv and are deterministic run to run."""
    got, ref = _wino_case(B, H, cin, cout, epi, seed=1500 + H + cin + epi, W=W, m=4)
    _close(got, ref, rel=REL[4])
    again, _ = _wino_case(B, H, cin, cout, epi, seed=1500 + H + cin + epi, W=W, m=4)
    assert torch.equal(again, got), "F(4x4) is not run-to-run deterministic"


@pytest.mark.parametrize("B,H,cin,cout", [
    (1, 14, 256, 256),   # 8 workgroups -> 16 splits of 1 K-step
    (1, 7, 512, 512),    # 16 workgroups -> 16 splits of 2 K-steps
    (3, 28, 128, 128),   # 20 workgroups -> 8 splits
    (1, 112, 64, 64),    # 50 workgroups -> 4 splits of 1 K-step
    (2, 15, 32, 64),     # Cin = 32: 2 K-steps -> 2 splits
    (7, 14, 224, 512),   # 64 items -> 4 splits of 4, 4, 4, 2 K-steps
])
@pytest.mark.parametrize("epi", [1, 2])
def test_winograd4_split_k_small_grids(B, H, cin, cout, epi):
    """Small grids split the F(4x4) K loop over workgroups (raw partial outputs in compact
    slots); wino4_part_fixup_kernel sums them in split order and applies the epilogue.  Both
    paths match the CPU conv, and each other to the same bar."""
    L = _frt.lib()
    outs = {}
    try:
        for mode in (1, 0):  # split K loop + reduce pass, no split
            L.frt_set_wino4_split(mode)
            got, ref = _wino_case(B, H, cin, cout, epi, seed=700 + H + cin + epi, m=4)
            _close(got, ref, rel=REL[4])
            outs[mode] = got
    finally:
        L.frt_set_wino4_split(1)
    _close(outs[1], outs[0], rel=REL[4])
    again, _ = _wino_case(B, H, cin, cout, epi, seed=700 + H + cin + epi, m=4)
    assert torch.equal(again, outs[1]), "split-K result is not run-to-run deterministic"


def _det_case(B, H, W, cin, cout, epi, seed):
    """The detector's epilogues (no pre-BN): 0 affine, 1 affine + PReLU, 5 affine + residual + PReLU."""
    x = _rand(B, cin, H, W, seed=seed)
    w = _rand(cout, cin, 3, 3, seed=seed + 1) / (cin * 9) ** 0.5
    post_s, post_b = _rand(cout, seed=seed + 4, lo=0.5, hi=1.5), _rand(cout, seed=seed + 5, lo=-0.2, hi=0.2)
    al = _rand(cout, seed=seed + 6, lo=0.0, hi=0.4)
    ref = F.conv2d(x, w, padding=1) * post_s.view(1, -1, 1, 1) + post_b.view(1, -1, 1, 1)
    res = None
    if epi == 5:
        r = _rand(B, cout, H, W, seed=seed + 7)
        ref = ref + r
        res = _nhwc(r).to(DEV)
    if epi in (1, 5):
        ref = torch.where(ref > 0, ref, ref * al.view(1, -1, 1, 1))
    got = _frt.conv2d_winograd(_nhwc(x).to(DEV), w.permute(0, 2, 3, 1).contiguous().to(DEV), B, H, W, cin, cout,
                               post=(post_s.to(DEV), post_b.to(DEV)), prelu=al.to(DEV) if epi in (1, 5) else None,
                               res=res, epi=epi, m=4)
    torch.cuda.synchronize()
    return got.cpu(), _nhwc(ref)


@pytest.mark.parametrize("B,H,W,cin,cout", [
    (32, 40, 40, 80, 80),   # detector stride-16 tower conv at 32 frames: 200 wide items
    (16, 20, 20, 80, 96),   # a full 96-cout item, 25 items
    (3, 17, 23, 48, 80),    # odd map (separator rows / columns), 3 K-steps
    (1, 4, 4, 16, 96),      # one item, one K-step, 15 of its 16 tiles outside
    (64, 10, 10, 96, 96),   # canvas of 2 images per row, 6 K-steps
    (32, 56, 80, 32, 32),   # detector stem conv (28 -> 32 channels): 280 tall items, 2 K-steps
    (32, 20, 20, 80, 32),   # detector head output (30 -> 32) at stride 16: 25 tall items, 5 K-steps
    (3, 17, 23, 48, 16),    # 16 couts: the second cout block of every tall item idle
    (1, 5, 3, 16, 32),      # one tall item, its second 16-tile plane empty
    (9, 13, 13, 64, 32),    # 4 images per canvas row, ragged last canvas row, ragged last item
])
@pytest.mark.parametrize("epi", [0, 1, 5])
def test_winograd4_item_shapes(B, H, W, cin, cout, epi):
    """Layers of 65..96 couts without pre-BN run items of 16 tiles x 96 couts (wino4w_kernel: six
    MFMA waves, two transform waves of two 4-tile passes), layers of at most 32 items of 32 tiles x
    32 couts (wino4t_kernel: MFMA wave per cout block and 16-tile plane, four transform waves of
    two passes), instead of 64-cout items: both match the CPU conv, and the 64-cout items bitwise
    (every output's products and sums are the same)."""
    L = _frt.lib()
    outs = {}
    try:
        L.frt_set_wino4_split(0)  # whole items at every grid size (small grids would split K)
        for mode in (2, 0):  # shaped items at every grid size, 64-cout items only
            L.frt_set_wino4_shapes(mode)
            got, ref = _det_case(B, H, W, cin, cout, epi, seed=1700 + H + cin + cout + epi)
            _close(got, ref, rel=REL[4])
            outs[mode] = got
    finally:
        L.frt_set_wino4_shapes(1)
        L.frt_set_wino4_split(1)
    assert torch.equal(outs[2], outs[0]), "wide / tall items differ from 64-cout items"


@pytest.mark.parametrize("B,H,W", [(5, 8, 14), (3, 12, 5), (6, 16, 10)])
def test_winograd4_pre_bn_partial_canvas_row(B, H, W):
    """Folded pre-BN (U from w * scale, shift / scale added at in-image pixels) on canvases
    whose last row of images is partial and whose image rows have no separator of their own
    (4 | H, W needs one): launch_wino4 adds the separator row so the absent images' pixels stay
    out of every stored output's window."""
    got, ref = _wino_case(B, H, 32, 48, 1, seed=910 + B + H + W, W=W, m=4)
    _close(got, ref, rel=REL[4])


def test_winograd4_small_cin():
    """Cin = 32: one transform-pass channel group, two 16-channel K-steps."""
    got, ref = _wino_case(2, 12, 32, 32, 1, seed=420, m=4)
    _close(got, ref, rel=REL[4])


@pytest.mark.parametrize("m", [2, 4])
def test_winograd_is_deterministic(m):
    a, _ = _wino_case(2, 14, 128, 128, 2, seed=410, m=m)
    b, _ = _wino_case(2, 14, 128, 128, 2, seed=410, m=m)
    assert torch.equal(a, b)


@pytest.mark.parametrize("arch", ["ir_50", "ir_101"])
def test_network_winograd_vs_direct_vs_oracle(arch):
    """Whole IR network: F(2x2), F(4x4) and the direct path all within 1e-5 of the PyTorch-CPU
    oracle per embedding element, and identical top-5 gallery order."""
    from facerecognitionpipeline_amd import weights as W
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from oracle.adaface_net import load_oracle
    from oracle import reference_path as rp

    sd = W.synthetic_state_dict(arch)
    crops = W.synthetic_crops(24, seed=W.CROP_SEED_GALLERY)
    probes = W.probe_crops(crops, 24)
    ref_g = rp.extract_embeddings_batch(load_oracle(arch, sd), list(crops))
    ref_p = rp.extract_embeddings_batch(load_oracle(arch, sd), list(probes))
    out = {}
    for algo in ("winograd", "winograd4", "direct"):
        emb = FaceEmbedder(architecture=arch, state_dict=sd, device="cuda:0", max_batch=32, conv_algorithm=algo)
        g = emb.extract_embeddings_batch(list(crops))
        p = emb.extract_embeddings_batch(list(probes))
        assert np.abs(g - ref_g).max() <= 1e-5, (algo, np.abs(g - ref_g).max())
        assert np.abs(p - ref_p).max() <= 1e-5, (algo, np.abs(p - ref_p).max())
        out[algo] = (g, p)
        del emb
    ref_s = ref_p @ ref_g.T
    ref_top = np.argsort(-ref_s, axis=1, kind="stable")[:, :5]
    for algo, (g, p) in out.items():
        s = p @ g.T
        assert np.abs(s - ref_s).max() <= 1e-4, algo
        assert np.array_equal(np.argsort(-s, axis=1, kind="stable")[:, :5], ref_top), algo
