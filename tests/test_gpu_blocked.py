"""Channel-blocked activations between F(4x4) layers (frt_set_wino4_blocked, default on).

In forwards the serving kernel does not take (n > 2 crops), a block's conv1 output and the block
outputs passed between F(4x4) layers are stored [n][C/16][H][W][16] instead of NHWC; the stem's,
the stride-2 / shortcut kernels' and the head's tensors stay NHWC, so the conv2 at each seam reads
its residual in one layout and writes its output in the other (the RMIX instances).  Only addresses
change, so every embedding must be BITWISE the all-NHWC forward's: the headline batch (256 crops,
two concurrent lanes), one-lane batches whose stage-3/4 layers run split-K (partial slots + the
fixup kernel's addressing), graph replay, the stream-K tail, and the ArcFace IResNet schema (a
conv shortcut in every stage).
"""
import pytest
import torch

from facerecognitionpipeline_amd import weights as W

pytestmark = pytest.mark.gpu


def _both(embedder, crops, L):
    h = embedder.model
    assert L.frt_set_wino4_blocked(h.h, 0) == 0
    ref = embedder.embed_tensor(crops).clone()
    assert L.frt_set_wino4_blocked(h.h, 1) == 0
    got = embedder.embed_tensor(crops).clone()
    return got, ref


@pytest.mark.parametrize("arch,model_type", [("ir_101", "adaface"), ("ir_50", "arcface")])
def test_blocked_forward_is_bitwise_nhwc(arch, model_type):
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from tests import _frt
    L = _frt.lib()
    sd = W.synthetic_state_dict(arch, model_type=model_type)
    emb = FaceEmbedder(architecture=arch, model_type=model_type, state_dict=sd, device="cuda:0", max_batch=256)
    crops = torch.from_numpy(W.synthetic_crops(256, seed=W.CROP_SEED_GALLERY)).cuda()
    try:
        for n in ((256, 64, 9, 3) if arch == "ir_101" else (64, 5)):
            got, ref = _both(emb, crops[:n].contiguous(), L)
            assert torch.equal(got, ref), (arch, n, (got - ref).abs().max().item())
        if arch == "ir_101":
            # graph replay of a serving-sized forward (n <= graph_batch): capture + replays
            nhwc = None
            for on in (0, 1, 1, 1):
                assert L.frt_set_wino4_blocked(emb.model.h, on) == 0
                e = emb.embed_tensor(crops[:8].contiguous()).clone()
                nhwc = e if nhwc is None else nhwc
                assert torch.equal(e, nhwc)
    finally:
        assert L.frt_set_wino4_blocked(emb.model.h, 1) == 0


def test_blocked_plan_with_uneven_lanes():
    """lanes of 3 and 2 crops (lanes_min 2, n = 5).  The 2-crop lane is within the
    serving kernel's batch limit, so no F(4x4) layout bit may be planned for the forward (the
    serving branch does not read them): embeddings bitwise the all-NHWC forward's, and equal to
    one-lane forwards of each lane's crops."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from tests import _frt
    L = _frt.lib()
    sd = W.synthetic_state_dict("ir_101")
    emb = FaceEmbedder(architecture="ir_101", state_dict=sd, device="cuda:0", max_batch=8, lanes_min=2)
    crops = torch.from_numpy(W.synthetic_crops(5, seed=W.CROP_SEED_GALLERY)).cuda()
    try:
        got, ref = _both(emb, crops, L)
        assert torch.equal(got, ref), (got - ref).abs().max().item()
    finally:
        assert L.frt_set_wino4_blocked(emb.model.h, 1) == 0
    one = FaceEmbedder(architecture="ir_101", state_dict=sd, device="cuda:0", max_batch=8, lanes_min=0)
    parts = torch.cat([one.embed_tensor(crops[:3].contiguous()), one.embed_tensor(crops[3:].contiguous())])
    assert torch.equal(got, parts), (got - parts).abs().max().item()
