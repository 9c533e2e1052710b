"""ArcFace branch (``model_type='arcface'``, face_embedder.py:64-88) on the HIP path.

The reference runs insightface IResNet ONNX exports under onnxruntime; both are
absent, so parity against the ONNX files is UNPINNED.  The checker is the
PyTorch-CPU restatement ``oracle/iresnet.py`` with the reference's ArcFace
preprocessing and normalisation (face_embedder.py:105-110, 163-182), on seeded
synthetic IResNet weights.  Bars as for AdaFace: embeddings within 1e-5, identical
top-k ids, scores within 1e-4.
"""
import numpy as np
import pytest
import torch

from facerecognitionpipeline_amd import weights as W

pytestmark = pytest.mark.gpu
EMB_TOL = 1e-5


@pytest.fixture(scope="module", params=["ir_50", "ir_101"])
def arc(request):
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from oracle.iresnet import load_oracle
    sd = W.synthetic_state_dict(request.param, model_type="arcface")
    emb = FaceEmbedder(architecture=request.param, model_type="arcface", state_dict=sd, max_batch=64)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    return request.param, emb, load_oracle(request.param, sd)


def test_arcface_embeddings_match_oracle(arc):
    from oracle import iresnet
    _arch, emb, model = arc
    base = W.synthetic_crops(8)
    probes = W.probe_crops(base, 8)
    crops = list(base) + list(probes)
    want = iresnet.extract_embeddings_batch(model, crops)
    got = emb.extract_embeddings_batch(crops)
    assert got.dtype == np.float32 and got.shape == (16, 512)
    assert np.abs(got - want).max() <= EMB_TOL
    # raw model output (normalize=False): no L2 inside the IResNet
    raw_want = iresnet.extract_embeddings_batch(model, crops[:4], normalize=False)
    raw_got = emb.extract_embeddings_batch(crops[:4], normalize=False)
    scale = np.abs(raw_want).max()
    assert np.abs(raw_got - raw_want).max() <= EMB_TOL * scale
    assert not np.allclose(np.linalg.norm(raw_got, axis=1), 1.0, atol=1e-3)
    # single-image path == batch path
    one = emb.extract_embedding(crops[3])
    assert np.abs(one - got[3]).max() <= 1e-6


def test_arcface_search_parity(arc, tmp_path):
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    from oracle import iresnet
    from oracle import reference_path as rp
    _arch, emb, model = arc
    base = W.synthetic_crops(8)
    probes = W.probe_crops(base, 8)
    ge_ref = iresnet.extract_embeddings_batch(model, list(base))
    pe_ref = iresnet.extract_embeddings_batch(model, list(probes))
    gm = GalleryManager(gallery_path=str(tmp_path / "g" / "s.npz"), device=emb.device, verbose=False)
    ge = emb.extract_embeddings_batch(list(base))
    for i in range(8):
        gm.add_student(f"S{i}", f"N{i}", ge[i])
    pe = emb.extract_embeddings_batch(list(probes))
    res = gm.search_batch(pe, top_k=3)
    ids = [f"S{i}" for i in range(8)]
    for i, r in enumerate(res):
        want = rp.search(ge_ref, ids, {s: s for s in ids}, pe_ref[i], top_k=3)
        assert [x[0] for x in r] == [x[0] for x in want]
        assert np.abs(np.array([x[2] for x in r]) - np.array([x[2] for x in want])).max() <= 1e-4


def test_arcface_onnx_model_path(tmp_path):
    """model_path='*.onnx' (the reference's ArcFace input, face_embedder.py:64-81): the graph's
    weights through onnx_import.  Unfused export: the same parameters as the state-dict path, so
    bit-identical embeddings; fused export (BN folded into the convs): the oracle's embeddings
    within 1e-5.  Graphs written by tests/_onnx_write.py (no real .onnx files offline: unpinned)."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    from oracle import iresnet
    from tests._onnx_write import iresnet_onnx
    sd = W.synthetic_state_dict("ir_50", model_type="arcface")
    crops = list(W.synthetic_crops(6))
    ref = FaceEmbedder(architecture="ir_50", model_type="arcface", state_dict=sd, max_batch=8)
    base = ref.extract_embeddings_batch(crops)
    for fused in (False, True):
        p = tmp_path / f"m{int(fused)}.onnx"
        p.write_bytes(iresnet_onnx(sd, "ir_50", fused=fused))
        e = FaceEmbedder(architecture="ir_50", model_type="arcface", model_path=str(p), max_batch=8)
        got = e.extract_embeddings_batch(crops)
        if not fused:
            assert np.array_equal(got, base)
        want = iresnet.extract_embeddings_batch(iresnet.load_oracle("ir_50", sd), crops)
        assert np.abs(got - want).max() <= EMB_TOL
    bad = tmp_path / "bad.onnx"
    bad.write_bytes(b"\x08\x07")
    with pytest.raises(ValueError):
        FaceEmbedder(architecture="ir_50", model_type="arcface", model_path=str(bad))


def test_arcface_checkpoint_roundtrip(tmp_path):
    """arcface_torch backbone.pth layout (module.-prefixed, as DDP saves it) loads with weights_only."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    sd = W.synthetic_state_dict("ir_50", model_type="arcface")
    p = tmp_path / "backbone.pth"
    torch.save({"module." + k: torch.as_tensor(np.asarray(v)) for k, v in sd.items()}, p)
    a = FaceEmbedder(architecture="ir_50", model_type="arcface", model_path=str(p), max_batch=8)
    b = FaceEmbedder(architecture="ir_50", model_type="arcface", state_dict=sd, max_batch=8)
    crops = list(W.synthetic_crops(2))
    assert np.array_equal(a.extract_embeddings_batch(crops), b.extract_embeddings_batch(crops))
