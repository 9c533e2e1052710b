"""End-to-end parity of the HIP hot path against the reference's own outputs.

Golden vectors (tests/golden/embed_*.npz) were produced by the REFERENCE
``FaceEmbedder`` / ``GalleryManager`` (tools/make_golden.py).  Bars, per
BASELINE.json north_star: identical top-k gallery ids, scores within 1e-4
(fp32).  Embedding elements are additionally held to 1e-5.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from facerecognitionpipeline_amd import weights as W

pytestmark = pytest.mark.gpu
SCORE_TOL = 1e-4
EMB_TOL = 1e-5


@pytest.fixture(scope="module", params=["ir_50", "ir_101"])
def arch_embedder(request):
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    return request.param, FaceEmbedder(architecture=request.param, model_path="synthetic", max_batch=256)


def _golden(golden_dir, arch):
    return np.load(os.path.join(golden_dir, f"embed_{arch}.npz"))


def test_golden_embeddings(arch_embedder, golden_dir):
    arch, emb = arch_embedder
    g = _golden(golden_dir, arch)
    base = W.synthetic_crops(8, int(g["gallery_seed"]))
    probes = W.probe_crops(base, 8)
    assert hashlib.sha256(base.tobytes()).hexdigest() == str(g["gallery_crops_sha256"])
    assert hashlib.sha256(probes.tobytes()).hexdigest() == str(g["probe_crops_sha256"])
    ge = emb.extract_embeddings_batch(list(base))
    pe = np.stack([emb.extract_embedding(p) for p in probes])
    assert ge.dtype == np.float32 and ge.shape == (8, 512)
    assert np.abs(ge - g["gallery_emb"]).max() <= EMB_TOL
    assert np.abs(pe - g["probe_emb"]).max() <= EMB_TOL
    # scores (probe x gallery) within the north-star bar
    assert np.abs(pe @ ge.T - g["probe_emb"] @ g["gallery_emb"].T).max() <= SCORE_TOL


def test_golden_search_top_ids(arch_embedder, golden_dir, tmp_path):
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    arch, emb = arch_embedder
    g = _golden(golden_dir, arch)
    base = W.synthetic_crops(8, int(g["gallery_seed"]))
    probes = W.probe_crops(base, 8)
    gm = GalleryManager(gallery_path=str(tmp_path / "g" / "students.npz"), device=emb.device, verbose=False)
    ge = emb.extract_embeddings_batch(list(base))
    for i in range(8):
        gm.add_student(f"S{i:03d}", f"N{i}", ge[i])
    pe = emb.extract_embeddings_batch(list(probes))
    res = gm.search_batch(pe, top_k=5)
    ids = np.array([[int(sid[1:]) for sid, _n, _s in r] for r in res])
    sc = np.array([[s for _sid, _n, s in r] for r in res], dtype=np.float32)
    assert np.array_equal(ids, g["search_idx"])
    assert np.abs(sc - g["search_score"]).max() <= SCORE_TOL
    # single-query API returns the reference tuple shape
    one = gm.search(pe[0], top_k=3)
    assert [r[0] for r in one] == [f"S{i:03d}" for i in g["search_idx"][0][:3]]
    assert isinstance(one[0][2], float)


def test_matches_oracle_and_batch_invariance_at_full_batch(arch_embedder):
    """B=256 (the bench batch): bitwise run-to-run determinism, batch invariance to 1e-6, 32 rows vs the CPU oracle."""
    from oracle.adaface_net import load_oracle
    from oracle import reference_path as rp
    arch, emb = arch_embedder
    crops = W.synthetic_crops(256, seed=777)
    dev = torch.from_numpy(crops).to(emb.device)
    full = emb.embed_tensor(dev).cpu().numpy()
    again = emb.embed_tensor(dev).cpu().numpy()
    assert np.array_equal(full, again), "forward is not deterministic"
    part = emb.embed_tensor(dev[100:105].contiguous()).cpu().numpy()
    # the stream-K schedule cuts a batch-dependent set of tiles along K, so rows of
    # different batch sizes may differ in the last bits (summation order), not more
    assert np.abs(full[100:105] - part).max() <= 1e-6, "forward is not batch-invariant"
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    model = load_oracle(arch, W.synthetic_state_dict(arch))
    ref = rp.extract_embeddings_batch(model, list(crops[:32]))
    assert np.abs(full[:32] - ref).max() <= EMB_TOL
    np.testing.assert_allclose(np.linalg.norm(full, axis=1), 1.0, atol=1e-5)


def test_embed_match_fused_equals_two_step(arch_embedder):
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    arch, emb = arch_embedder
    gal = W.synthetic_crops(64, seed=5)
    probes = W.probe_crops(gal, 48, seed=6)
    ge = emb.extract_embeddings_batch(list(gal))
    gm = GalleryManager(gallery_path="/tmp/_fr_fused/students.npz", device=emb.device, verbose=False)
    for i in range(64):
        gm.add_student(f"S{i}", f"N{i}", ge[i])
    dev = torch.from_numpy(probes).to(emb.device)
    idx = torch.empty((48, 5), dtype=torch.int32, device=emb.device)
    sc = torch.empty((48, 5), dtype=torch.float32, device=emb.device)
    e_out = torch.empty((48, 512), dtype=torch.float32, device=emb.device)
    emb.model.gallery_set(torch.from_numpy(ge).to(emb.device))
    emb.model.embed_match(dev, 5, idx, sc, e_out)
    i2, s2 = gm.search_device(e_out, 5)
    assert torch.equal(idx, i2) and torch.equal(sc, s2)
    assert (idx[:, 0].cpu().numpy() == np.arange(48)).all()  # probes are noisy copies of gallery rows


def test_match_large_gallery_vs_numpy():
    """C5-sized gallery (100k rows) against numpy fp32 sgemv + the tie policy."""
    from oracle.reference_path import topk_policy
    from facerecognitionpipeline_amd import _lib
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "embed_ir_101.npz"))
    E = W.expand_gallery(g["gallery_emb"], 100_000)
    rng = np.random.default_rng(3)
    Q = (E[rng.integers(0, 100_000, 16)] + 0.01 * rng.standard_normal((16, 512))).astype(np.float32)
    h = _lib.Handle("ir_50", "adaface", torch.device("cuda", 0), max_batch=1)
    h.gallery_set(torch.from_numpy(E).cuda())
    idx = torch.empty((16, 5), dtype=torch.int32, device="cuda")
    sc = torch.empty((16, 5), dtype=torch.float32, device="cuda")
    h.match(torch.from_numpy(Q).cuda(), 5, idx, sc)
    qn = Q / (np.linalg.norm(Q, axis=1, keepdims=True) + 1e-8)
    S = qn @ E.T
    ri, rv = topk_policy(S, 5)
    assert np.array_equal(idx.cpu().numpy()[:, 0], ri[:, 0])
    assert np.abs(sc.cpu().numpy() - rv).max() <= SCORE_TOL


def test_backup_fixture_search_on_gpu(golden_dir):
    """The reference's committed galleries: GPU search == reference GalleryManager.search."""
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    for name in ("adaface_ir_101", "adaface_ir_50", "arcface_ir_101", "arcface_ir_50"):
        f = np.load(os.path.join(golden_dir, f"backup_{name}.npz"))
        gm = GalleryManager(gallery_path=f"/tmp/_fr_b/{name}/students.npz", device="cuda:0", verbose=False)
        for sid, e in zip(f["student_ids"], f["embeddings"]):
            gm.add_student(str(sid), str(sid), e)
        res = gm.search_batch(f["embeddings"].reshape(-1, 512), top_k=5)
        ids = [[gm._ids.index(s) for s, _n, _sc in r] for r in res]
        sc = np.array([[x for _s, _n, x in r] for r in res], dtype=np.float32)
        assert np.array_equal(np.array(ids), f["search_idx"]), name
        assert np.abs(sc - f["search_score"]).max() <= SCORE_TOL, name


def test_edge_cases(arch_embedder, tmp_path):
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    arch, emb = arch_embedder
    out = emb.extract_embeddings_batch([])
    assert isinstance(out, np.ndarray) and out.size == 0
    with pytest.raises(ValueError):
        emb.extract_embedding(np.zeros((224, 224, 3), np.uint8))
    with pytest.raises(ValueError):
        FaceEmbedder(architecture="ir_7", model_path="synthetic")
    with pytest.raises(ValueError):
        FaceEmbedder(architecture="ir_50", model_type="nope")
    with pytest.raises(FileNotFoundError):  # face_embedder.py:72-73: the registry's ONNX file is absent
        FaceEmbedder(architecture="ir_50", model_type="arcface")
    with pytest.raises(RuntimeError):
        sd = W.synthetic_state_dict("ir_50")
        sd.pop("body.3.res_layer.4.weight")
        FaceEmbedder(architecture="ir_50", state_dict=sd)
    gm = GalleryManager(gallery_path=str(tmp_path / "e" / "s.npz"), device=emb.device, verbose=False)
    assert gm.search(np.ones(512, np.float32)) == []
    e = emb.extract_embeddings_batch(list(W.synthetic_crops(3, seed=9)))
    for i in range(3):
        gm.add_student(f"S{i}", f"N{i}", e[i])
    assert len(gm.search(e[0], top_k=10)) == 3      # top_k > G keeps G rows
    assert gm.search(e[0], top_k=0) == []
    assert len(gm.search(e[0], top_k=-1)) == 2       # argsort(...)[::-1][:-1]
    gm.delete_student("S0")
    assert gm.search(e[0], top_k=1)[0][0] != "S0"    # device copy refreshed after mutation
    # all-black and all-white crops stay finite
    ext = emb.extract_embeddings_batch([np.zeros((112, 112, 3), np.uint8), np.full((112, 112, 3), 255, np.uint8)])
    assert np.isfinite(ext).all()


@pytest.mark.parametrize("arch", ["ir_50", "ir_101"])
def test_bf16x3_mode_drift_vs_golden(arch, golden_dir):
    """Opt-in bf16x3 conv arithmetic: same top-5 ids as the reference, scores within 1e-4."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    g = _golden(golden_dir, arch)
    emb = FaceEmbedder(architecture=arch, model_path="synthetic", precision="bf16x3", max_batch=64)
    base = W.synthetic_crops(8, int(g["gallery_seed"]))
    probes = W.probe_crops(base, 8)
    ge = emb.extract_embeddings_batch(list(base))
    pe = emb.extract_embeddings_batch(list(probes))
    S = pe @ ge.T
    S_ref = g["probe_emb"] @ g["gallery_emb"].T
    assert np.abs(S - S_ref).max() <= SCORE_TOL
    assert np.array_equal(np.argsort(-S, axis=1)[:, :5], g["search_idx"])
    with pytest.raises(ValueError):
        FaceEmbedder(architecture=arch, model_path="synthetic", precision="fp8")


def test_torch_library_ops_match_python_api(arch_embedder):
    """torch.ops.frhip.* run the same kernels as FaceEmbedder / GalleryManager."""
    from facerecognitionpipeline_amd import torch_ops
    arch, emb = arch_embedder
    hid = torch_ops.register(emb)
    try:
        base = W.synthetic_crops(8)
        rgb = torch.from_numpy(W.probe_crops(base, 8)).to(emb.device)
        e = torch.ops.frhip.embed(rgb, hid, True)
        assert torch.equal(e, emb.embed_tensor(rgb))
        emb.model.gallery_set(emb.embed_tensor(torch.from_numpy(base).to(emb.device)))
        idx, score = torch.ops.frhip.match_topk(e, hid, 3)
        assert (idx[:, 0].cpu().numpy() == np.arange(8)).all()
        i2, s2, e2 = torch.ops.frhip.embed_match(rgb, hid, 3)
        assert torch.equal(i2, idx) and torch.equal(s2, score) and torch.equal(e2, e)
    finally:
        torch_ops.unregister(hid)
        emb.model.gallery_set(torch.empty((0, 512), device=emb.device))
