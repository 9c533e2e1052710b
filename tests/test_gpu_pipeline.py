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


def _check_topk_vs_reference(idx, sc, ref_idx, ref_sc, tie=1e-5):
    """Top-1 ids identical, every rank's score within SCORE_TOL; ranks 2..k identical ids
    except inside reference near-ties (adjacent scores closer than `tie`), where the id must
    come from the same tie group (fp32 summation order may swap them)."""
    assert np.array_equal(idx[:, 0], ref_idx[:, 0]), np.nonzero(idx[:, 0] != ref_idx[:, 0])
    assert np.abs(sc - ref_sc).max() <= SCORE_TOL
    n, k = ref_idx.shape
    swaps = 0
    for r in range(n):
        for j in range(1, k):
            if idx[r, j] == ref_idx[r, j]:
                continue
            group = [m for m in range(k) if abs(float(ref_sc[r, m]) - float(ref_sc[r, j])) < tie]
            assert idx[r, j] in ref_idx[r, group] or abs(float(sc[r, j]) - float(ref_sc[r, k - 1])) < tie, (r, j)
            swaps += 1
    return swaps


def test_c3_exact_config_vs_reference(golden_dir):
    """BASELINE.json configs[2] exactly -- IR-101, B = 256 crops, 1,000-row gallery, top-5 --
    through fr_embed_match, against the REFERENCE's own outputs on the same crops
    (tests/golden/c3_ir_101.npz: reference FaceEmbedder + GalleryManager.add_student/search).
    All 256 top-1 ids identical and |d score| <= 1e-4 at every rank, with the gallery embedded
    on the GPU and with the reference's gallery matrix."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    g = np.load(os.path.join(golden_dir, "c3_ir_101.npz"))
    gal = W.synthetic_crops(1000, int(g["gallery_seed"]))
    probes = W.probe_crops(gal, 256, seed=int(g["probe_seed"]))
    assert hashlib.sha256(gal.tobytes()).hexdigest() == str(g["gallery_crops_sha256"])
    assert hashlib.sha256(probes.tobytes()).hexdigest() == str(g["probe_crops_sha256"])
    emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=256)
    dev = emb.device
    ge = emb.embed_tensor(torch.from_numpy(gal).to(dev))
    assert np.abs(ge.cpu().numpy() - g["gallery_emb"]).max() <= EMB_TOL
    rgb = torch.from_numpy(probes).to(dev)
    idx = torch.empty((256, 5), dtype=torch.int32, device=dev)
    sc = torch.empty((256, 5), dtype=torch.float32, device=dev)
    e_out = torch.empty((256, 512), dtype=torch.float32, device=dev)
    for gallery in (ge, torch.from_numpy(g["gallery_emb"]).to(dev)):
        emb.model.gallery_set(gallery)
        emb.model.embed_match(rgb, 5, idx, sc, e_out)
        torch.cuda.synchronize()
        assert np.abs(e_out.cpu().numpy() - g["probe_emb"]).max() <= EMB_TOL
        _check_topk_vs_reference(idx.cpu().numpy(), sc.cpu().numpy(), g["search_idx"], g["search_score"])
    emb.model.gallery_set(torch.empty((0, 512), device=dev))


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
    for name in ("adaface_ir_101", "adaface_ir_50", "arcface_ir_101", "arcface_ir_50", "root_adaface_ir_50"):
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
        emb.extract_embedding(np.zeros((112, 112), np.uint8))        # not HxWx3
    with pytest.raises(ValueError):
        emb.extract_embedding(np.full((112, 112, 3), 0.5))           # fractional pixels: not LUT-exact
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


@pytest.mark.parametrize("hw", [(224, 224), (150, 130), (96, 96), (113, 111), (1, 1), (480, 640), (112, 200)])
def test_resize_crops_bit_exact(hw):
    """cv2.resize(crop, (112, 112), INTER_LINEAR) on the device (face_embedder.py:94-96) equals the
    fixed-point restatement oracle/scrfd.resize_linear_u8 byte for byte (parity vs cv2 unpinned)."""
    from facerecognitionpipeline_amd import _lib
    from oracle.scrfd import resize_linear_u8
    h = _lib.Handle("ir_50", "adaface", torch.device("cuda", 0), max_batch=4)
    r = np.random.default_rng(hw[0] * 1000 + hw[1])
    crops = r.integers(0, 256, size=(3,) + hw + (3,), dtype=np.uint8)
    out = torch.empty((3, 112, 112, 3), dtype=torch.uint8, device="cuda")
    h.resize_crops(torch.from_numpy(crops).cuda(), out)
    got = out.cpu().numpy()
    for i in range(3):
        assert np.array_equal(got[i], resize_linear_u8(crops[i], 112, 112)), (hw, i)


def test_resize_branch_embeddings_vs_reference(golden_dir):
    """Non-112 crops through the reference wrapper (tests/golden/resize_ir_50.npz: reference
    FaceEmbedder with the restated cv2.resize) vs the device resize + forward: mixed sizes in one
    extract_embeddings_batch, the single-crop API, and the C ABI host entry with 224x224 input."""
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    f = np.load(os.path.join(golden_dir, "resize_ir_50.npz"))
    r = np.random.Generator(np.random.PCG64(int(f["crop_seed"])))
    crops = [r.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for h, w in f["sizes"]]
    emb = FaceEmbedder(architecture="ir_50", model_path="synthetic", max_batch=8)
    got = emb.extract_embeddings_batch(crops)
    assert np.abs(got - f["emb"]).max() <= EMB_TOL
    assert np.abs(emb.extract_embedding(crops[6]) - f["emb"][6]).max() <= EMB_TOL
    # fr_embed_host with 224x224 input (the enrollment crop size, enroll_students.py:67-81,222)
    from facerecognitionpipeline_amd import _lib
    big = np.ascontiguousarray(np.stack(crops[:6]))
    out = np.empty((6, 512), np.float32)
    _lib.check(_lib.load().fr_embed_host(emb.model.h, big.ctypes.data, 6, 224, 224, out.ctypes.data, 1), emb.model.h)
    assert np.abs(out - f["emb"][:6]).max() <= EMB_TOL
    # a 224x224 float crop is refused: the reference resizes it in float64 (cv2.resize on the
    # original dtype, face_embedder.py:94-96), which the uint8 device resize does not restate
    with pytest.raises(ValueError, match="must already be 112x112"):
        emb.extract_embeddings_batch([crops[0].astype(np.float64)])


def test_fused_shortcut_matches_two_launches(arch_embedder):
    """The stride-2 conv2 of a block with a conv shortcut runs with that shortcut as one GEMM
    (BN scales folded into the weights, extra K-steps over the block input).  It must agree with
    the two-launch form (conv2 + BN + residual of the separately computed BN(conv1x1)) within the
    embedding bar; the default path's parity vs the reference is pinned by the tests above."""
    from tests import _frt
    arch, emb = arch_embedder
    crops = torch.from_numpy(W.synthetic_crops(24, seed=W.CROP_SEED_GALLERY)).cuda()
    L = _frt.lib()
    fused = emb.embed_tensor(crops).clone()
    assert L.frt_set_fuse_shortcut(emb.model.h, 0) == 0
    try:
        two = emb.embed_tensor(crops).clone()
    finally:
        assert L.frt_set_fuse_shortcut(emb.model.h, 1) == 0
    assert (fused - two).abs().max().item() <= EMB_TOL
    assert torch.equal(emb.embed_tensor(crops), fused)


def test_stride2_band_kernel_matches_implicit_gemm(arch_embedder):
    """The stage-1 stride-2 conv2 (MaxPool2d(1,2) shortcut) of batches >= 16 runs on its band
    kernel (conv_s2.hip); the whole network must agree with the implicit-GEMM form of that layer
    within the embedding bar, and be run-to-run deterministic."""
    from tests import _frt
    _arch, emb = arch_embedder
    crops = torch.from_numpy(W.synthetic_crops(24, seed=W.CROP_SEED_GALLERY)).cuda()
    L = _frt.lib()
    band = emb.embed_tensor(crops).clone()
    assert L.frt_set_s2_band(0) == 0
    try:
        gemm = emb.embed_tensor(crops).clone()
    finally:
        assert L.frt_set_s2_band(1) == 0
    assert (band - gemm).abs().max().item() <= EMB_TOL
    assert torch.equal(emb.embed_tensor(crops), band)
