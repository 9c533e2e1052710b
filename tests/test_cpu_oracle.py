"""CPU-only: pin the oracle to the reference's own outputs and fixtures.

* golden embed vectors: produced by the reference ``FaceEmbedder`` (tools/make_golden.py)
* backup fixtures: the reference's committed ``gallery/backups/*.json`` and the
  reference ``GalleryManager`` templates / search results on them.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from facerecognitionpipeline_amd import weights as W
from oracle import reference_path as rp
from oracle.adaface_net import build_model, load_oracle

# gallery/backups/*.json and backups/*.json (the fifth, "root_", is array-identical to
# gallery/backups' IR-50 AdaFace export; only its JSON timestamps differ)
BACKUPS = ("adaface_ir_101", "adaface_ir_50", "arcface_ir_101", "arcface_ir_50", "root_adaface_ir_50")


@pytest.mark.parametrize("arch,params", [("ir_50", 43_585_600), ("ir_101", 65_150_912)])
def test_oracle_parameter_count_matches_adaface(arch, params):
    m = build_model(arch)
    assert sum(p.numel() for p in m.parameters()) == params
    from facerecognitionpipeline_amd.arch import state_dict_schema
    assert set(state_dict_schema(arch)) == set(m.state_dict())


@pytest.mark.parametrize("arch", ["ir_50", "ir_101"])
def test_oracle_reproduces_reference_embeddings(arch, golden_dir):
    g = np.load(os.path.join(golden_dir, f"embed_{arch}.npz"))
    base = W.synthetic_crops(8, int(g["gallery_seed"]))
    probes = W.probe_crops(base, 8)
    assert hashlib.sha256(base.tobytes()).hexdigest() == str(g["gallery_crops_sha256"])
    assert hashlib.sha256(probes.tobytes()).hexdigest() == str(g["probe_crops_sha256"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    model = load_oracle(arch, W.synthetic_state_dict(arch))
    ge = rp.extract_embeddings_batch(model, list(base))
    pe = np.stack([rp.extract_embedding(model, p) for p in probes])
    # same op sequence as the reference on the same torch build: equal to fp32 rounding
    assert np.abs(ge - g["gallery_emb"]).max() <= 1e-6
    assert np.abs(pe - g["probe_emb"]).max() <= 1e-6
    for q, ids, sc in zip(pe, g["search_idx"], g["search_score"]):
        s = rp.search_scores(g["gallery_matrix"], q)
        top = np.argsort(s)[::-1][:5]
        assert np.array_equal(top, ids)
        assert np.abs(s[top] - sc).max() <= 1e-6


@pytest.mark.parametrize("name", BACKUPS)
def test_backup_template_kat(name, golden_dir):
    f = np.load(os.path.join(golden_dir, f"backup_{name}.npz"))
    ours = np.stack([rp.aggregate_template(e, "mean") for e in f["embeddings"]])
    assert np.array_equal(ours, f["ref_template"])                 # == reference GalleryManager, bit for bit
    assert np.abs(ours - f["stored_template"]).max() <= 5e-8        # == committed templates
    e = f["embeddings"].astype(np.float64)
    n = e.shape[1]
    avg = (np.einsum("snd,smd->s", e, e) - n) / (n * (n - 1))       # enroll_students.py:227-228
    ok = np.isfinite(f["avg_similarity"])
    assert np.abs(avg[ok] - f["avg_similarity"][ok]).max() <= 2e-7


@pytest.mark.parametrize("name", BACKUPS)
def test_backup_search_kat(name, golden_dir):
    f = np.load(os.path.join(golden_dir, f"backup_{name}.npz"))
    q = f["embeddings"].reshape(-1, f["embeddings"].shape[-1])
    idx, val = rp.topk_policy(np.stack([rp.search_scores(f["ref_template"], x) for x in q]), 5)
    assert np.array_equal(idx, f["search_idx"])
    assert np.abs(val - f["search_score"]).max() <= 1e-6
    if name == "adaface_ir_101":  # 184/184 self top-1
        assert (idx[:, 0] == np.repeat(np.arange(23), 8)).all()


def test_topk_policy_ties():
    s = np.array([[0.5, 0.9, 0.9, 0.1, 0.9]], np.float32)
    idx, val = rp.topk_policy(s, 4)
    assert idx.tolist() == [[4, 2, 1, 0]]       # = np.argsort(s, kind="stable")[::-1]
    assert val.tolist() == [[np.float32(0.9)] * 3 + [np.float32(0.5)]]
    r = np.random.default_rng(0)
    for n in (3, 16, 17, 100):
        t = r.integers(0, 4, (5, n)).astype(np.float32)   # many ties
        i, _ = rp.topk_policy(t, n)
        assert np.array_equal(i, np.argsort(t, axis=1, kind="stable")[:, ::-1])


def test_synthetic_weights_deterministic():
    a = W.synthetic_state_dict("ir_50")
    b = W.synthetic_state_dict("ir_50")
    assert all(np.array_equal(a[k], b[k]) for k in a)
    assert W.synthetic_state_dict("ir_50", seed=1)["input_layer.0.weight"][0, 0, 0, 0] != a["input_layer.0.weight"][0, 0, 0, 0]


def test_flop_accounting():
    from facerecognitionpipeline_amd.arch import conv_macs_per_face, flop_per_face
    assert conv_macs_per_face("ir_101")["total"] == 12_076_761_088       # 12.077 GMAC
    assert conv_macs_per_face("ir_50")["total"] == 6_296_485_888         # 6.296 GMAC
    assert abs(flop_per_face("ir_101", 1000) - 24.155e9) < 1e6


@pytest.mark.parametrize("arch", ["ir_50", "ir_101"])
def test_arcface_schema_matches_iresnet_restatement(arch):
    """ArcFace branch (face_embedder.py:64-88): the C ABI's IResNet key schema equals the
    restated insightface module's state dict; the synthetic weights load strictly."""
    from facerecognitionpipeline_amd.arch import arcface_state_dict_schema, flop_per_face
    from facerecognitionpipeline_amd import weights as W
    from oracle.iresnet import IResNet, load_oracle
    m = IResNet(arch)
    sd = m.state_dict()
    sc = arcface_state_dict_schema(arch)
    assert list(sd) == list(sc) and all(tuple(sd[k].shape) == sc[k] for k in sc)
    load_oracle(arch, W.synthetic_state_dict(arch, model_type="arcface"))
    # the stage-1 conv1x1 downsample is the only extra work vs AdaFace
    extra = 2.0 * 64 * 64 * 56 * 56
    assert flop_per_face(arch, model_type="arcface") - flop_per_face(arch) == extra


def test_arcface_preprocess_lut():
    """(x - 127.5) / 127.5 in float64 then float32 (face_embedder.py:105-110) is a 256-entry LUT."""
    from oracle import iresnet
    img = np.arange(256 * 3, dtype=np.int64).reshape(16, 16, 3) % 256
    img = img.astype(np.uint8)
    t = iresnet.preprocess(img)[0]
    lut = np.array([np.float32((v - 127.5) / 127.5) for v in range(256)], np.float32)
    assert np.array_equal(t, lut[img[:, :, ::-1]].transpose(2, 0, 1))


def test_oracle_reproduces_reference_c3_fixture(golden_dir):
    """Headline config (tests/golden/c3_ir_101.npz, reference-run): the oracle's embeddings of a
    sample of the 1,000 gallery / 256 probe crops, and the oracle search over the reference's
    full gallery matrix for all 256 probes, equal the reference's."""
    g = np.load(os.path.join(golden_dir, "c3_ir_101.npz"))
    gal = W.synthetic_crops(1000, int(g["gallery_seed"]))
    probes = W.probe_crops(gal, 256, seed=int(g["probe_seed"]))
    assert hashlib.sha256(gal.tobytes()).hexdigest() == str(g["gallery_crops_sha256"])
    assert hashlib.sha256(probes.tobytes()).hexdigest() == str(g["probe_crops_sha256"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    model = load_oracle("ir_101", W.synthetic_state_dict("ir_101"))
    sel = np.arange(0, 1000, 125)
    assert np.abs(rp.extract_embeddings_batch(model, list(gal[sel])) - g["gallery_emb"][sel]).max() <= 1e-6
    assert np.abs(rp.extract_embeddings_batch(model, list(probes[:8])) - g["probe_emb"][:8]).max() <= 1e-6
    ids = [f"S{i:04d}" for i in range(1000)]
    names = {s: s for s in ids}
    for q, ref_i, ref_s in zip(g["probe_emb"], g["search_idx"], g["search_score"]):
        res = rp.search(g["gallery_emb"], ids, names, q, top_k=5)
        assert [int(s[1:]) for s, _n, _v in res] == ref_i.tolist()
        assert np.array_equal(np.array([v for _s, _n, v in res], np.float32), ref_s)
    assert (g["search_idx"][:, 0] == np.arange(256)).all()  # probes are noisy copies of rows 0..255


def test_oracle_resize_branch_reproduces_reference(golden_dir):
    """face_embedder.py:94-96: non-112 crops (224x224 enrollment crops and odd sizes) through the
    reference wrapper with the restated INTER_LINEAR resize (tests/golden/resize_ir_50.npz)."""
    f = np.load(os.path.join(golden_dir, "resize_ir_50.npz"))
    r = np.random.Generator(np.random.PCG64(int(f["crop_seed"])))
    crops = [r.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for h, w in f["sizes"]]
    assert hashlib.sha256(np.concatenate([c.ravel() for c in crops]).tobytes()).hexdigest() == str(f["crops_sha256"])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    model = load_oracle("ir_50", W.synthetic_state_dict("ir_50"))
    assert np.abs(rp.extract_embeddings_batch(model, crops) - f["emb"]).max() <= 1e-6
