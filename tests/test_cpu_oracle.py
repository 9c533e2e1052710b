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

BACKUPS = ("adaface_ir_101", "adaface_ir_50", "arcface_ir_101", "arcface_ir_50")


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
    assert idx.tolist() == [[1, 2, 4, 0]]
    assert val.tolist() == [[np.float32(0.9)] * 3 + [np.float32(0.5)]]


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
