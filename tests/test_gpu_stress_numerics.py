"""Conv numerics under trained-like BatchNorm statistics (tests/_stress.py).

The default weights are well conditioned; trained IR networks carry BN scales spread
over ~4 orders of magnitude, heavy-tailed gammas and mixed-sign PReLU slopes, and the
F(4x4,3x3) transforms (entries up to 5 in, 8 out per direction) could amplify rounding
under them.  Bars (BASELINE.json north_star): identical top-1 gallery ids and cosine
scores within 1e-4 of the PyTorch-CPU oracle for every conv algorithm; each embedding
element within 2e-5 (the error is reported in the assertion message).
"""
import numpy as np
import pytest
import torch

from facerecognitionpipeline_amd import weights as W
from tests._stress import bn_scale_spread, trained_like_state_dict

pytestmark = pytest.mark.gpu
SCORE_TOL = 1e-4
EMB_TOL = 2e-5


@pytest.fixture(scope="module")
def stress_case():
    from oracle.adaface_net import load_oracle
    from oracle import reference_path as rp
    torch.set_num_threads(16)
    sd = trained_like_state_dict("ir_101")
    lo, hi = bn_scale_spread(sd)
    assert hi / lo > 1e3, (lo, hi)  # the profile really is spread
    crops = W.synthetic_crops(32, seed=W.CROP_SEED_GALLERY)
    probes = W.probe_crops(crops, 32)
    model = load_oracle("ir_101", sd)
    return sd, crops, probes, rp.extract_embeddings_batch(model, list(crops)), rp.extract_embeddings_batch(model, list(probes))


@pytest.mark.parametrize("algo", ["winograd4", "winograd", "direct"])
def test_trained_like_weights_parity(stress_case, algo):
    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    sd, crops, probes, ref_g, ref_p = stress_case
    emb = FaceEmbedder(architecture="ir_101", state_dict=sd, device="cuda:0", max_batch=64, conv_algorithm=algo)
    g = emb.extract_embeddings_batch(list(crops))
    p = emb.extract_embeddings_batch(list(probes))
    err = max(np.abs(g - ref_g).max(), np.abs(p - ref_p).max())
    S, S_ref = p @ g.T, ref_p @ ref_g.T
    serr = np.abs(S - S_ref).max()
    assert np.array_equal(S.argmax(1), S_ref.argmax(1)), (algo, err, serr)
    assert serr <= SCORE_TOL, (algo, "score", serr, "emb", err)
    assert err <= EMB_TOL, (algo, "emb", err)
