"""Trained-like AdaFace weights for numerics stress tests (test infrastructure only).

The seeded weights of ``facerecognitionpipeline_amd.weights`` are well conditioned:
BN gamma ~ 1, running_var U(0.5, 1.5), PReLU 0.25.  Trained IR networks are not:
BatchNorm running variances follow the activations they saw (some channels nearly
dead, some large), gammas are spread over orders of magnitude, PReLU slopes vary
(some negative).  Those per-channel scales are folded into the Winograd filters and
epilogues, so they are what could amplify the F(4x4,3x3) transform rounding.

``trained_like_state_dict`` draws heavy-tailed gammas / betas / PReLU slopes, then
CALIBRATES every BatchNorm's running statistics on a seeded crop batch with the
PyTorch-CPU oracle (train-mode forward with momentum 1, dropout off), so running_mean
/ running_var are the statistics the activations really have -- the way training
leaves them -- and finally detunes each running_var by a log-uniform factor in
[1/4, 4] (train/test statistic mismatch).  The result spans running_var from ~1e-4 to
~1e2 and BN scales gamma/sqrt(var) over ~4 orders of magnitude, while the network
stays finite (every BN re-normalises what it sees).
"""
from __future__ import annotations

import zlib

import numpy as np
import torch

from facerecognitionpipeline_amd import weights as W

STRESS_SEED = 0x57E55


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(key.encode()), 7])))


def trained_like_state_dict(arch: str, seed: int = STRESS_SEED, calib: int = 16):
    from oracle.adaface_net import load_oracle
    sd = W.synthetic_state_dict(arch, seed=seed)
    for key in list(sd):
        r = _rng(seed, key)
        leaf = key.rsplit(".", 1)[1]
        shape = sd[key].shape
        is_prelu = ".res_layer.3." in key or key.startswith("input_layer.2.")
        if is_prelu:
            sd[key] = r.uniform(-0.15, 0.75, size=shape).astype(np.float32)       # spread slopes, some < 0
        elif leaf == "weight" and len(shape) == 1:
            sd[key] = np.exp(r.normal(0.0, 1.0, size=shape)).astype(np.float32)   # gamma: log-normal, ~e^+-2
        elif leaf == "bias" and len(shape) == 1 and key != "output_layer.3.bias":
            sd[key] = r.normal(0.0, 0.5, size=shape).astype(np.float32)           # beta
    model = load_oracle(arch, sd)
    bns = [m for m in model.modules() if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm1d))]
    for m in bns:
        m.momentum = 1.0           # running stats := this batch's statistics
    model.train()
    model.output_layer[1].eval()  # Dropout(0.4) off
    crops = W.synthetic_crops(calib, seed=seed)
    from oracle import reference_path as rp
    x = torch.cat([rp.preprocess(c) for c in crops])
    with torch.no_grad():
        model(x)
    model.eval()
    out = model.state_dict()
    res = {}
    for k, v in out.items():
        a = v.detach().cpu().numpy().copy()
        if k.endswith("running_var"):
            r = _rng(seed, k)
            a = (a * np.exp(r.uniform(np.log(0.25), np.log(4.0), size=a.shape))).astype(np.float32)
        res[k] = a
    return res


def bn_scale_spread(sd) -> tuple:
    """(min, max) over every BatchNorm of gamma / sqrt(running_var + 1e-5)."""
    lo, hi = np.inf, 0.0
    for k, v in sd.items():
        if k.endswith("running_var"):
            p = k[: -len("running_var")]
            g = sd.get(p + "weight", np.ones_like(v))
            s = np.abs(g) / np.sqrt(v.astype(np.float64) + 1e-5)
            lo, hi = min(lo, float(s.min())), max(hi, float(s.max()))
    return lo, hi
