"""Stem kernel (preprocess + conv 3->64 + BN + PReLU) alone at B=256: time per launch and the
output write rate.  usage: python tools/stem_bench.py [--so path/to/libfrhip.so]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--so", default=None, help="a libfrhip.so build to load instead of the package's")
a = ap.parse_args()
from facerecognitionpipeline_amd import _lib  # noqa: E402
if a.so:
    _lib.LIB_PATH = os.path.abspath(a.so)
from tests import _frt  # noqa: E402

dev = torch.device("cuda", 0)
B = a.batch
img = torch.randint(0, 256, (B, 112, 112, 3), dtype=torch.uint8, device=dev)
lut = torch.linspace(-1, 1, 256, device=dev)
w = torch.randn(27, 64, device=dev) * 0.2
sc, sh, al = torch.rand(64, device=dev) + 0.5, torch.rand(64, device=dev) - 0.5, torch.full((64,), 0.25, device=dev)
y = torch.empty(B, 112, 112, 64, device=dev)
L = _frt.lib()
st = torch.cuda.current_stream().cuda_stream


def run():
    _frt._lib.check(L.frt_stem(_frt._p(img), B, _frt._p(lut), _frt._p(w), _frt._p(sc), _frt._p(sh), _frt._p(al),
                               _frt._p(y), st))


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(f"stem B={B}: {us:.1f} us, output {B * 112 * 112 * 64 * 4 / us / 1e6:.2f} TB/s")
# calibration: a plain fill of the same 822 MB (torch's kernel), same stream
e0.record()
for _ in range(20):
    y.fill_(1.0)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(f"fill of the output: {us:.1f} us, {B * 112 * 112 * 64 * 4 / us / 1e6:.2f} TB/s")
