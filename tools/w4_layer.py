#!/usr/bin/env python3
"""Time one stride-1 3x3 conv layer through the Winograd test entry points (F(2x2) or F(4x4)).

usage: w4_layer.py [--m 4] [--B 256] [--H 14] [--cin 256] [--cout 256] [--epi 2] [--iters 20]
Prints average kernel time (HIP events around each launch, filter transform included once
outside the timed loop is NOT possible through frt_*, so the per-call time includes it:
use rocprofv3 --kernel-trace for the conv kernel alone).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests import _frt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--H", type=int, default=14)
    ap.add_argument("--cin", type=int, default=256)
    ap.add_argument("--cout", type=int, default=256)
    ap.add_argument("--epi", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="alternative libfrhip.so (tools/w4_variants.sh)")
    a = ap.parse_args()
    if a.lib:
        from facerecognitionpipeline_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(a.B, a.H, a.H, a.cin, generator=g).to(dev)
    w = (torch.randn(a.cout, 3, 3, a.cin, generator=g) / (9 * a.cin) ** 0.5).to(dev)
    ps, ph = torch.rand(a.cin).to(dev) + 0.5, torch.rand(a.cin).to(dev) - 0.5
    qs, qh = torch.rand(a.cout).to(dev) + 0.5, torch.rand(a.cout).to(dev) - 0.5
    al = torch.rand(a.cout).to(dev) * 0.3
    res = torch.randn(a.B, a.H, a.H, a.cout, generator=g).to(dev) if a.epi == 2 else None
    kw = dict(pre=(ps, ph) if a.epi == 1 else None, post=(qs, qh), prelu=al if a.epi == 1 else None, res=res,
              epi=a.epi, m=a.m)
    for _ in range(2):
        _frt.conv2d_winograd(x, w, a.B, a.H, a.H, a.cin, a.cout, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        _frt.conv2d_winograd(x, w, a.B, a.H, a.H, a.cin, a.cout, **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    flop = 2.0 * a.B * a.H * a.H * a.cout * 9 * a.cin
    print(f"m={a.m} B={a.B} H={a.H} {a.cin}->{a.cout} epi={a.epi}: {dt * 1e6:.1f} us per call "
          f"(incl. filter transform + alloc) = {flop / dt / 1e12:.1f} TF/s direct-equivalent")


if __name__ == "__main__":
    main()
