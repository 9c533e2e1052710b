"""conv_small.hip's serving kernel alone: µs per launch (back to back, HIP events) on the IR-101
batch-1 layer shapes.  --so loads a libfrhip.so variant (tools/lib_variant.py) instead.

    python tools/convs_bench.py [--so tools/wv/lib_X.so] [--n 1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=None)
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    from facerecognitionpipeline_amd import _lib
    if args.so:
        _lib.LIB_PATH = os.path.abspath(args.so)
    from tests import _frt
    n = args.n
    shapes = [  # (H, cin, cout, stride, cin2, epi, pre, name)
        (14, 256, 256, 1, 0, 2, False, "s3.conv2"), (14, 256, 256, 1, 0, 1, True, "s3.conv1"),
        (28, 128, 128, 1, 0, 2, False, "s2.conv2"), (56, 64, 64, 1, 0, 1, True, "s1.conv1@56"),
        (7, 512, 512, 1, 0, 2, False, "s4.conv2"), (112, 64, 64, 1, 0, 1, True, "s1.conv1@112"),
        (28, 256, 256, 2, 128, 0, False, "s3.conv2+sc/s2")]
    g = torch.Generator().manual_seed(0)
    for H, cin, cout, st, cin2, epi, pre, name in shapes:
        Ho = (H - 1) // st + 1
        x = torch.rand(n, H, H, cin, generator=g).cuda()
        x2 = torch.rand(n, H, H, cin2, generator=g).cuda() if cin2 else None
        w = (torch.rand(cout, 9 * cin + cin2, generator=g) - 0.5).cuda()
        ps, ph = torch.ones(cin).cuda(), torch.zeros(cin).cuda()
        qs, qh, al = torch.ones(cout).cuda(), torch.zeros(cout).cuda(), torch.full((cout,), 0.25).cuda()
        res = torch.rand(n, Ho, Ho, cout, generator=g).cuda() if epi == 2 else None
        run = lambda: _frt.conv2d_small(x, w, n, H, H, cin, cout, stride=st, x2=x2, cin2=cin2,
                                        pre=(ps, ph) if pre else None, post=(qs, qh),
                                        prelu=al if epi == 1 else None, res=res, epi=epi)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        print(f"{name:16s} n={n} {us:7.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
