#!/usr/bin/env python3
"""Time fr_detect on a batch of synthetic 1080p frames (seeded SCRFD-10G weights), optionally
against another libfrhip.so build (A/B of detector tile rules).  GPU only.
usage: python tools/det_time.py [--frames 32] [--reps 20] [--so lib.so ...]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--so", default=None)
    ap.add_argument("--shapes", type=int, default=None, help="frt_set_wino4_shapes before the detector is built")
    ap.add_argument("--nbg", type=int, default=None, help="frt_set_wino4_nbg (F(4x4) tile blocks per XCD item group)")
    a = ap.parse_args()
    from facerecognitionpipeline_amd import _lib
    if a.so:
        _lib.LIB_PATH = os.path.abspath(a.so)
    if a.shapes is not None or a.nbg is not None:
        from tests import _frt
        if a.shapes is not None:
            _lib.check(_frt.lib().frt_set_wino4_shapes(a.shapes))
        if a.nbg is not None:
            _lib.check(_frt.lib().frt_set_wino4_nbg(a.nbg))
    from facerecognitionpipeline_amd.face_recognition import FaceDetector
    from facerecognitionpipeline_amd.detector_arch import synthetic_detector_state_dict
    import bench
    dev = torch.device("cuda", 0)
    frames, _ = bench.c4_inputs(a.frames * 8, 8, dev)
    det = FaceDetector(device=dev, max_frames=min(32, frames.shape[0]), max_faces=64,
                       state_dict=synthetic_detector_state_dict())
    for _ in range(3):
        dets, counts = det.model.detect(frames, det.det_thresh, det.max_faces)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        dets, counts = det.model.detect(frames, det.det_thresh, det.max_faces)
    dt = (time.perf_counter() - t0) / a.reps
    tag = ("" if a.shapes is None else f" shapes={a.shapes}") + ("" if a.nbg is None else f" nbg={a.nbg}")
    print(f"{os.path.basename(a.so or 'libfrhip.so')}{tag}: {frames.shape[0]} frames {dt * 1e3:.3f} ms per detect "
          f"({frames.shape[0] / dt:.0f} frames/s), detections {int(counts.sum())}", flush=True)


if __name__ == "__main__":
    main()
