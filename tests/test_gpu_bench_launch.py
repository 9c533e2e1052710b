"""bench.py --gpus N on hardware: the launcher starts N ranks itself and the N>1 code path runs.

The driver measures the scaling curve as ``bench.py --gpus N`` (or under torchrun).  This box
has one GPU, so the two ranks share cuda:0 over gloo (``--same-gpu --dist-backend gloo``; RCCL
refuses two ranks on one GPU) -- everything else is bench.py's own N>1 path: rank-0 gallery
embed -> broadcast_gallery, barriers and the MAX-over-ranks timing, faces = world*batch*steps,
rank 0's single JSON line.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, timeout=420):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints, once
    return json.loads(lines[0])


def test_bench_gpus2_gloo_same_gpu():
    out = _run("--gpus", "2", "--dist-backend", "gloo", "--same-gpu")
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 512 and out["config"]["batch_per_gpu"] == 256
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["gallery_exchange"] == "gloo broadcast"
    assert out["config"]["ranks_share_gpu"] is True
    # value = world * batch * steps / (max-over-ranks seconds)
    secs = out["ms_per_step"] * out["steps"] / 1e3
    assert abs(out["value"] - 2 * 256 * 2 / secs) <= 1e-3 * out["value"] + 0.02
    assert out["top1_self_match"] == 1.0  # the worst rank's
    assert out["cpu_baseline"] is None
    # the gallery broadcast is measured (max over ranks) and the rank spread reported
    ex = out["gallery_exchange"]
    assert ex["collective"] == "broadcast" and ex["bytes"] == 1000 * 512 * 4
    assert ex["ms"] > 0 and ex["ms_steady"] > 0 and ex["reps"] == 3
    assert out["gallery_exchange_ms"] > 0 and out["gallery_exchange_GBps"] > 0
    assert 0 < out["rank_ms_per_step_min"] <= out["rank_ms_per_step_max"]
    assert abs(out["rank_ms_per_step_max"] - out["ms_per_step"]) <= 1e-3 * out["ms_per_step"] + 1e-3


def test_torchrun_form_without_gpus_flag():
    """The driver's torchrun form with no --gpus: WORLD_SIZE decides (advisor, round 4)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(REPO, "bench.py"),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist-backend", "gloo", "--same-gpu",
           "--exchange-reps", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 512
    assert out["gallery_exchange"]["reps"] == 1


def test_bench_gpus1_line_unchanged_shape():
    out = _run()
    # the library that ran is this tree's build, and the line says which one it is
    from facerecognitionpipeline_amd.build import build_id
    assert out["roofline"]["library_build"].endswith("build " + build_id())
    assert (out["roofline"]["traffic"] is None) == (out["roofline"]["traffic_source"] is None)
    assert out["n_gpus"] == 1 and out["config"]["global_batch"] == 256
    assert out["config"]["gallery_exchange"] == "none" and "ranks_share_gpu" not in out["config"]
    assert "gallery_exchange_ms" not in out and "rank_ms_per_step_min" not in out
    assert out["top1_self_match"] == 1.0
    assert out["roofline"]["bound"] == "mfma"
