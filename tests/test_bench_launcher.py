"""CPU-only: bench.py --gpus N refuses to run fewer ranks than asked, and rejects inconsistent flags.

These paths end before any GPU call (torch.cuda.device_count() is 0 here), so they run on CPU.
The launch itself is covered on hardware by tests/test_gpu_bench_launch.py.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=300)


def test_more_gpus_than_visible_fails_loudly():
    p = _bench("--gpus", "64")
    assert p.returncode != 0
    assert "refusing to run fewer ranks" in p.stderr
    assert "{" not in p.stdout


def test_same_gpu_needs_gloo():
    p = _bench("--gpus", "2", "--same-gpu")
    assert p.returncode != 0 and "--dist-backend gloo" in p.stderr


def test_world_size_must_match_gpus():
    p = _bench("--gpus", "4", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
