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
    # no GPU here: either the KFD / amdsmi count is 0, or there is nothing to count with
    assert "refusing to run fewer ranks" in p.stderr or "cannot count the visible GPUs" in p.stderr
    assert "{" not in p.stdout


def test_same_gpu_needs_gloo():
    p = _bench("--gpus", "2", "--same-gpu")
    assert p.returncode != 0 and "--dist-backend gloo" in p.stderr


def test_world_size_must_match_gpus():
    p = _bench("--gpus", "4", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_torchrun_without_gpus_flag_takes_world_size():
    """``torchrun --nproc-per-node N bench.py`` (no --gpus) runs as rank r of N."""
    b = _bench_module()
    assert b.resolve_world(None, {"WORLD_SIZE": "2"}) == 2
    assert b.resolve_world(2, {"WORLD_SIZE": "2"}) == 2
    assert b.resolve_world(None, {}) == 1
    assert b.resolve_world(4, {}) == 4
    import pytest
    with pytest.raises(SystemExit):
        b.resolve_world(4, {"WORLD_SIZE": "2"})


def test_gpu_count_never_initialises_hip(monkeypatch):
    """The launcher's count reads KFD / amdsmi only; visibility variables cap it."""
    b = _bench_module()
    n = b.count_gpus()
    assert n is None or n >= 0
    if n is not None:
        monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
        assert b.count_gpus() <= 1


def test_pmc_figures_attach_only_to_the_profiled_build(tmp_path):
    """bench.py's roofline.traffic / mfma_busy come from a committed PMC profile only when that
    profile was stamped with the loaded library's build (fr_version() hash)."""
    import json
    b = _bench_module()
    pj = {"build_id": "0123456789abcdef",
          "kernels": {"winograd": {"hbm_bytes_per_launch": 4.2e8, "alg_bytes_per_launch": 2e8, "mfma_busy_frac": 0.55}}}
    f = tmp_path / "layers_pmc.json"
    f.write_text(json.dumps(pj))
    t, a, m, src, note = b.profile_figures(str(f), "winograd", "frhip 0.1 gfx950 fp32-mfma build 0123456789abcdef", True)
    assert (t, a, m) == (4.2e8, 2e8, 0.55) and "0123456789abcdef" in src and note is None
    t, a, m, src, note = b.profile_figures(str(f), "winograd", "frhip 0.1 gfx950 fp32-mfma build ffffffffffffffff", True)
    assert t is a is m is src is None and "not attached" in note
    pj.pop("build_id")
    f.write_text(json.dumps(pj))
    assert b.profile_figures(str(f), "winograd", "x build 0123456789abcdef", True)[0] is None
    assert b.profile_figures(str(f), "winograd", "x build 0123456789abcdef", False)[0] is None
    # the library carries its content hash (tests/test_gpu_bench_launch.py checks it is this tree's)
    import re
    from facerecognitionpipeline_amd import _lib
    assert re.fullmatch(r"[0-9a-f]{16}", b.build_id_of(_lib.load().fr_version().decode()))
