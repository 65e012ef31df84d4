"""bench.py's rank-count contract, checked without a GPU: the JSON line's n_gpus must be the number of
ranks that ran, so inconsistent requests fail before any rank starts."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=120, cwd=ROOT)


def test_gpus_beyond_visible_devices_fails_before_spawning():
    import torch
    n = max(torch.cuda.device_count() + 1, 2)
    r = _run(["--gpus", str(n), "--no-cpu-baseline"], LONER_DIST_BACKEND="nccl")
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_gpus_must_match_launcher_world_size():
    r = _run(["--gpus", "3", "--no-cpu-baseline"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in r.stderr


def test_single_gpu_configs_refuse_multiple_ranks():
    r = _run(["--config", "C3", "--no-cpu-baseline"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "single-GPU bench" in r.stderr
