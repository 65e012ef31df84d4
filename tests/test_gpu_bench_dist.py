"""The multi-rank bench harness and the RCCL path on the one-GPU box.

* ``bench.py --gpus 2`` with no launcher starts its own two rank processes; with
  LONER_DIST_BACKEND=gloo both share GPU 0, and the JSON line must report the ranks that really ran.
* StepEngine through torch.distributed with backend ``nccl`` (RCCL) at world size 1: the bucketed
  asynchronous all-reduce, its stream waits and the per-range accumulation must reproduce the
  single engine bit for bit (the driver's N-GPU runs take this code path)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(text):
    lines = [l for l in text.splitlines() if l.startswith("{")]
    assert lines, text[-2000:]
    return json.loads(lines[-1])


def test_bench_spawns_two_gloo_ranks():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["LONER_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C4", "--steps", "3",
                        "--warmup", "1", "--no-cpu-baseline", "--field", "init"], env=env, capture_output=True, text=True, timeout=110,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2
    assert line["dist"] == {"backend": "gloo", "ranks": 2}
    # C4 at N > 1 defaults to strong scaling: the 16 KF x 576 = 9216-ray batch split over the ranks
    assert line["scaling"] == "strong"
    assert line["config"]["global_rays"] == 9216 and line["config"]["rays_per_gpu"] == 4608
    assert line["value"] > 0 and line["loss"] == line["loss"]


RCCL_WORKER = r"""
import os, sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.environ["LNR_ROOT"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
from loner_amd import step as S_
from loner_amd import synthetic as syn
win = syn.make_window("forest", n_kf=2, seed=3)
rays, dgt = syn.build_batch(win, "forest", rays_per_kf=64, sky_per_kf=8, strategy="MASK", seed=1)
rays, dgt = rays.cuda(), dgt.cuda()
out = {}
for tag, hook in (("single", None), ("rccl", lambda t, async_op=False: dist.all_reduce(t, async_op=async_op))):
    st = S_.FieldState(S_.StepConfig(n_samples=512, occ_lr=1e-3), device="cuda:0", table_init=0.5, seed=5)
    eng = S_.StepEngine(st, rays.shape[0], seed=9, allreduce=hook)
    for k in range(3):  # step 10 runs the OGM update, whose gradient is all-reduced too
        eng.step(rays, dgt, global_step=9 + k, scale=syn.CUBES["forest"][0], far_ref=float(rays[0, -1]))
    torch.cuda.synchronize()
    out[tag] = (st.grad.cpu().numpy(), st.params.cpu().numpy(), st.occ.cpu().numpy(), eng.loss_out.cpu().numpy())
for a, b in zip(out["single"], out["rccl"]):
    assert np.array_equal(a, b), float(np.abs(a - b).max())
dist.destroy_process_group()
print("rccl world-1 bitwise ok")
"""


def test_rccl_world1_step_is_bitwise_single_engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, LNR_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", RCCL_WORKER], env=env, capture_output=True, text=True, timeout=110,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "rccl world-1 bitwise ok" in r.stdout
