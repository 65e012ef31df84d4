"""World-size-2 data-parallel step on CPU (gloo): each rank runs the oracle step on its shard with
global normalisers and global-index draws, exchanging the opaque count and the gradient through
torch.distributed all_reduce; the summed result must equal the single-batch step.  This is the
decomposition StepEngine(ray_offset, allreduce, n_rays_global) relies on."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from loner_amd.shard import shard_range

LOSS = dict(loss_selection="L1_JS", JS_loss=dict(min_js_score=1.0, max_js_score=10.0, alpha=1.0),
            decay_los_lambda=False, los_lambda=1000.0, min_los_lambda=10.0, los_lambda_decay_rate=0.001,
            los_lambda_decay_steps=15000, decay_depth_eps=True, depth_eps=3.0, min_depth_eps=0.5,
            depth_eps_decay_rate=0.95, depth_eps_decay_steps=1, depthloss_lambda=0.005)
S = 64


def _batch():
    from loner_amd import synthetic as syn
    win = syn.make_window("quad", 2, seed=3)
    rays, dgt = syn.build_batch(win, "quad", 7, 0, "RANDOM", seed=5)  # 14 rays: uneven 2-way split
    return rays.numpy(), dgt.numpy(), syn.CUBES["quad"][0]


def _small_field():
    from oracle import step as ostep
    f = ostep.OracleField(n_levels=16, log2_hashmap_size=12, table_init=0.3)
    f.params[2048:3072] *= 8.0
    return f


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import step as ostep

    def allreduce(a):
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    rays, dgt, scale = _batch()
    s0, s1 = shard_range(rays.shape[0], rank, world)
    field = _small_field()
    loss, z, grad = ostep.train_step(field, rays[s0:s1], dgt[s0:s1], scale, LOSS, 1, n_samples=S, key=77,
                                     ray_offset=s0, allreduce=allreduce, n_rays_global=rays.shape[0],
                                     far_ref=float(rays[0, -1]))
    loss_sum = allreduce(np.array([loss]))[0]
    if rank == 0:
        np.savez(out_path, loss=loss_sum, grad=grad, params=field.params)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for n in (0, 1, 5, 9216):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def test_two_rank_step_equals_single_batch(tmp_path):
    from oracle import step as ostep
    out = str(tmp_path / "rank0.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    rays, dgt, scale = _batch()
    field = _small_field()
    loss, _, grad = ostep.train_step(field, rays, dgt, scale, LOSS, 1, n_samples=S, key=77)
    assert abs(got["loss"] - loss) <= 1e-6 * abs(loss)
    assert np.linalg.norm(got["grad"] - grad) <= 1e-6 * np.linalg.norm(grad)
    np.testing.assert_allclose(got["params"], field.params, rtol=0, atol=1e-7)
