"""One full optimiser step composed from the oracle modules — TEST INFRASTRUCTURE ONLY.

Used as (a) the end-to-end checker of the HIP step and (b) the ``cpu_baseline`` leg of bench.py
(single-threaded numpy restatement; the reference has no CPU MLP path — SURVEY.md §8(c)).
Follows the step body of ``Optimizer._do_iterate_optimizer`` (src/mapping/optimizer.py:354-475):
OGM sampling -> sigma field (HashGrid + FullyFusedMLP) -> raw2outputs -> LiDAR loss ->
backward -> Adam -> OGM update every N_iters_acc global steps.
"""
import numpy as np

from . import hashgrid as ohg
from . import loss as oloss
from . import mlp as omlp
from . import optim as ooptim
from . import render as orender
from . import rng as orng

F32 = np.float32


class OracleField:
    def __init__(self, n_levels=16, log2_hashmap_size=18, base_resolution=16, seed=1337, table_init=1e-4,
                 occ_res=100):
        self.layout = ohg.GridLayout(n_levels, 2, log2_hashmap_size, base_resolution)
        a0 = np.sqrt(6.0 / (32 + 64))
        a1 = np.sqrt(6.0 / (64 + 16))
        w0 = omlp.uniform_fill(64 * 32, seed, -a0, a0)
        w1 = omlp.uniform_fill(16 * 64, seed + 1, -a1, a1)
        tab = omlp.uniform_fill(2 * self.layout.n_entries, seed + 2, -table_init, table_init)
        self.params = np.concatenate([w0, w1, tab]).astype(F32)
        self.m = np.zeros_like(self.params)
        self.v = np.zeros_like(self.params)
        self.adam_step = 0
        self.occ = np.zeros((occ_res,) * 3, F32)

    def split16(self):
        p16 = self.params.astype(np.float16)
        return p16[:2048].reshape(64, 32), p16[2048:3072].reshape(16, 64), p16[3072:].reshape(-1, 2)


def train_step(field, rays, depth_gt, scale, loss_cfg, global_step, n_samples=512, key=0, ray_offset=0, lr=0.01,
               occ_lr=1e-4, n_iters_acc=10, noise_std=1.0, z=None, allreduce=None, n_rays_global=None,
               far_ref=None):
    """One step; returns (loss, z, grad).  Draws come from oracle.rng with the HIP path's keys.

    ``z`` (R, n_samples) replaces the sampler's output when given: the finest hash levels have
    cells of ~2e-6 (scale 16*2^15), so a 1-ulp difference in a sample depth moves its trilinear
    weights by percents; a checker that wants to isolate the field/backward from the sampler
    feeds the sampler's GPU output back in here (the sampler is checked on its own).

    Data-parallel shard: ``ray_offset`` = global index of this shard's first
    ray (keys the draws), ``n_rays_global``, ``far_ref`` = far bound of global ray 0, and
    ``allreduce(np.ndarray) -> np.ndarray`` summing over shards: the opaque count and the
    gradient are exchanged before the loss and before Adam.  Returns this shard's loss share."""
    R = rays.shape[0]
    H = n_samples // 2
    if z is None:
        a, b = orng.ray_sample_grid(np.arange(ray_offset, ray_offset + R), H)
        uj = orng.uniform(key, orng.STREAM_JITTER, a, b)
        up = orng.uniform(key, orng.STREAM_PDF, a, b)
        z = orender.ogm_samples(rays, n_samples, field.occ, uj, up)
    a2, b2 = orng.ray_sample_grid(np.arange(ray_offset, ray_offset + R), n_samples)
    noise = orng.normal(key, orng.STREAM_NOISE, a2, b2) * F32(noise_std)
    w0, w1, table = field.split16()
    xyz = (rays[:, None, 0:3] + rays[:, None, 3:6] * z[:, :, None]).astype(F32)
    pos = ((xyz + F32(1)) / F32(2)).astype(F32).reshape(-1, 3)
    x = ohg.encode(pos, table, field.layout)
    out16, hid = omlp.forward(x, [w0, w1])
    sig = out16[:, 0].astype(F32).reshape(R, n_samples)
    far = rays[:, -1:]
    ro = orender.raw2outputs(sig, z, rays[:, 3:6], noise, far)
    n_op = n_tot = None
    if allreduce is not None:
        f0 = np.float32(far[0, 0] if far_ref is None else far_ref)
        cnt = np.array([float(((depth_gt > 0) & ~(depth_gt > f0)).sum())])
        n_op = int(allreduce(cnt)[0])
        n_tot = (R if n_rays_global is None else n_rays_global) * n_samples
    res = oloss.lidar_loss(ro["weights"], z, ro["depth"], ro["opacity"], depth_gt, far, scale, loss_cfg, global_step,
                           n_opaque=n_op, n_total=n_tot, far_ref=far_ref)
    ds = orender.composite_backward(sig, z, rays[:, 3:6], noise, far, res["g_w"], res["g_depth"], res["g_opacity"])
    dout = np.zeros((R * n_samples, 16))
    dout[:, 0] = ds.reshape(-1)
    dx, dws = omlp.backward(x, [w0, w1], hid, dout)
    g_table = ohg.encode_backward(pos, dx, field.layout).reshape(-1)
    grad = np.concatenate([dws[0].reshape(-1), dws[1].reshape(-1), g_table])
    if allreduce is not None:
        grad = allreduce(grad)
    grad = grad.astype(F32)
    field.adam_step += 1
    ooptim.adam_step(field.params, grad, field.m, field.v, field.adam_step, lr)
    if global_step % n_iters_acc == 0:
        ooptim.ogm_step(field.occ, rays, z, depth_gt, scale, occ_lr)
    return res["loss"], z, grad
