"""CPU checks of the joint pose + map chain (loner_amd/pose.py): the pose tensor's matrix
(pytorch3d axis_angle_to_matrix, against scipy), and the per-keyframe pose gradient that the fused
step forms from its per-sample dL/dpos01 and per-ray [dL/d|d|, dL/dfar] (ray_gradients ->
keyframe_gradients), against torch autograd through the module-level ray build
(loner_amd.rays.build_lidar_rays = ray_utils.py:269-322, the sky rays from the detached pose as
keyframe.py:98 builds them) in float64.  The GPU side (the step's d_ray / d_pos against the module-level
render_rays chain) is tests/test_gpu_pose.py."""
import numpy as np
import pytest
import torch

from loner_amd import pose as P
from loner_amd.rays import WorldCube, build_lidar_rays


def test_axis_angle_to_matrix_matches_scipy():
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(0)
    aa = rng.normal(0, 1, (64, 3))
    aa[0] = 0.0
    aa[1] = [1e-9, -2e-9, 0.0]   # the small-angle branch
    aa[2] = [np.pi - 1e-4, 0.0, 0.0]
    R = P.axis_angle_to_matrix(torch.from_numpy(aa)).numpy()
    ref = Rotation.from_rotvec(aa).as_matrix()
    np.testing.assert_allclose(R, ref, atol=1e-12)
    # and matrix_to_pose6 inverts it (transform_to_tensor), float32
    T = np.tile(np.eye(4), (64, 1, 1))
    T[:, :3, :3] = ref
    T[:, :3, 3] = rng.normal(0, 3, (64, 3))
    p6 = P.matrix_to_pose6(T).double()
    np.testing.assert_allclose(P.axis_angle_to_matrix(p6[:, 3:]).numpy(), ref, atol=2e-6)
    np.testing.assert_allclose(p6[:, :3].numpy(), T[:, :3, 3], atol=1e-5)
    aa_t = torch.from_numpy(rng.normal(0, 1, (5, 3))).requires_grad_()
    assert torch.autograd.gradcheck(P.axis_angle_to_matrix, (aa_t,))


@pytest.mark.parametrize("far_range_m", [30.0, 14.0])
def test_keyframe_gradient_matches_autograd(far_range_m):
    """Synthetic upstream gradients: L = sum dpos . pos01 + sum g_dn |d| + sum g_far far over every
    sample of every ray.  ray_gradients + keyframe_gradients give autograd's dL/d(pose tensor) for the
    optimised keyframes and exactly zero for the anchored one; sky rays add nothing."""
    torch.manual_seed(0)
    rng = np.random.default_rng(1)
    dt = torch.float64
    K, Pn, Q, S = 4, 37, 9, 16
    scale = 20.0
    wc = WorldCube(torch.tensor(scale, dtype=dt), torch.tensor([0.5, -0.3, 0.2], dtype=dt))
    ray_range = (1.0, far_range_m)
    p6 = torch.zeros(K, 6, dtype=dt)
    p6[:, :3] = torch.from_numpy(rng.uniform(-12, 12, (K, 3)))
    p6[:, 3:] = torch.from_numpy(rng.normal(0, 0.8, (K, 3)))
    p6[2, 3:] = torch.tensor([1e-8, 0.0, -1e-8])  # the small-angle branch
    p6 = p6.requires_grad_()
    optimise = torch.tensor([False, True, True, True])  # keyframe 0 anchored (optimizer.py:196-197)
    rays, kf, flag = [], [], []
    for k in range(K):
        Rk = P.axis_angle_to_matrix(p6[k, 3:])
        M = torch.cat([torch.cat([Rk, p6[k, :3, None]], 1), torch.tensor([[0, 0, 0, 1]], dtype=dt)], 0)
        Mk = M if optimise[k] else M.detach()
        dirs = torch.from_numpy(rng.normal(0, 1, (3, Pn)))
        dirs = dirs / dirs.norm(dim=0, keepdim=True)
        r, _ = build_lidar_rays(dirs, torch.ones(Pn, dtype=dt), Mk, ray_range, wc, ignore_world_cube=True)
        sky = torch.from_numpy(rng.normal(0, 1, (3, Q)))
        sr, _ = build_lidar_rays(sky / sky.norm(dim=0, keepdim=True), torch.ones(Q, dtype=dt), M.detach(), ray_range,
                                 wc, ignore_world_cube=True)
        rays += [r, sr]
        kf += [k] * (Pn + Q)
        flag += [1.0 if optimise[k] else 0.0] * Pn + [0.0] * Q
    rays = torch.cat(rays)
    n = rays.shape[0]
    z = torch.sort(torch.from_numpy(rng.uniform(0.01, 1.2, (n, S))), 1)[0]
    dpos = torch.from_numpy(rng.normal(0, 1, (n, S, 3)))
    dray = torch.from_numpy(rng.normal(0, 1, (n, 2)))
    o, d = rays[:, 0:3], rays[:, 3:6]
    pos01 = (o[:, None, :] + z[..., None] * d[:, None, :] + 1.0) / 2.0
    loss = (dpos * pos01).sum() + (dray[:, 0] * d.norm(dim=1)).sum() + (dray[:, 1] * rays[:, 12]).sum()
    loss.backward()
    ref = p6.grad.clone()
    g_o, g_d = P.ray_gradients(rays.detach(), z, dpos.reshape(-1, 3), dray, ray_range[1] / scale)
    g = P.keyframe_gradients(rays.detach(), g_o, g_d, torch.tensor(kf), torch.tensor(flag, dtype=dt), p6.detach(),
                             scale, K)
    np.testing.assert_allclose(g[1:].numpy(), ref[1:].numpy(), rtol=1e-9, atol=1e-9)
    assert torch.all(g[0] == 0) and torch.all(ref[0] == 0)
    # the far clip is active on some rays and the range on others (both branches exercised)
    clip = P.far_value(o.detach(), d.detach(), 1e9)
    frac = float((clip < ray_range[1] / scale).double().mean())
    assert (0.0 < frac < 1.0) or far_range_m == 30.0


def test_adam_travel_bound():
    """The bound holds for adversarial gradient sequences (constant, alternating, growing)."""
    lr, n = 1e-3, 50
    b = P.adam_travel_bound(lr, n, 0.99)
    for seq in (np.ones(n), (-1.0) ** np.arange(n), 1.5 ** np.arange(n), np.r_[np.zeros(20), np.ones(30)] * 1e-3,
                np.r_[1e3, np.ones(n - 1) * 1e-6]):
        x = torch.zeros(1, requires_grad=True)
        opt = torch.optim.Adam([x], lr=lr)
        for it, gv in enumerate(seq):
            for pg in opt.param_groups:
                pg["lr"] = lr * 0.99 ** it
            x.grad = torch.tensor([float(gv)])
            opt.step()
        assert abs(float(x)) <= b + 1e-12, (float(x), b)
    assert b >= lr * 0.99 ** 0  # a first step moves lr
