"""Joint pose + map optimisation on the fused step: the per-keyframe pose gradient and the pose Adam.

The reference optimises every un-anchored keyframe's pose tensor in the same Adam as the map when an
iteration config has ``freeze_poses: False`` (src/mapping/optimizer.py:235-262; the default mapper
schedule's joint config, cfg/defaults.yaml:93-97), at ``lrate_pose`` (default_model_config.yaml:30) with
the same ExponentialLR.  A pose tensor is [t (3), axis-angle (3)] (Pose, src/common/pose.py:34-56;
``tensor_to_transform``, src/common/pose_utils.py:354-368, pytorch3d ``axis_angle_to_matrix``), and the
rays depend on it through ``LidarRayDirections.build_lidar_rays`` (src/common/ray_utils.py:269-322):

    o   = (t + shift) / scale                    (every ray of the keyframe)
    d   = R v / |R v|                            (v: the scan's sensor-frame direction)
    far = min(r_max / scale, get_far_val(o, d))  (:31-60, with no_nan's +1e-15)

Sky rays are built from the DETACHED pose (src/mapping/keyframe.py:98), and the samples z are detached
(the sampler's no_grad, src/models/ray_sampling.py:75-90).  The loss then sees the ray through the sample
positions xyz = o + z d (pos01 = (xyz + 1) / 2 into the hash grid), the deltas' |d|
(rendering_tcnn.py:248) and the far term of the depth (:274-278).

On the fused step (``StepEngine`` with ``pose_grad=True``):
* ``lnr_field_train`` writes per ray [dL/d|d|, dL/dfar] (``lnr_loss_params.dev_d_ray``);
* ``lnr_hashgrid_bwd_rays_jac`` writes per sample dL/dpos01 (``d_pos``, tcnn's input gradient) from the
  step's compact encoding gradient, before the table's Adam changes the table;
* ``ray_gradients`` reduces them to dL/do and dL/dd per ray and adds the far term;
* ``keyframe_gradients`` sums the rays of each keyframe into dL/dt and dL/dR without the scan
  directions: with u = R v and d = u / |u|, dL/dR = (1/|u|) (I - d d^T) g_d v^T = (I - d d^T) g_d d^T R;
* autograd through ``axis_angle_to_matrix`` (K 3x3 matrices) gives dL/d(axis-angle).

``PoseWindow`` holds the window's pose tensors (K, 6) on the device and, after each step, runs the chain
(``lnr_pose_grad``, csrc/pose.hip: the per-ray reduction, the far term and the per-keyframe sums in one pass
over the step's d_pos, then the axis-angle derivative in closed form) and the poses' Adam
(``lnr_pose_adam``), which rewrites the window's (K, 12) pose rows the next step's ray build (or HIP graph
replay) reads: three launches, no host synchronisation.  The torch functions below state the same chain;
they are the tests' reference for the kernels.
"""
import numpy as np
import torch


# ----------------------------------------------------------------------------- pose tensors
def axis_angle_to_matrix(aa):
    """pytorch3d.transforms.axis_angle_to_matrix (v0.7: axis_angle_to_quaternion, then
    quaternion_to_matrix), restated: (..., 3) -> (..., 3, 3), differentiable."""
    angles = torch.norm(aa, p=2, dim=-1, keepdim=True)
    half = 0.5 * angles
    eps = 1e-6
    small = angles.abs() < eps
    safe = torch.where(small, torch.ones_like(angles), angles)
    sin_half_over = torch.where(small, 0.5 - (angles * angles) / 48, torch.sin(half) / safe)
    q = torch.cat([torch.cos(half), aa * sin_half_over], dim=-1)
    r, i, j, k = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(aa.shape[:-1] + (3, 3))


def matrix_to_pose6(T):
    """``transform_to_tensor`` (src/common/pose_utils.py:321-347): (4, 4) or (K, 4, 4) -> [t, axis-angle]
    float32 (the axis-angle in float64 on the host, scipy's as_rotvec = pytorch3d matrix_to_axis_angle)."""
    from scipy.spatial.transform import Rotation
    M = np.asarray(T.detach().cpu() if isinstance(T, torch.Tensor) else T, dtype=np.float64)
    one = M.ndim == 2
    M = M.reshape(-1, 4, 4)
    out = np.concatenate([M[:, :3, 3], Rotation.from_matrix(M[:, :3, :3]).as_rotvec()], 1).astype(np.float32)
    return torch.from_numpy(out[0] if one else out)


def pose6_to_rows(p6):
    """(K, 6) pose tensors -> (K, 12) rows [R | t] (the RayWindow's pose layout), differentiable."""
    R = axis_angle_to_matrix(p6[:, 3:6])
    return torch.cat([R, p6[:, 0:3, None]], 2).reshape(-1, 12)


# ----------------------------------------------------------------------------- the chain
def far_value(o, d, far_range):
    """far = min(r_max / scale, get_far_val(o, d, no_nan=True)) (ray_utils.py:31-60, :307-311)."""
    dd = d + 1e-15
    sgn = torch.tensor([[-1.0], [1.0]], device=o.device, dtype=o.dtype)
    t = (sgn[..., None] - o[:, [0, 1, 2]]) / dd[:, [0, 1, 2]]
    clip = t.clamp(min=0).max(dim=0)[0].min(dim=1)[0]
    return torch.minimum(torch.full_like(clip, float(far_range)), clip)


def ray_gradients(rays, z, d_pos, d_ray, far_range):
    """Per ray dL/do and dL/dd (both (R, 3)) from the step's per-sample dL/dpos01 ``d_pos`` (R*S, 3),
    the per-ray [dL/d|d|, dL/dfar] ``d_ray`` (R, 2), the rays (R, 13) and samples z (R, S):
        xyz = o + z d, pos01 = (xyz + 1) / 2:   dL/do = sum_s dpos / 2,  dL/dd = sum_s z dpos / 2
        deltas = dl |d|:                        dL/dd += dL/d|d| d / |d|
        far = min(far_range, far_clip(o, d)):   dL/d{o, d} += dL/dfar dfar/d{o, d}   (autograd)"""
    n, S = z.shape
    dp = d_pos[:n * S].view(n, S, 3)
    o, d = rays[:n, 0:3], rays[:n, 3:6]
    g_o = 0.5 * dp.sum(1)
    g_d = 0.5 * torch.bmm(z[:, None, :], dp)[:, 0]
    g_d = g_d + d_ray[:n, 0:1] * (d / d.norm(dim=1, keepdim=True))
    with torch.enable_grad():
        o_ = o.detach().requires_grad_()
        d_ = d.detach().requires_grad_()
        far = far_value(o_, d_, far_range)
        go, gd = torch.autograd.grad(far, (o_, d_), d_ray[:n, 1])
    return g_o + go, g_d + gd


def keyframe_gradients(rays, g_o, g_d, ray_kf, ray_pose, p6, scale, n_kf):
    """Per-keyframe dL/d(pose tensor) (K, 6) from per-ray dL/do, dL/dd: rays of keyframe ``ray_kf``
    whose ``ray_pose`` (float 0/1: LiDAR ray of an optimised pose) is set.  o = (t + shift) / scale gives
    dL/dt = sum dL/do / scale; d = R v / |R v| gives dL/dR = sum (I - d d^T) g_d d^T R (the module
    docstring); dL/d(axis-angle) by autograd through ``axis_angle_to_matrix``."""
    n = g_o.shape[0]
    d = rays[:n, 3:6]
    m = ray_pose[:n].to(g_o.dtype)[:, None]
    g_perp = (g_d - d * (d * g_d).sum(1, keepdim=True)) * m
    kf = ray_kf[:n].long()
    gt = torch.zeros(n_kf, 3, dtype=g_o.dtype, device=g_o.device).index_add_(0, kf, g_o * m) / scale
    gm = torch.zeros(n_kf, 9, dtype=g_o.dtype, device=g_o.device).index_add_(
        0, kf, (g_perp[:, :, None] * d[:, None, :]).reshape(n, 9)).view(n_kf, 3, 3)
    with torch.enable_grad():
        aa = p6[:, 3:6].detach().requires_grad_()
        Rm = axis_angle_to_matrix(aa)
        g_aa, = torch.autograd.grad(Rm, aa, gm @ Rm.detach())
    return torch.cat([gt, g_aa], 1)


# ----------------------------------------------------------------------------- the window's poses
class PoseWindow:
    """The optimisable poses of one ``RayWindow``: pose tensors (K, 6) on the device, initialised from
    the window's poses (``transform_to_tensor``) unless given, and rewritten into the window's pose rows
    (``tensor_to_transform``: the reference builds every ray from the pose tensor's matrix).
    ``optimise``: (K,) bools, the keyframes whose pose is optimised (the reference's un-anchored
    keyframes of the active window, optimizer.py:248-262).  ``lr``: lrate_pose; the step's
    ``lr_factor`` (ExponentialLR) scales it as it scales the map's.  Each ``step`` after an engine step,
    three launches and no host synchronisation: ``lnr_pose_grad`` (the pose gradient of that step's rays:
    ``slots`` their window slots, or None for the engine's slots [ray_offset, ray_offset + n)), the all-reduce
    of the (K, 6) gradient when data-parallel (``allreduce``), and ``lnr_pose_adam`` (torch.optim.Adam's step on
    the (K, 6) tensor: a keyframe held fixed has a zero gradient, its pose does not move; then the window's
    pose rows).  ``ray_gradients`` / ``keyframe_gradients`` above state the same chain in torch
    (tests/test_gpu_pose.py compares the two)."""

    def __init__(self, window, optimise, lr, pose6=None, allreduce=None, n_iter=None, lr_gamma=1.0):
        from . import _lib as L
        self._L = L
        dev = window.device
        K = window.n_kf
        if pose6 is None:
            M = torch.zeros(K, 4, 4)
            M[:, :3, :4] = window.poses.detach().cpu().view(K, 3, 4)
            M[:, 3, 3] = 1.0
            pose6 = matrix_to_pose6(M)
        self.p6 = torch.as_tensor(pose6, dtype=torch.float32).reshape(K, 6).to(dev).clone()
        self.optimise = torch.as_tensor(optimise, dtype=torch.bool).reshape(K).to(dev)
        self._opt_u8 = self.optimise.to(torch.uint8)
        self.window = window
        self.lr = float(lr)
        self.allreduce = allreduce
        self.m = torch.zeros(K, 6, dtype=torch.float32, device=dev)
        self.v = torch.zeros(K, 6, dtype=torch.float32, device=dev)
        self.adam_step = 0
        self.grad = torch.zeros(K, 6, device=dev)
        self._ray_ws = None
        # per window slot: its keyframe, and whether the ray follows the pose (a LiDAR ray of an
        # optimised keyframe; sky rays use the detached pose)
        off, nsel = window.ray_off_host, window.n_sel_host
        kf = np.zeros(window.n_slots, np.int32)
        lid = np.zeros(window.n_slots, np.float32)
        opt = self.optimise.cpu().numpy()
        for k in range(K):
            kf[off[k]:off[k + 1]] = k
            lid[off[k]:off[k] + nsel[k]] = 1.0 if opt[k] else 0.0
        self.slot_kf = torch.from_numpy(kf).to(dev)
        self.slot_pose = torch.from_numpy(lid).to(dev)
        self.far_range = window.ray_range[1] / window.scale
        # Can a ray of this window fail the 1 m filter (ray_utils.py:319-322) while its pose moves?  A ray's
        # far bound is at least the origin's L-inf distance to the cube's faces (its direction is a unit
        # vector), and n_iter Adam steps move a translation by at most adam_travel_bound per coordinate:
        # when every keyframe keeps 1 - max|o| above near + 1 m after that, no ray can turn invalid and the
        # step needs no per-step host check (StepEngine.step_window's fixed-size path); otherwise it
        # filters every step (one host synchronisation per step).
        t = self.p6.cpu().numpy()[:, 0:3].astype(np.float64)
        shift = np.array([window.desc.shift[i] for i in range(3)], np.float64)
        o = (t + shift[None]) / window.scale
        travel = adam_travel_bound(self.lr, n_iter if n_iter is not None else 10 ** 6, lr_gamma) / window.scale
        need = (window.ray_range[0] + 1.0) / window.scale
        margin = 1.0 - np.abs(o).max(1) - np.where(opt, travel, 0.0)
        self.stay_valid = bool((margin > need).all() and self.far_range > need)
        self.write_window()

    def write_window(self):
        L = self._L
        L.call("lnr_pose_adam", self.p6, None, None, None, None, self.window.n_kf, 0, 0.0, 0.9, 0.999, 1e-8,
               self.window.poses, L.stream(self.p6.device))

    def matrices(self):
        """(K, 4, 4) float32 on the host: the current poses (``Pose.get_transformation_matrix``)."""
        rows = self.window.poses.detach().cpu().view(-1, 3, 4)
        M = torch.zeros(rows.shape[0], 4, 4)
        M[:, :3, :] = rows
        M[:, 3, 3] = 1.0
        return M

    def gradient(self, engine, rays, slots=None, slot0=None):
        """dL/d(pose tensors) (K, 6), written into ``self.grad``, of the engine's last step (``pose_grad`` on):
        ``rays`` the step's (R, 13) rays, ``slots`` their window slots (R,) int64, or None for slot0 + r."""
        L = self._L
        n = rays.shape[0]
        if self._ray_ws is None or self._ray_ws.numel() < 12 * max(n, 1):
            self._ray_ws = torch.empty(12 * max(n, 1), dtype=torch.float32, device=rays.device)
        L.call("lnr_pose_grad", rays, engine.z, engine.d_pos, engine.d_ray, n, engine.S, slots,
               engine.ray_offset if slot0 is None else int(slot0), self.slot_kf, self.slot_pose, self.p6,
               self.window.n_kf, self.window.scale, self.far_range, self._ray_ws, self.grad, L.stream(rays.device))
        if self.allreduce is not None:
            self.allreduce(self.grad)
        return self.grad

    def step(self, engine, rays, slots=None, lr_factor=1.0):
        L = self._L
        self.gradient(engine, rays, slots)
        self.adam_step += 1
        L.call("lnr_pose_adam", self.p6, self.m, self.v, self.grad, self._opt_u8, self.window.n_kf, self.adam_step,
               self.lr * lr_factor, 0.9, 0.999, 1e-8, self.window.poses, L.stream(rays.device))
        return self.grad


def adam_travel_bound(lr, n_iter, gamma=1.0, beta1=0.9, beta2=0.999):
    """An upper bound on how far (per coordinate) ``n_iter`` Adam steps at lr * gamma^it can move a
    parameter, whatever its gradients: |m_hat_t| / sqrt(v_hat_t) <= (1 - b1) sqrt((1 - c^t) / (1 - c))
    sqrt(1 - b2^t) / (sqrt(1 - b2) (1 - b1^t)) with c = b1^2 / b2 (Cauchy-Schwarz over the moment sums).
    The optimiser uses it to prove a window's rays stay valid while its poses move (no per-step check)."""
    c = beta1 * beta1 / beta2
    tot = 0.0
    for t in range(1, int(n_iter) + 1):
        r = (1 - beta1) * np.sqrt((1 - c ** t) / (1 - c)) * np.sqrt(1 - beta2 ** t) / (np.sqrt(1 - beta2) * (1 - beta1 ** t))
        tot += lr * gamma ** (t - 1) * r
    return float(tot)
