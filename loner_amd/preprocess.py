"""Per-keyframe scan preprocessing on the GPU (the north-star driver's per-keyframe steps,
examples/fdt_optimize_implicit_map.py:594-607), feeding ``loner_amd.rays.RayWindow``:

    motion_compensate   LidarScan.motion_compensate (src/common/sensors.py:169-231)
    sky_rays            compute_sky_rays (examples/fdt_optimize_implicit_map_utils.py:38-77)

The per-scan constants (relative rotation log, target inverse) are formed on the host in float64
from the two 4x4 poses; the per-point / per-bin work runs in HIP (``csrc/preprocess.hip``).
"""
import numpy as np
import torch

from . import _lib as L

NUMERIC_TOLERANCE = 1e-9  # src/common/sensors.py:20


def _np(m):
    return np.asarray(m.detach().cpu() if isinstance(m, torch.Tensor) else m, dtype=np.float64)


def _rotvec(R):
    """Axis-angle of a rotation matrix (pytorch3d matrix_to_axis_angle), float64."""
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(R).as_rotvec()


def motion_comp_params(start_pose, end_pose, t0, t1, target_pose):
    s, e, tg = _np(start_pose), _np(end_pose), _np(target_pose)
    mc = L.MotionComp()
    rv = _rotvec(s[:3, :3].T @ e[:3, :3])  # inv(start_rot) @ end_rot
    ang = float(np.linalg.norm(rv))
    mc.identity = 1 if ang < NUMERIC_TOLERANCE else 0
    axis = rv / ang if ang >= NUMERIC_TOLERANCE else np.zeros(3)
    inv = np.linalg.inv(tg)
    for i in range(9):
        mc.start_rot[i] = float(s[:3, :3].reshape(-1)[i])
    for i in range(3):
        mc.start_t[i] = float(s[i, 3])
        mc.delta_t[i] = float(e[i, 3] - s[i, 3])
        mc.axis[i] = float(axis[i])
    mc.angle = ang
    mc.t0, mc.t1 = float(t0), float(t1)
    for i in range(12):
        mc.target_inv[i] = float(inv[:3, :].reshape(-1)[i])
    return mc


def motion_compensate(dirs, dists, timestamps, poses, timestamps_pose, target_pose):
    """dirs (P,3) and dists (P,) device tensors, rewritten in place; timestamps (P,) device.
    ``poses`` = (start, end) 4x4, ``timestamps_pose`` = (t0, t1)."""
    mc = motion_comp_params(poses[0], poses[1], timestamps_pose[0], timestamps_pose[1], target_pose)
    L.call("lnr_motion_compensate", L.ctypes.byref(mc), timestamps, dirs, dists, dists.numel(),
           L.stream(dirs.device))
    return dirs, dists


def sky_rays(dirs, lidar_pose, top_rows=3, horizon_deg=10.0):
    """Sky directions (Q,3) of one scan with sensor-frame dirs (P,3) on the GPU; rotated by the lidar
    pose rotation as the reference does.  One host synchronisation (Q)."""
    dev = dirs.device
    sp = L.SkyParams()
    R = _np(lidar_pose)[:3, :3]
    for i in range(9):
        sp.rot[i] = float(R.reshape(-1)[i])
    sp.top_rows = int(top_rows)
    sp.horizon_deg = float(horizon_deg)
    cap = int(L.lib().lnr_sky_rays_capacity())
    out = torch.empty(cap, 3, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("lnr_sky_rays", dirs, dirs.shape[0], L.ctypes.byref(sp), out, cap, cnt, L.stream(dev))
    return out[:int(cnt.item())].clone()
