"""Per-keyframe scan preprocessing restated in numpy — TEST INFRASTRUCTURE ONLY.

motion_compensate  LidarScan.motion_compensate (src/common/sensors.py:169-231): interp factor
                   s = (t - t0)/(t1 - t0); translation start + s (end - start); rotation
                   start_R @ exp(s * log(inv(start_R) end_R)) (pytorch3d matrix_to_axis_angle /
                   axis_angle_to_matrix: absent here, restated as the Rodrigues map); points
                   dirs * dists re-expressed by inv(T_world_to_target) @ T_world_to_compensated.
sky_rays           compute_sky_rays (examples/fdt_optimize_implicit_map_utils.py:38-77) with
                   kornia.morphology.dilation / erosion (absent here) restated for a 3x3 ones kernel
                   with kornia's default geodesic border: out-of-image neighbours are ignored.
float64 arithmetic (the reference runs float32 torch); parity unpinned against pytorch3d / kornia
themselves, whose outputs no reference test holds.
"""
import numpy as np


def _rodrigues(axis, ang):
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * (K @ K)


def motion_compensate(dirs, dists, ts, start, end, t0, t1, target):
    """dirs (3,P), dists (P,), ts (P,), poses 4x4 -> (dirs (3,P), dists (P,))."""
    from scipy.spatial.transform import Rotation
    start, end, target = (np.asarray(m, np.float64) for m in (start, end, target))
    s = (np.asarray(ts, np.float64) - t0) / (t1 - t0)
    trans = (end[:3, 3] - start[:3, 3])[None] * s[:, None] + start[:3, 3][None]
    rv = Rotation.from_matrix(start[:3, :3].T @ end[:3, :3]).as_rotvec()
    ang = np.linalg.norm(rv)
    pts = np.asarray(dirs, np.float64) * np.asarray(dists, np.float64)[None]
    out = np.empty_like(pts)
    tinv = np.linalg.inv(target)
    for i in range(pts.shape[1]):
        R = np.eye(3) if ang < 1e-9 else _rodrigues(rv / ang, ang * s[i])
        w = start[:3, :3] @ R @ pts[:, i] + trans[i]
        out[:, i] = tinv[:3, :3] @ w + tinv[:3, 3]
    d = np.linalg.norm(out, axis=0)
    return out / d, d


def sky_rays(dirs, rot, top_rows=3, horizon_deg=10.0):
    """dirs (3,P) sensor frame, rot (3,3) -> sky directions (3,Q), rotated by rot (reference quirk)."""
    x, y, z = np.asarray(dirs, np.float32).astype(np.float64)
    theta = np.rint(np.rad2deg(np.arctan2(y, x))).astype(np.int64)
    phi = np.rint(np.rad2deg(np.arctan2(np.sqrt(x ** 2 + y ** 2), z))).astype(np.int64)
    phi_img, theta_img = phi - phi.min(), theta - theta.min()
    theta_img[theta_img == 360] = 0
    img = np.zeros((phi_img.max() + 1, 360))
    img[phi_img, theta_img] = 1

    def morph(a, fn, fill):
        p = np.pad(a, 1, constant_values=fill)
        st = np.stack([p[1 + dr:1 + dr + a.shape[0], 1 + dc:1 + dc + a.shape[1]] for dr in (-1, 0, 1) for dc in (-1, 0, 1)])
        return fn(st, axis=0)

    img = morph(morph(img, np.max, -np.inf), np.min, np.inf)
    img[:top_rows] = 1
    zr, zc = np.nonzero(img == 0)
    zp, zt = np.deg2rad(zr + phi.min()), np.deg2rad(zc + theta.min())
    d = np.vstack([np.sin(zp) * np.cos(zt), np.sin(zp) * np.sin(zt), np.cos(zp)])
    dw = np.asarray(rot, np.float64) @ d
    phw = 90 - np.rad2deg(np.arctan2(np.sqrt(dw[0] ** 2 + dw[1] ** 2), dw[2]))
    return dw[:, phw > horizon_deg]
