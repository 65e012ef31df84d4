"""Ray construction restated in numpy — TEST INFRASTRUCTURE ONLY.

get_far_val        ``src/common/ray_utils.py:31-60`` (no_nan adds 1e-15 to directions)
build_lidar_rays   ``LidarRayDirections.build_lidar_rays`` ``src/common/ray_utils.py:269-322``:
                   13 columns [o(3) d(3) viewdir(3) 0 0 near far], rays kept only if
                   far > near + 1 m / scale; depths normalised by the world-cube scale
sky depth          ``KeyFrame.build_lidar_rays`` ``src/mapping/keyframe.py:94-103``: sky rays get
                   distance ray_range[1] + 1 (``sensors.py:164-167``)
world_cube_bbox    ``compute_world_cube`` bbox branch ``src/common/pose_utils.py:222-314``
                   (lidar-only, identity rotations; callers pass padding 0.3: loner.py:104)
"""
import numpy as np

F32 = np.float32


def get_far_val(o, d, no_nan=True):
    d = d.astype(F32)
    if no_nan:
        d = (d + F32(1e-15)).astype(F32)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = ((np.array([-1.0, 1.0], F32)[:, None, None] - o[None].astype(F32)) / d[None]).astype(F32)
    t = np.maximum(t, F32(0)).max(0)
    return t.min(1, keepdims=True).astype(F32)


def build_lidar_rays(dirs_sensor, dists, pose4x4, ray_range, scale, shift, ignore_world_cube=False):
    """dirs_sensor (3,P), dists (P,), pose (4,4) -> (rays (P',13), depths (P',)) fp32."""
    scale = F32(scale)
    depths = (dists.astype(F32) / scale).astype(F32)
    o = ((pose4x4[:3, 3].astype(F32) + shift.astype(F32)) / scale).astype(F32)
    o = np.tile(o, (dirs_sensor.shape[1], 1))
    d = (pose4x4[:3, :3].astype(F32) @ dirs_sensor.astype(F32)).T.astype(F32)
    d = (d / np.sqrt((d * d).sum(1, keepdims=True, dtype=F32))).astype(F32)
    near = np.full((len(depths), 1), F32(ray_range[0]) / scale, F32)
    far_range = np.full((len(depths), 1), F32(ray_range[1]) / scale, F32)
    far = np.minimum(far_range, get_far_val(o, d, True))
    rays = np.concatenate([o, d, -d, np.zeros((len(depths), 2), F32), near, far], 1).astype(F32)
    if ignore_world_cube:
        return rays, depths
    valid = (far > (near + F32(1.0) / scale))[:, 0]
    return rays[valid], depths[valid]


def world_cube_bbox(bbox, ray_range, padding=0.3):
    xs, ys, zs = bbox["x"], bbox["y"], bbox["z"]
    combos = np.array([[x, y, z] for x in xs for y in ys for z in zs], F32)
    m = F32(ray_range[1])
    corners = np.array([[sx * m, sy * m, sz * m] for sz in (-1, 1) for sx in (-1, 1) for sy in (-1, 1)], F32)
    pts = np.concatenate([(c + corners) for c in combos] + [combos], 0).astype(F32)
    mn, mx = pts.min(0), pts.max(0)
    origin = (mn + (mx - mn) / F32(2)).astype(F32)
    scale = F32(np.linalg.norm((mx - mn).astype(F32)) / (F32(2) * np.sqrt(F32(3)))) * F32(1 + padding)
    return F32(scale), (-origin).astype(F32)
