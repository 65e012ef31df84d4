"""Trajectory segmentation into submaps (C5), restated from
examples/fdt_segment_and_optimize_submaps.py:24-25,86-162 and the submap branch of
src/common/pose_utils.py:222-314 (compute_world_cube), as the fdt driver calls it for a submap
(examples/fdt_optimize_implicit_map.py:208-233).  Host-side numpy.  Pinned by tests/golden/submaps.npz,
which tests/golden/make_golden.py (``r3``) wrote by running the reference's own segmentation script and
compute_world_cube on the committed haveri keyframe trajectory (tests/test_submaps.py).

Split (:86-109): walk the ground-truth poses accumulating the distance between consecutive positions;
when adding the next step would pass MAX_LENGTH (50 m) the part closes, and the next part starts WITH
the previous pose (consecutive parts share their boundary pose) and a zero distance.
Padding (:136-147): every part but the first is written with the previous part's poses [-30, -1)
before it, every part but the last with the next part's poses [1, 30) after it: in trajectory
indices the padded submap is the contiguous range [start - 29, end + 29].  Those indexings need both
neighbouring parts to hold at least 30 poses; the reference raises IndexError otherwise, and so does
``padded_ranges``.
World cube (pose_utils.py:244-314 with submap set): the poses are used as they are (not re-based on the
first pose, :245-248).  The hpk (haveri) dataset family has no calibration object
(examples/utils.py:119-123), so camera_to_lidar is None and the LiDAR branch runs (:285-302): the 8
corners (+-max range)^3 are transformed by every pose (rotation AND translation, :296-298), and the
points are those corners plus every pose's position; origin = the points' box centre, scale = |box
diagonal| / (2 sqrt 3) * (1 + padding), shift = -origin.  The camera-frustum branch (:262-283, taken
only with a Fusion Portable calibration) is restated with the other branches in
``loner_amd.rays.compute_world_cube`` and pinned by tests/golden/world_cube_camera.npz."""
import numpy as np

MAX_LENGTH = 50.0  # metres (:24)
PADDING = 30       # poses (:25)


def split_trajectory(positions, max_length=MAX_LENGTH):
    """positions (N, 3) -> list of (start, end) inclusive trajectory indices of the parts."""
    p = np.asarray(positions, np.float64)
    parts = []
    start, cur = 0, 0.0
    for i in range(1, len(p)):
        d = float(np.linalg.norm(p[i - 1] - p[i]))
        if cur + d > max_length:
            parts.append((start, i - 1))
            start, cur = i - 1, 0.0  # the new part starts with the previous pose
        cur += d
    parts.append((start, len(p) - 1))
    return parts


def padded_ranges(parts, n_poses, padding=PADDING):
    """(start, end) inclusive index ranges of the submaps as written (:136-147).  Raises IndexError,
    as the reference's part_previous[-30] / part_next[29] do, when a neighbouring part holds fewer than
    ``padding`` poses."""
    out = []
    for k, (s, e) in enumerate(parts):
        for j in ([k - 1] if k > 0 else []) + ([k + 1] if k < len(parts) - 1 else []):
            if parts[j][1] - parts[j][0] + 1 < padding:
                raise IndexError(f"part {j} has {parts[j][1] - parts[j][0] + 1} poses, fewer than the {padding}-pose "
                                 f"padding of its neighbour {k} (fdt_segment_and_optimize_submaps.py:139,146)")
        lo = s - (padding - 1) if k > 0 else s
        hi = e + (padding - 1) if k < len(parts) - 1 else e
        if lo < 0 or hi >= n_poses:
            raise IndexError(f"part {k} is too short for the reference's {padding}-pose padding")
        out.append((lo, hi))
    return out


def middle_points(positions, parts):
    """The midpoint of each part's first and last pose (:33-37,120-121), saved by the reference as
    submaps_middlepoints.npy."""
    p = np.asarray(positions, np.float64)
    return np.stack([(p[s] + p[e]) / 2 for s, e in parts])


def poses_from_tum(tum, zero_origin=False):
    """pose_utils.build_poses_from_df(df, zero_origin) (:387-409): rows [t x y z qx qy qz qw] ->
    (N, 4, 4) float32 (the quaternion normalised, as scipy's Rotation.from_quat does; fp64, then fp32).
    ``zero_origin``: every pose is expressed relative to the first (the inverse of the first pose, formed
    as [R^T | -R^T t], applied on the left, in fp64), as the driver does for whole runs (:208-213)."""
    tum = np.asarray(tum, np.float64)
    q = tum[:, 4:8] / np.linalg.norm(tum[:, 4:8], axis=1, keepdims=True)
    x, y, z, w = q.T
    Rm = np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                   np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                   np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], 1)
    P = np.zeros((len(tum), 4, 4))
    P[:, :3, :3] = Rm
    P[:, :3, 3] = tum[:, 1:4]
    P[:, 3, 3] = 1.0
    if zero_origin:
        inv = np.eye(4)
        inv[:3, :3] = P[0, :3, :3].T
        inv[:3, 3] = -P[0, :3, :3].T @ P[0, :3, 3]
        P = inv[None] @ P
    return P.astype(np.float32)


def world_cube_from_poses(poses, ray_range, padding=0.3):
    """compute_world_cube (LiDAR branch, submap) of (N, 4, 4) poses: (scale, shift) with shift = -origin,
    in the reference's float32 arithmetic."""
    P = np.asarray(poses, np.float32).reshape(-1, 4, 4)
    m = np.float32(ray_range[1])
    # lidar_view_corners (:287-294), homogeneous, in the reference's order
    V = np.array([[sx * m, sy * m, sz * m, 1.0] for sz in (-1, 1) for sx in (-1, 1) for sy in (-1, 1)], np.float32)
    corners = np.einsum("nij,kj->nki", P[:, :3, :], V).reshape(-1, 3)  # c2l[:3, :] @ corners.T per pose
    pts = np.concatenate([corners, P[:, :3, 3]], 0)
    mn, mx = pts.min(0), pts.max(0)
    origin = (mn + (mx - mn) / np.float32(2)).astype(np.float32)
    scale = np.float32(np.linalg.norm((mx - mn).astype(np.float32)) / (np.float32(2) * np.sqrt(np.float32(3))))
    return float(scale * np.float32(1 + padding)), (-origin).astype(np.float32)
