"""Trajectory segmentation into submaps (C5), restated from
examples/fdt_segment_and_optimize_submaps.py:24-25,86-147 and the submap branch of
src/common/pose_utils.py:222-314 (compute_world_cube).  Host-side numpy; the script itself is not
importable here (it pulls the ROS / open3d stack), so its split is restated from the text and pinned
by tests/test_submaps.py's properties and boundaries (parity unpinned).

Split (:86-116): walk the ground-truth poses accumulating the distance between consecutive positions;
when adding the next step would pass MAX_LENGTH (50 m) the part closes, and the next part starts WITH
the previous pose (consecutive parts share their boundary pose) and a zero distance.
Padding (:131-146): every part but the first is written with the previous part's poses [-30, -1)
before it, every part but the last with the next part's poses [1, 30) after it: in trajectory
indices the padded submap is the contiguous range [start - 29, end + 29].
World cube (pose_utils.py:222-314 with submap set and no camera): the poses are used as they are (not
re-based on the first pose); the points are every pose's position and the 8 corners of a cube of
half-size max range around it; origin = the points' box centre, scale = |box diagonal| / (2 sqrt 3)
* (1 + padding)."""
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
    """(start, end) inclusive index ranges of the submaps as written (:131-146)."""
    out = []
    for k, (s, e) in enumerate(parts):
        lo = s - (padding - 1) if k > 0 else s
        hi = e + (padding - 1) if k < len(parts) - 1 else e
        if lo < 0 or hi >= n_poses:
            raise IndexError(f"part {k} is too short for the reference's {padding}-pose padding")
        out.append((lo, hi))
    return out


def world_cube_from_poses(positions, ray_range, padding=0.3):
    """compute_world_cube (LiDAR only, submap): (scale, shift) with shift = -origin."""
    t = np.asarray(positions, np.float32).reshape(-1, 3)
    m = np.float32(ray_range[1])
    corners = np.array([[sx * m, sy * m, sz * m] for sz in (-1, 1) for sx in (-1, 1) for sy in (-1, 1)], np.float32)
    pts = np.concatenate([(t[:, None, :] + corners[None]).reshape(-1, 3), t], 0)
    mn, mx = pts.min(0), pts.max(0)
    origin = (mn + (mx - mn) / np.float32(2)).astype(np.float32)
    scale = np.float32(np.linalg.norm((mx - mn).astype(np.float32)) / (np.float32(2) * np.sqrt(np.float32(3))))
    return float(scale * np.float32(1 + padding)), (-origin).astype(np.float32)
