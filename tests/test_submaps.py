"""C5 trajectory segmentation and per-submap world cubes (loner_amd.submaps) against
tests/golden/submaps.npz: tests/golden/make_golden.py (``r3``) ran the reference's own
examples/fdt_segment_and_optimize_submaps.py:39-162 on the committed haveri keyframe trajectory and then,
per written submap trajectory, pose_utils.build_poses_from_df(df, False) + compute_world_cube(..., submap=)
as examples/fdt_optimize_implicit_map.py:208-233 does.  CPU only."""
import os

import numpy as np
import pytest

from loner_amd import submaps as SM

G = os.path.join(os.path.dirname(__file__), "golden")
TUM = np.load(os.path.join(G, "haveri_keyframe_trajectory.npz"))["tum"]
SUB = np.load(os.path.join(G, "submaps.npz"))


def _steps(p):
    return np.linalg.norm(np.diff(p, axis=0), axis=1)


def _golden_rows():
    off = SUB["row_offsets"]
    return [SUB["row_index"][off[k]:off[k + 1]] for k in range(len(off) - 1)]


def test_split_boundaries_and_properties():
    pos = TUM[:, 1:4]
    parts = SM.split_trajectory(pos)
    assert parts == [(0, 311), (311, 622), (622, 934), (934, 1093)]
    d = _steps(pos)
    for k, (s, e) in enumerate(parts):
        assert d[s:e].sum() <= SM.MAX_LENGTH  # each part's path is at most 50 m
        if k + 1 < len(parts):
            assert parts[k + 1][0] == e  # the next part starts with this part's last pose
            assert d[s:e + 1].sum() > SM.MAX_LENGTH  # one more step would have passed 50 m
    assert parts[0][0] == 0 and parts[-1][1] == len(pos) - 1
    np.testing.assert_allclose(SM.middle_points(pos, parts), SUB["middle_points"], rtol=0, atol=1e-12)


def test_padded_ranges_match_reference_files():
    """The poses each reference submap file holds, in order, are the padded index range."""
    ranges = SM.padded_ranges(SM.split_trajectory(TUM[:, 1:4]), len(TUM))
    rows = _golden_rows()
    assert len(ranges) == len(rows) == len(SUB["names"])
    for (lo, hi), idx in zip(ranges, rows):
        np.testing.assert_array_equal(idx, np.arange(lo, hi + 1))


def test_world_cubes_match_reference():
    """compute_world_cube with the corners rotated by every pose (pose_utils.py:296-298)."""
    ranges = SM.padded_ranges(SM.split_trajectory(TUM[:, 1:4]), len(TUM))
    for k, (lo, hi) in enumerate(ranges):
        scale, shift = SM.world_cube_from_poses(SM.poses_from_tum(TUM[lo:hi + 1]), tuple(SUB["ray_range"]))
        np.testing.assert_allclose(scale, SUB["scale"][k], rtol=1e-6)
        np.testing.assert_allclose(shift, SUB["shift"][k], rtol=1e-6, atol=1e-5)
        # every pose's rotated +-45 m cube lies inside [-1, 1]^3 after (x + shift) / scale
        P = SM.poses_from_tum(TUM[lo:hi + 1]).astype(np.float64)
        c = np.array([[sx, sy, sz] for sx in (-45, 45) for sy in (-45, 45) for sz in (-45, 45)], np.float64)
        q = (np.einsum("nij,kj->nki", P[:, :3, :3], c) + P[:, None, :3, 3] + shift) / scale
        assert np.abs(q).max() <= 1.0


def test_short_neighbour_raises_like_reference():
    """A part with fewer poses than the padding: the reference's part_next[k] / part_previous[-30]
    raise IndexError (fdt_segment_and_optimize_submaps.py:139,146), before any submap is optimised."""
    assert bool(SUB["short_raises"]) and int(SUB["short_calls"]) == 0
    short = SUB["short_tum"]
    parts = SM.split_trajectory(short[:, 1:4])
    assert min(e - s + 1 for s, e in parts) < SM.PADDING
    with pytest.raises(IndexError):
        SM.padded_ranges(parts, len(short))


def test_submap_window_is_its_segment():
    from loner_amd import synthetic as syn
    scans, cube, info = syn.submap_window(5, n_kf=4, seed=1)
    assert info["n_parts"] == 4 and info["part"] == 1 and info["padded"] == [282, 651]
    t = np.stack([s["pose"][:3, 3].numpy() for s in scans])
    np.testing.assert_allclose(t[0], TUM[282, 1:4], atol=1e-5)
    np.testing.assert_allclose(t[-1], TUM[651, 1:4], atol=1e-5)
    assert float(cube.scale_factor[0]) == info["cube_scale"]
    np.testing.assert_allclose(info["cube_scale"], SUB["scale"][1], rtol=1e-6)
    np.testing.assert_allclose(cube.shift.numpy(), SUB["shift"][1], rtol=1e-6, atol=1e-5)


def test_compute_world_cube_every_branch_golden():
    """loner_amd.rays.compute_world_cube against the reference's own compute_world_cube
    (tests/golden/world_cube_camera.npz, make_golden.py r4): the camera-frustum branch (Fusion Portable
    calibrations, examples/fdt_optimize_implicit_map.py:195-233) with one K / image size and with one per
    pose, re-based and submap poses; the LiDAR branch; the trajectory bounding box with and without a camera.
    fp32 matrix products in another order: rtol 1e-5."""
    import torch
    from loner_amd.rays import compute_world_cube
    g = np.load("tests/golden/world_cube_camera.npz")
    tum = g["tum"]
    zero = torch.from_numpy(SM.poses_from_tum(tum, zero_origin=True))
    raw = torch.from_numpy(SM.poses_from_tum(tum))
    c2l, K, Ks = torch.from_numpy(g["camera_to_lidar"]), torch.from_numpy(g["K"]), torch.from_numpy(g["Ks"])
    hw = tuple(int(v) for v in g["image_size"])
    bbox = dict(x=list(g["bbox"][0]), y=list(g["bbox"][1]), z=list(g["bbox"][2]))
    cases = {
        "camera_rebased": (c2l, K, hw, zero, (1.0, 50.0), None, None),
        "camera_submap_per_pose": (c2l, Ks, torch.from_numpy(g["sizes"]), raw, (1.0, 50.0), None, "submap_1"),
        "lidar_rebased": (None, None, None, zero, (2.5, 45.0), None, None),
        "bbox_camera": (c2l, K, hw, None, (1.0, 50.0), bbox, None),
        "bbox_lidar": (None, None, None, None, (1.0, 75.0), bbox, None),
    }
    for name, (c, k, s, poses, rr, bb, sub) in cases.items():
        wc = compute_world_cube(c, k, s, poses, rr, padding=0.3, traj_bounding_box=bb, submap=sub)
        np.testing.assert_allclose(float(wc.scale_factor[0]), g[f"{name}_scale"], rtol=1e-5, err_msg=name)
        np.testing.assert_allclose(wc.shift.numpy(), g[f"{name}_shift"], rtol=1e-5, atol=1e-4, err_msg=name)
    assert float(g["bbox_lidar_scale"]) == pytest.approx(121.426537, rel=1e-6)  # the quad cube
