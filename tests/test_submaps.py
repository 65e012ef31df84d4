"""C5 trajectory segmentation (loner_amd.submaps), restated from
examples/fdt_segment_and_optimize_submaps.py:24-25,86-147 and pose_utils.py:222-314 on the committed
haveri keyframe trajectory.  The script is not importable here (ROS / open3d imports): its split is
pinned by the properties its loop guarantees and by the boundaries it yields on this trajectory
(parity unpinned: restated from the text).  CPU only."""
import os

import numpy as np

from loner_amd import submaps as SM

TUM = np.load(os.path.join(os.path.dirname(__file__), "golden", "haveri_keyframe_trajectory.npz"))["tum"]


def _steps(p):
    return np.linalg.norm(np.diff(p, axis=0), axis=1)


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


def test_padding_and_world_cubes():
    parts = SM.split_trajectory(TUM[:, 1:4])
    ranges = SM.padded_ranges(parts, len(TUM))
    # previous part's poses [-30, -1) before, next part's [1, 30) after (29 each)
    assert ranges == [(0, 311 + 29), (311 - 29, 622 + 29), (622 - 29, 934 + 29), (934 - 29, 1093)]
    for lo, hi in ranges:
        scale, shift = SM.world_cube_from_poses(TUM[lo:hi + 1, 1:4], (2.5, 45.0))
        p = TUM[lo:hi + 1, 1:4]
        # every pose's +-45 m box lies inside the cube [-1, 1]^3 after (x + shift) / scale
        q = (np.concatenate([p - 45.0, p + 45.0]) + shift) / scale
        assert np.abs(q).max() <= 1.0
        # the cube is the padded bounding sphere of those boxes (pose_utils.py:306-314)
        ext = (p.max(0) + 45.0) - (p.min(0) - 45.0)
        assert np.isclose(scale, np.linalg.norm(ext) / (2 * np.sqrt(3)) * 1.3, rtol=1e-5)


def test_submap_window_is_its_segment():
    from loner_amd import synthetic as syn
    scans, cube, info = syn.submap_window(5, n_kf=4, seed=1)
    assert info["n_parts"] == 4 and info["part"] == 1 and info["padded"] == [282, 651]
    t = np.stack([s["pose"][:3, 3].numpy() for s in scans])
    np.testing.assert_allclose(t[0], TUM[282, 1:4], atol=1e-5)
    np.testing.assert_allclose(t[-1], TUM[651, 1:4], atol=1e-5)
    assert float(cube.scale_factor[0]) == info["cube_scale"]
