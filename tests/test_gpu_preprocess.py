"""Per-keyframe scan preprocessing on the GPU (loner_amd.preprocess) against the numpy oracle
(oracle/preprocess.py): motion compensation (sensors.py:169-231) and sky rays
(fdt_optimize_implicit_map_utils.py:38-77)."""
import numpy as np
import pytest
import torch

from oracle import preprocess as opre

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import preprocess
    return preprocess


def _pose(yaw, pitch, t):
    from scipy.spatial.transform import Rotation
    m = np.eye(4)
    m[:3, :3] = Rotation.from_euler("zy", [yaw, pitch]).as_matrix()
    m[:3, 3] = t
    return m


def test_motion_compensate_vs_oracle(P):
    from loner_amd import synthetic as syn
    scan = syn.make_window("quad", 1, seed=4)[0]
    dirs = scan["directions"].numpy().astype(np.float64)
    dists = scan["distances"].numpy().astype(np.float64)
    n = dists.shape[0]
    ts = np.linspace(0, 0.1, n)
    start, end = _pose(0.3, 0.02, [1.0, 2.0, 0.5]), _pose(0.45, -0.01, [1.8, 2.3, 0.6])
    d_dev = torch.from_numpy(dirs.T.astype(np.float32)).cuda().contiguous()
    r_dev = torch.from_numpy(dists.astype(np.float32)).cuda()
    t_dev = torch.from_numpy(ts.astype(np.float32)).cuda()
    P.motion_compensate(d_dev, r_dev, t_dev, (start, end), (0.0, 0.1), end)
    torch.cuda.synchronize()
    idx = np.arange(0, n, 97)
    od, orr = opre.motion_compensate(dirs[:, idx], dists[idx], ts[idx], start, end, 0.0, 0.1, end)
    np.testing.assert_allclose(d_dev.cpu().numpy()[idx].T, od, atol=2e-5)
    np.testing.assert_allclose(r_dev.cpu().numpy()[idx], orr, rtol=2e-5, atol=2e-5)
    # identity motion leaves the scan unchanged
    d2 = torch.from_numpy(dirs.T.astype(np.float32)).cuda().contiguous()
    r2 = torch.from_numpy(dists.astype(np.float32)).cuda()
    P.motion_compensate(d2, r2, t_dev, (start, start), (0.0, 0.1), start)
    np.testing.assert_allclose(d2.cpu().numpy(), dirs.T, atol=2e-6)
    np.testing.assert_allclose(r2.cpu().numpy(), dists, rtol=2e-6)


@pytest.mark.parametrize("kind", ["quad", "forest", "canteen"])
def test_sky_rays_vs_oracle(P, kind):
    from loner_amd import synthetic as syn
    scan = syn.make_window(kind, 1, seed=2)[0]
    dirs = scan["directions"].numpy()
    pose = scan["pose"].numpy()
    got = P.sky_rays(torch.from_numpy(dirs.T.copy()).cuda(), pose).cpu().numpy().T
    ref = opre.sky_rays(dirs, pose[:3, :3])
    # 1-degree bins from float32 atan2: a point on a bin's rounding edge may land one bin over
    assert abs(got.shape[1] - ref.shape[1]) <= max(3, 0.01 * ref.shape[1]), (got.shape, ref.shape)
    if ref.shape[1]:
        # every GPU direction has an oracle direction within float32 rounding, and vice versa
        dots = got.T @ ref
        assert np.mean(dots.max(1) > 1 - 1e-6) > 0.99 and np.mean(dots.max(0) > 1 - 1e-6) > 0.99
        assert np.allclose(np.linalg.norm(got, axis=0), 1, atol=1e-5)
