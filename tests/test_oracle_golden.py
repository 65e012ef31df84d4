"""Pin the CPU oracle against golden vectors produced by the reference's own code
(tests/golden/make_golden.py).  CPU only."""
import ast

import numpy as np
import pytest

from oracle import loss as oloss
from oracle import optim as ooptim
from oracle import rays as orays
from oracle import render as orender


def test_build_lidar_rays(golden):
    g = golden("rays")
    rays, depths = orays.build_lidar_rays(g["dirs"], g["dist"], g["pose"], g["ray_range"], g["scale"], g["shift"])
    assert rays.shape == g["rays"].shape
    np.testing.assert_allclose(rays, g["rays"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(depths, g["depths"], rtol=1e-6)
    far = orays.get_far_val(g["rays"][:, :3], g["rays"][:, 3:6], True)
    np.testing.assert_allclose(far, g["far_val"], rtol=1e-6)


def test_world_cube(golden):
    g = golden("world_cube")
    for name, bbox, rr in [("quad", dict(x=[-5, 50], y=[-25, 15], z=[-3, 10]), [1, 75]),
                           ("haveri_bbox", dict(x=[-10, 10], y=[-10, 10], z=[-10, 10]), [2.5, 45])]:
        scale, shift = orays.world_cube_bbox(bbox, rr, padding=0.3)
        np.testing.assert_allclose(scale, g[name][0], rtol=1e-6)
        np.testing.assert_allclose(shift, g[name][1:], rtol=1e-6, atol=1e-6)
    # quad cube scale 121.426537, shift [-22.5, 5, -3.5]
    np.testing.assert_allclose(g["quad"], [121.426537, -22.5, 5.0, -3.5], rtol=1e-6)


def test_sample_pdf(golden):
    g = golden("sample_pdf")
    s = orender.sample_pdf(g["bins"], g["weights"], 256, g["u"])
    np.testing.assert_allclose(s, g["samples"], rtol=1e-5, atol=5e-6)


def test_grid_sample(golden):
    g = golden("samplers")
    v = orender.grid_sample_3d(g["occ"], g["pts"])
    np.testing.assert_allclose(v, g["interp"], rtol=1e-5, atol=1e-6)


def test_samplers(golden):
    g = golden("samplers")
    z = orender.ogm_samples(g["rays"], 512, g["occ"], g["u_jitter"], g["u_pdf"])
    np.testing.assert_allclose(z, g["z_ogm"], rtol=1e-5, atol=5e-6)
    zu = orender.uniform_samples(g["rays"], 64, g["u_jitter_uniform"])
    np.testing.assert_allclose(zu, g["z_uniform"], rtol=1e-6, atol=1e-8)


def test_raw2outputs(golden):
    g = golden("composite")
    out = orender.raw2outputs(g["sigma"], g["z"], g["rays"][:, 3:6], g["noise"], g["rays"][:, -1:])
    np.testing.assert_allclose(out["weights"], g["weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out["depth"], g["depth"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["opacity"], g["opacity"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["variance"], g["variance"], rtol=1e-3, atol=1e-8)


def test_raw2outputs_adjusted(golden):
    g = golden("composite")
    out = orender.raw2outputs_adjusted(g["sigma"], g["z"], g["rays"][:, 3:6])
    np.testing.assert_allclose(out["weights"], g["adj_weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(out["depth"], g["adj_depth"])
    np.testing.assert_allclose(out["variance"], g["adj_variance"], rtol=1e-3, atol=1e-8)


def test_loss_helpers(golden):
    g = golden("loss_helpers")
    np.testing.assert_allclose(oloss.get_weights_gt(g["s"], g["g"], g["eps"]), g["weights_gt"], rtol=1e-5, atol=5e-6)
    np.testing.assert_array_equal(oloss.logits_grad(g["s"], g["g"]), g["logits_grad"])
    np.testing.assert_allclose(oloss.js_divergence(g["g"], np.float32(0.5 / 3.0), g["m2"], g["s2"]), g["js"], rtol=1e-5,
                               atol=1e-6)


@pytest.mark.parametrize("tag", ["l1js_default", "l1js_haveri", "l1los", "l2js"])
def test_compute_loss_and_grad(golden, tag):
    g = golden("loss_" + tag)
    cfg = ast.literal_eval(str(g["cfg_json"]))
    occ = golden("samplers")["occ"]
    rays = g["rays"]
    z = orender.ogm_samples(rays, 512, occ, g["u_jitter"], g["u_pdf"])
    np.testing.assert_allclose(z, g["z"], rtol=1e-5, atol=5e-6)
    far = rays[:, -1:]
    out = orender.raw2outputs(g["sigma"], g["z"], rays[:, 3:6], g["noise"], far)
    np.testing.assert_allclose(out["weights"], g["weights"], rtol=1e-4, atol=1e-6)
    res = oloss.lidar_loss(out["weights"], g["z"], out["depth"], out["opacity"], g["depth_gt"], far, g["scale"], cfg,
                           int(g["global_step"]), int(g["iteration_idx"]))
    assert res["loss"] == pytest.approx(float(g["loss"]), rel=2e-5)
    assert res["mean_eps"] == pytest.approx(float(g["depth_eps"]), rel=1e-5)
    ds = orender.composite_backward(g["sigma"], g["z"], rays[:, 3:6], g["noise"], far, res["g_w"], res["g_depth"],
                                    res["g_opacity"])
    # fp32 autograd of the reference: same sign decisions for the L1 terms as fp32 weights
    ref = g["dsigma"].reshape(ds.shape)
    err = np.abs(ds - ref).max() / (np.abs(ref).max() + 1e-30)
    assert err < 1e-5, err
    # fp64 autograd: differs only where |w - w_gt| flips sign below fp32 resolution (L1 kink)
    ref64 = g["dsigma64"].reshape(ds.shape)
    assert np.linalg.norm(ds - ref64) / np.linalg.norm(ref64) < 5e-3
    # OGM update (optimizer.py:897-908): sparse delta
    grid = occ.copy()
    ooptim.ogm_step(grid, rays, g["z"], g["depth_gt"], g["scale"], float(g["occ_lr"]))
    delta = grid.reshape(-1) - occ.reshape(-1)
    idx = g["occ_delta_idx"]
    assert set(np.flatnonzero(delta).tolist()) <= set(idx.tolist()) | set(np.flatnonzero(np.abs(delta) > 0).tolist())
    np.testing.assert_allclose(delta[idx], g["occ_delta"], rtol=1e-3, atol=2e-7)
