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


# ------------------------------------------------------------------ round-2 fixtures (make_golden.py r2)
def test_camera_rays_golden(golden):
    """CameraRayDirections.build_rays (ray_utils.py:175-212) and get_ray_directions (:62-124) as the
    reference computes them: the oracle's restatement and the host-side pinhole table."""
    import torch

    from loner_amd.camera import pinhole_directions
    from oracle import camera as ocam
    g = golden("camera_rays")
    W = int(g["width"])
    dirs = pinhole_directions(W, int(g["height"]), g["K"]).numpy()
    np.testing.assert_array_equal(dirs, g["directions"])
    np.testing.assert_array_equal(g["grid_x"][:, 0], np.arange(W * int(g["height"])) % W)  # i = column
    T = g["pose"]
    img = g["image"].reshape(-1, 3)
    rays, inten = ocam.build_camera_rays(g["directions"], img, g["pixels"], T[:3], g["scale"], g["shift"],
                                         g["ray_range"][0], W)
    ref = g["rays"]
    np.testing.assert_allclose(rays[:, 0:9], ref[:, 0:9], rtol=1e-6, atol=2e-7)
    np.testing.assert_array_equal(rays[:, 9:11], ref[:, 9:11])
    np.testing.assert_allclose(rays[:, 11:13], ref[:, 11:13], rtol=1e-6)
    np.testing.assert_array_equal(inten, g["intensities"])
    assert torch.is_tensor(torch.from_numpy(dirs))


def test_colour_compositing_and_camera_loss_golden(golden):
    """raw2outputs with sigma_only=False and a white background (rendering_tcnn.py:219-295) and
    compute_loss_camera's l1 loss with its per-sample colour gradient (optimizer.py:861-894), from the
    reference run through a fixed-colour stand-in model."""
    from oracle import camera as ocam
    g = golden("camera_loss")
    rays, far = g["rays"], g["rays"][:, -1:]
    out = orender.raw2outputs(g["sigma"], g["z"], rays[:, 3:6], g["noise"], far)
    np.testing.assert_allclose(out["weights"], g["weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(out["depth"], g["depth"], rtol=1e-5)
    rgb = ocam.composite_rgb(g["weights"], g["colors"])
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-6, atol=1e-6)
    loss, dcol = ocam.rgb_loss_grad(g["rgb"], g["gt"], g["weights"], rays.shape[0])
    assert loss == pytest.approx(float(g["loss"]), rel=1e-6)
    np.testing.assert_allclose(dcol, g["d_colors"], rtol=1e-6, atol=1e-12)


def test_adam_on_tcnn_fp16_params_golden(golden):
    """torch.optim.Adam (optimizer.py:257-265,460) on fp16 params with tcnn's fp16 gradients: with the
    reference's eps = 1e-8, (1 - beta2) g^2 underflows fp16 for every |g| < ~7.7e-3 and the update
    divides by a zero denominator, so almost every parameter (and every untouched table entry, 0/0)
    is non-finite after one step.  The same steps on an fp32 parameter (the master this build keeps,
    as tcnn's binding keeps fp32 params and hands the native code an fp16 copy) are exact Adam in
    fp32 and match the oracle's restatement."""
    g = golden("adam_fp16")
    bad16 = ~np.isfinite(g["params_fp16"][0])
    assert bad16.mean() > 0.9 and bad16[3000:].all()
    assert np.isfinite(g["params_fp32"]).all()
    p = g["p0"].copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for k in range(g["grad_f16"].shape[0]):
        ooptim.adam_step(p, g["grad_f16"][k], m, v, k + 1, float(g["lr"]))
        np.testing.assert_allclose(p, g["params_fp32"][k], rtol=2e-6, atol=1e-8)  # fp32 rounding of p - step
    np.testing.assert_allclose(v, g["exp_avg_sq_fp32"], rtol=1e-6, atol=1e-30)


def test_checkpoint_keys_golden():
    """The checkpoint's module paths and sizes against the reference's own Model / OccupancyGridModel
    state_dict keys (make_golden.py r2, tcnn replaced by a shape-only stand-in)."""
    import json
    import os

    from loner_amd import _lib as L
    from loner_amd import checkpoint as ck
    keys = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ckpt_keys.json")))
    net = keys["network_state_dict"]
    assert set(net) == {ck.SIGMA_KEY, ck.COLOR_GRID_KEY, ck.DIR_ENC_KEY, ck.COLOR_MLP_KEY}
    assert keys["occ_model_state_dict"] == {"occupancy_grid": [1, 1, 100, 100, 100]}
    sigma = L.grid_desc(16, 2, 18, 16)
    colour = L.grid_desc(16, 2, 19, 16)
    assert net[ck.SIGMA_KEY] == [L.SIGMA_MLP_PARAMS + 2 * int(sigma.n_entries)]
    assert net[ck.COLOR_GRID_KEY] == [2 * int(colour.n_entries)]
    assert net[ck.DIR_ENC_KEY] == [0]
    assert net[ck.COLOR_MLP_KEY] == [64 * 48 + 3 * 64 * 64 + 16 * 64]  # 48 -> 64 x4 -> 3 (padded to 16)
