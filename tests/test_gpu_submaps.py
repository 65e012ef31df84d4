"""C5 (fdt_segment_and_optimize_submaps): one optimiser step of a submap on the HIP path, in the
submap's own world cube (loner_amd.submaps, pinned to the reference in tests/test_submaps.py), against
the oracle step on the same rays and draws (GPU only)."""
import numpy as np
import pytest
import torch

from oracle import rays as orays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import _lib
    _lib.lib()
    return _lib


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("part", [0, 2])
def test_submap_step_vs_oracle(L, part):
    import bench
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    from oracle import step as ostep
    kind, _, _, _, strat, Sn, preset = syn.CONFIGS["C5"]
    scans, cube, info = syn.submap_window(part, n_kf=2, seed=40 + part)
    assert info["part"] == part
    rr = syn.SENSORS[kind]["ray_range"]
    win = RayWindow(scans, cube, rr, n_lidar=96, n_sky=16, strategy=strat, device="cuda:0")
    assert win.all_valid
    scale = float(cube.scale_factor[0])
    loss_cfg = bench.LOSS_PRESETS[preset]
    st = S_.FieldState(S_.StepConfig(n_samples=Sn, occ_lr=1e-3, loss=S_.LossConfig.from_dict(loss_cfg)),
                       device="cuda:0")
    eng = S_.StepEngine(st, win.n_slots, seed=91)
    gstep = 20  # an OGM step (N_iters_acc = 10)
    out = host(eng.step_window(win, global_step=gstep))
    rays, dgt = host(eng.rays), host(eng.depth_gt)
    # the rays are the submap cube's: built by the oracle from the same selection
    key = L.step_key(91, gstep)
    sel = orays.select_window(scans, strat, 96, 16, key)
    o_rays, o_dep, o_valid = orays.build_window(scans, [s["pose"].numpy() for s in scans], sel, rr, scale,
                                                cube.shift.numpy())
    assert o_valid.all()
    np.testing.assert_allclose(rays, o_rays, rtol=2e-6, atol=2e-7)
    np.testing.assert_array_equal(dgt, o_dep)
    assert np.abs(rays[:, :3]).max() < 1.0  # origins inside the submap's cube (ray_utils.py:301-303)
    # the step: sampler, then field + loss + backward + Adam + OGM on the GPU's samples
    _, z_ref, _ = ostep.train_step(ostep.OracleField(), rays, dgt, scale, loss_cfg, gstep, n_samples=Sn, key=key)
    z = host(eng.z)
    assert np.abs(z - z_ref).max() < 4e-6, np.abs(z - z_ref).max()
    field = ostep.OracleField()
    loss_ref, _, g_ref = ostep.train_step(field, rays, dgt, scale, loss_cfg, gstep, n_samples=Sn, key=key, z=z,
                                          occ_lr=1e-3)
    assert abs(out[0] - loss_ref) <= 1e-4 * abs(loss_ref), (out[0], loss_ref)
    g = host(st.grad)[:st.n_params]
    assert np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref) < 1e-4
    np.testing.assert_allclose(host(st.occ).reshape(100, 100, 100), field.occ, rtol=1e-5, atol=1e-7)
