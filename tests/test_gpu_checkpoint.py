"""Reference-format checkpoints (loner_amd.checkpoint; mapper.py:161-175,
fdt_optimize_implicit_map.py:344-359): round trip through torch.save / torch.load(weights_only=True),
key layout of the tcnn-compatible Model, and a resumed step identical to an uninterrupted one."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NERF_CFG = dict(enable_view_dependence=True,
                pos_encoding_sigma=dict(otype="HashGrid", n_levels=16, n_features_per_level=2, log2_hashmap_size=18,
                                        base_resolution=16),
                sigma_network=dict(otype="FullyFusedMLP", activation="ReLU", output_activation="None", n_neurons=64,
                                   n_hidden_layers=1),
                pos_encoding_intensity=dict(otype="HashGrid", n_levels=16, n_features_per_level=2,
                                            log2_hashmap_size=19, base_resolution=16),
                dir_encoding_intensity=dict(otype="SphericalHarmonics", degree=4),
                intensity_network=dict(otype="FullyFusedMLP", activation="ReLU", output_activation="None",
                                       n_neurons=64, n_hidden_layers=4))


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import checkpoint as C
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    return C, S_, syn


def test_roundtrip_and_resume(mods, tmp_path):
    C, S_, syn = mods
    cfg = S_.StepConfig(n_samples=128)
    win = syn.make_window("quad", 1, seed=2)
    rays, dgt = syn.build_batch(win, "quad", 64, 0, "RANDOM", seed=1)
    rays, dgt = rays.cuda(), dgt.cuda()
    far = float(rays[0, -1])
    scale = syn.CUBES["quad"][0]
    a = S_.FieldState(cfg, device="cuda:0", table_init=0.3)
    ea = S_.StepEngine(a, 64, seed=5)
    for it in range(1, 12):  # crosses an OGM update (step 10)
        ea.step(rays, dgt, global_step=it, scale=scale, far_ref=far)
    # fp32 master written as fp32 here so the resumed run is bit-identical
    ck = C.build_ckpt(a, 11, poses=torch.eye(4)[None], params_dtype=torch.float32)
    path = tmp_path / "final.tar"
    torch.save(ck, path)
    b = S_.FieldState(cfg, device="cuda:0", seed=999)
    loaded = C.load_checkpoint(str(path), b)
    assert loaded["global_step"] == 11 and b.adam_step == a.adam_step
    assert torch.equal(b.params, a.params) and torch.equal(b.m, a.m) and torch.equal(b.v, a.v)
    assert torch.equal(b.occ, a.occ) and torch.equal(b.shadow, a.shadow)
    assert set(loaded) == {"global_step", "network_state_dict", "optimizer_state_dict", "poses",
                           "occ_model_state_dict", "occ_optimizer_state_dict"}
    assert loaded["occ_model_state_dict"]["occupancy_grid"].shape == (1, 1, 100, 100, 100)
    eb = S_.StepEngine(b, 64, seed=5)
    oa = ea.step(rays, dgt, global_step=12, scale=scale, far_ref=far).cpu().numpy()
    ob = eb.step(rays, dgt, global_step=12, scale=scale, far_ref=far).cpu().numpy()
    np.testing.assert_array_equal(oa, ob)
    assert torch.equal(a.params, b.params)


def test_default_fp16_params_and_model_keys(mods):
    """The default checkpoint stores tcnn's fp16 params under the reference Model's module paths,
    and the tcnn-compatible Model loads it with load_state_dict."""
    C, S_, syn = mods
    from loner_amd import model as M
    st = S_.FieldState(S_.StepConfig(), device="cuda:0", table_init=0.2)
    model = M.Model(dict(model_type="nerf_decoupled", num_colors=3, nerf_config=NERF_CFG, ray_range=[1, 75],
                         render=dict(N_samples_train=512, N_samples_test=2048, retraw=True, perturb=1.0,
                                     raw_noise_std=1.0, chunk=16384, netchunk=0)))
    sd = model.state_dict()
    assert C.SIGMA_KEY in sd and sd[C.SIGMA_KEY].numel() == st.n_params
    ck = C.build_ckpt(st, 3, other_params=sd)
    net = ck["network_state_dict"]
    assert net[C.SIGMA_KEY].dtype == torch.float16 and set(net) == set(sd)
    model.load_state_dict(net)
    got = model.get_sigma_parameters()[0].detach()
    assert torch.equal(got.cpu(), st.params[:st.n_params].half().float().cpu())
