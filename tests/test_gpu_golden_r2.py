"""The HIP path against the round-2 reference fixtures (tests/golden/make_golden.py r2), GPU only:
camera rays (CameraRayDirections.build_rays, ray_utils.py:175-212), the compositing weights of the
colour render (raw2outputs, rendering_tcnn.py:219-295), Adam fed tcnn's fp16-rounded gradients
(optimizer.py:257-265,460) and the checkpoint's module paths and sizes (mapper.py:161-175)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import _lib
    _lib.lib()
    return _lib


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def test_camera_rays_golden(L):
    g = np.load(os.path.join(GOLDEN, "camera_rays.npz"))
    W, H = int(g["width"]), int(g["height"])
    cam = L.CameraDesc()
    cam.width, cam.height, cam.channels = W, H, 3
    cam.scale, cam.r_min = float(g["scale"]), float(g["ray_range"][0])
    for i in range(3):
        cam.shift[i] = float(g["shift"][i])
    for i, v in enumerate(g["pose"][:3].reshape(-1).tolist()):
        cam.pose[i] = v
    pix = g["pixels"].astype(np.int64)
    n = len(pix)
    rays = torch.empty(n, 13, dtype=torch.float32, device="cuda")
    inten = torch.empty(n, 3, dtype=torch.float32, device="cuda")
    L.call("lnr_build_camera_rays", L.ctypes.byref(cam), cu(g["directions"]), cu(g["image"].reshape(-1, 3)), cu(pix),
           n, rays, inten, L.stream())
    got, ref = host(rays), g["rays"]
    np.testing.assert_allclose(got[:, 0:9], ref[:, 0:9], rtol=1e-6, atol=2e-7)
    np.testing.assert_array_equal(got[:, 9:11], ref[:, 9:11])
    np.testing.assert_allclose(got[:, 11:13], ref[:, 11:13], rtol=1e-6)
    np.testing.assert_array_equal(host(inten), g["intensities"])


def test_colour_render_weights_golden(L):
    """The weights the colour map composites with (sigma_only=False path of raw2outputs): lnr_composite
    on the fixture's sigma, z and noise; then rgb = sum w c + 1 - sum w with the fixture's colours."""
    g = np.load(os.path.join(GOLDEN, "camera_loss.npz"))
    rays, z, sig, noise = g["rays"], g["z"], g["sigma"], g["noise"]
    R, S = z.shape
    w = torch.empty(R, S, dtype=torch.float32, device="cuda")
    d = torch.empty(R, dtype=torch.float32, device="cuda")
    L.call("lnr_composite", cu(rays), cu(z), cu(sig), R, S, 0, 1.0, cu(noise), 0, 0, w, d, None, None, L.stream())
    wg = host(w)
    np.testing.assert_allclose(wg, g["weights"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(host(d), g["depth"], rtol=1e-5, atol=1e-6)
    rgb = (wg[..., None].astype(np.float64) * g["colors"]).sum(1) + (1 - wg.astype(np.float64).sum(1, keepdims=True))
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-5, atol=1e-5)


def _passthrough_colour_mlp(n_hidden_layers=4):
    """tcnn-flat weights of a colour network that hands its first three inputs through: W0 puts relu(x_j)
    and relu(-x_j) on hidden units 2j and 2j + 1, the hidden layers are identities on them and the output
    layer takes their difference, so the network's output j is x_j exactly (every value fp16, every
    product by +-1)."""
    mats = [np.zeros((64, 48), np.float32)] + [np.eye(64, dtype=np.float32)] * (n_hidden_layers - 1) + \
        [np.zeros((16, 64), np.float32)]
    for j in range(3):
        mats[0][2 * j, j], mats[0][2 * j + 1, j] = 1.0, -1.0
        mats[-1][j, 2 * j], mats[-1][j, 2 * j + 1] = 1.0, -1.0
    return np.concatenate([m.reshape(-1) for m in mats]).astype(np.float16)


def test_colour_map_golden_through_rgb_render(L):
    """lnr_rgb_render's own colour map (rgb = sum w c + 1 - sum w, rendering_tcnn.py:283-289) on the
    fixture's colours: the colour-grid encodings carry the colours' logits into a pass-through network
    (_passthrough_colour_mlp), so the kernel's sigmoid gives back the reference's colours (to fp16) and
    its compositing runs on the HIP weights of the fixture's sigma, z and noise."""
    g = np.load(os.path.join(GOLDEN, "camera_loss.npz"))
    rays, z, sig, noise, col = g["rays"], g["z"], g["sigma"], g["noise"], g["colors"].astype(np.float64)
    R, S = z.shape
    w = torch.empty(R, S, dtype=torch.float32, device="cuda")
    d = torch.empty(R, dtype=torch.float32, device="cuda")
    L.call("lnr_composite", cu(rays), cu(z), cu(sig), R, S, 0, 1.0, cu(noise), 0, 0, w, d, None, None, L.stream())
    c = np.clip(col, 1e-7, 1 - 1e-7)
    logit = np.clip(np.log(c) - np.log1p(-c), -15.0, 15.0).astype(np.float16).reshape(R * S, 3)
    feats = np.zeros((16, R * S, 2), np.float16)  # level-major half2: level l holds features 2l, 2l + 1
    feats[0, :, 0], feats[0, :, 1], feats[1, :, 0] = logit[:, 0], logit[:, 1], logit[:, 2]
    enc = cu(feats.view(np.uint32).reshape(16, R * S))
    mlp = cu(_passthrough_colour_mlp().view(np.uint16))
    rgb = torch.empty(R, 3, dtype=torch.float32, device="cuda")
    L.call("lnr_rgb_render", mlp, 4, enc, R * S, cu(rays), w, R, S, rgb, L.stream())
    got, wg = host(rgb), host(w).astype(np.float64)
    # the kernel's arithmetic: colour = fp16(sigmoid(fp16 logit)), fp32 sums of w c
    col16 = (1.0 / (1.0 + np.exp(-logit.astype(np.float32)))).astype(np.float16).astype(np.float64).reshape(R, S, 3)
    emu = (wg[..., None] * col16).sum(1) + (1 - wg.sum(1, keepdims=True))
    np.testing.assert_allclose(got, emu, rtol=1e-5, atol=2e-6)
    # and the reference's rgb: the colours differ from the fixture's by the fp16 logit and colour roundings
    # (|dc| <= 0.23 * 2^-11 + 2^-12)
    np.testing.assert_allclose(got, g["rgb"], rtol=0, atol=5e-4)


def test_adam_with_tcnn_fp16_gradients_golden(L):
    """lnr_adam_step fed the fp16-rounded gradients tcnn's binding hands back, against torch.optim.Adam on
    an fp32 parameter (the reference's literal fp16-parameter Adam is non-finite after one step at these
    gradient magnitudes: test_oracle_golden.test_adam_on_tcnn_fp16_params_golden)."""
    g = np.load(os.path.join(GOLDEN, "adam_fp16.npz"))
    n = g["p0"].shape[0]
    tp = cu(g["p0"])
    tm = torch.zeros(n, dtype=torch.float32, device="cuda")
    tv = torch.zeros(n, dtype=torch.float32, device="cuda")
    sh = torch.empty(n, dtype=torch.float16, device="cuda")
    for k in range(g["grad_f16"].shape[0]):
        L.call("lnr_adam_step", tp, sh, cu(g["grad_f16"][k]), tm, tv, n, k + 1, float(g["lr"]), 0.9, 0.999, 1e-8,
               None, L.stream())
        np.testing.assert_allclose(host(tp), g["params_fp32"][k], rtol=2e-6, atol=1e-8)
    np.testing.assert_allclose(host(tv), g["exp_avg_sq_fp32"], rtol=1e-6, atol=1e-30)


def test_checkpoint_matches_reference_keys(L):
    from loner_amd import camera as C
    from loner_amd import checkpoint as ck
    from loner_amd import step as S_
    keys = json.load(open(os.path.join(GOLDEN, "ckpt_keys.json")))
    st = S_.FieldState(S_.StepConfig(), device="cuda:0")
    cs = C.ColorState(device="cuda:0")
    d = ck.build_ckpt(st, 7, other_params=ck.color_params(cs))
    assert {k: list(v.shape) for k, v in d["network_state_dict"].items()} == keys["network_state_dict"]
    assert {k: list(v.shape) for k, v in d["occ_model_state_dict"].items()} == keys["occ_model_state_dict"]


def test_adam_ranges_match_single_launches(L):
    """lnr_adam_step_ranges (the sharded optimiser's chunks in one launch) is bitwise lnr_adam_step on
    each range, tails (n not a multiple of 4) and a NULL shadow included."""
    g = np.load(os.path.join(GOLDEN, "adam_fp16.npz"))
    p0, gr = g["p0"].astype(np.float32), g["grad_f16"][0].astype(np.float32)
    cuts = [(0, 1000), (1024, 1024 + 777), (2048, 4096)]
    a = [cu(p0.copy()) for _ in range(2)]
    m = [torch.zeros(len(p0), device="cuda") for _ in range(2)]
    v = [torch.zeros(len(p0), device="cuda") for _ in range(2)]
    sh = [torch.zeros(len(p0), dtype=torch.float16, device="cuda") for _ in range(2)]
    gd = cu(gr)
    for step in (1, 2):
        for k, (o, e) in enumerate(cuts):
            L.call("lnr_adam_step", a[0][o:e], sh[0][o:e] if k else None, gd[o:e], m[0][o:e], v[0][o:e], e - o, step,
                   1e-3, 0.9, 0.999, 1e-8, None, L.stream())
        rng = (L.AdamRange * len(cuts))()
        for k, (o, e) in enumerate(cuts):
            rng[k] = L.AdamRange(L.ptr(a[1][o:e]), L.ptr(sh[1][o:e]) if k else None, L.ptr(gd[o:e]), L.ptr(m[1][o:e]),
                                 L.ptr(v[1][o:e]), e - o)
        L.call("lnr_adam_step_ranges", rng, len(cuts), step, 1e-3, 0.9, 0.999, 1e-8, None, L.stream())
    torch.cuda.synchronize()
    for x, y in ((a[0], a[1]), (m[0], m[1]), (v[0], v[1]), (sh[0], sh[1])):
        assert torch.equal(x, y)
    assert not torch.equal(a[1], cu(p0))
