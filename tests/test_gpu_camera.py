"""Colour-head training, the camera phase (optimizer.py:541-688,861-894): lnr_build_camera_rays and
lnr_rgb_train against oracle/camera.py, and the CameraStepEngine end to end (GPU only).

Gradient tolerance (parity unpinned: tcnn's fp16 backward is not vendored): the HIP backward runs
the chain in fp16 MFMA operands with per-wave power-of-two scaling and fp32 accumulation; against
the fp64 restatement from the same fp16 activations the relative L2 error of d_enc and of every
weight matrix's gradient must stay below 1e-2."""
import numpy as np
import pytest
import torch

from oracle import camera as ocam
from oracle import mlp as omlp

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


def _rays(R, rng):
    o = rng.uniform(-0.5, 0.5, (R, 3))
    d = rng.normal(size=(R, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, -d, np.zeros((R, 2)), np.full((R, 1), 0.01), np.full((R, 1), 1.0)], 1)
    return rays.astype(np.float32)


def _rel(got, ref):
    return np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)


@pytest.mark.parametrize("n_hidden", [1, 2, 4])
def test_rgb_train_vs_oracle(L, n_hidden):
    from loner_amd.camera import ColorState
    rng = np.random.default_rng(n_hidden)
    R, S = 96, 64
    N = R * S
    cs = ColorState(n_hidden_layers=n_hidden, device="cuda:0", seed=3)
    enc16 = rng.uniform(-1, 1, (N, 32)).astype(np.float16)
    enc_lm = enc16.view(np.uint32).reshape(N, 16).T.copy()  # level-major half2
    rays = _rays(R, rng)
    w = rng.dirichlet(np.full(S, 0.3), R) * rng.uniform(0.2, 0.95, (R, 1))
    w = w.astype(np.float32)
    mats = omlp.unflatten(host(cs.mlp_f16), omlp.layer_shapes(48, 3, 64, n_hidden))
    rgb0, _, _, _ = ocam.rgb_forward(enc16, rays, w, mats, S)
    gt = (rgb0 + rng.choice([-1, 1], rgb0.shape) * rng.uniform(0.05, 0.2, rgb0.shape)).astype(np.float32)
    ref = ocam.rgb_train(enc16, rays, w, gt, mats, S)

    dev = "cuda:0"
    t_enc = torch.from_numpy(enc_lm.view(np.int32)).to(dev)
    t_rays, t_w, t_gt = (torch.from_numpy(a).to(dev) for a in (rays, w, gt))
    rgb = torch.empty(R, 3, device=dev)
    loss = torch.zeros(1, device=dev)
    d_enc = torch.empty(16, N, 2, device=dev)
    P = int(L.lib().lnr_rgb_mlp_params(n_hidden))
    d_w = torch.full((P,), float("nan"), device=dev)
    nb = int(L.lib().lnr_rgb_train_workspace_bytes(n_hidden, R))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    lmax = torch.full((16,), 7.0, dtype=torch.float32, device=dev)  # overwritten
    L.call("lnr_rgb_train", cs.mlp_f16, n_hidden, t_enc, N, t_rays, t_w, t_gt, R, S, 1.0 / (3 * R), rgb, loss,
           d_enc, d_w, ws, nb, lmax, L.stream(torch.device(dev)))
    # the colour grid backward's record scales: max |d_enc| per level, exactly
    np.testing.assert_array_equal(host(lmax), np.abs(host(d_enc)).max(axis=(1, 2)))
    got_rgb = host(rgb)
    assert np.abs(got_rgb - ref["rgb"]).max() < 5e-3
    assert abs(float(host(loss)[0]) - ref["loss"]) < 1e-3 * ref["loss"] + 1e-6
    de = host(d_enc).transpose(1, 0, 2).reshape(N, 32)
    assert _rel(de, ref["d_enc"]) < 1e-2, _rel(de, ref["d_enc"])
    dw = host(d_w)
    assert np.isfinite(dw).all()
    off = 0
    for (o, i) in omlp.layer_shapes(48, 3, 64, n_hidden):
        g, r = dw[off:off + o * i].reshape(o, i), ref["d_w"][off:off + o * i].reshape(o, i)
        if o == 16:  # padded output rows 3..15 get no gradient
            assert np.all(g[3:] == 0)
            g, r = g[:3], r[:3]
        assert _rel(g, r) < 1e-2, (o, i, _rel(g, r))
        off += o * i
    # deterministic: a second call gives the same bits
    d_w2 = torch.empty_like(d_w)
    L.call("lnr_rgb_train", cs.mlp_f16, n_hidden, t_enc, N, t_rays, t_w, t_gt, R, S, 1.0 / (3 * R), rgb, loss,
           d_enc, d_w2, ws, nb, None, L.stream(torch.device(dev)))
    assert torch.equal(d_w, d_w2)


def test_camera_rays_vs_oracle(L):
    from loner_amd import camera as C
    rng = np.random.default_rng(0)
    W, H = 40, 30
    K = np.array([[30.0, 0, 19.5], [0, 30.0, 14.5], [0, 0, 1]])
    dirs = C.pinhole_directions(W, H, K).numpy()
    img = rng.uniform(0, 1, (H * W, 3)).astype(np.float32)
    ang = 0.4
    pose = np.array([[np.cos(ang), -np.sin(ang), 0, 3.0], [np.sin(ang), np.cos(ang), 0, -2.0], [0, 0, 1, 0.5]])
    cube = dict(scale_factor=20.0, shift=[1.0, 2.0, -0.5])
    fr = C.CameraFrames(dirs, W, H, [img], [pose], cube, (1.0, 50.0), n_rays_per_kf=100, seed=1, device="cuda:0")
    for it in (0, 3):
        n = fr.n_rays(it)
        rays = torch.empty(n, 13, device="cuda:0")
        inten = torch.empty(n, 3, device="cuda:0")
        assert fr.build(it, rays, inten) == n
        lo, hi = fr.iteration_slice(it)
        pix = host(fr.perm[0][lo:hi])
        ro, io = ocam.build_camera_rays(dirs, img, pix, pose.astype(np.float32), 20.0, [1.0, 2.0, -0.5], 1.0, W)
        np.testing.assert_allclose(host(rays), ro, rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(host(inten), io)
    assert fr.n_rays(0) == 99 and fr.n_rays(1) == 100  # the reference's first-iteration off-by-one
    assert len(set(host(fr.perm[0]).tolist())) == fr.keep


def _camera_setup(seed=0, n_kf=2, W=48, H=32, n_per_kf=128, skip_zero=None):
    from loner_amd import camera as C
    from loner_amd import step as S_
    st = S_.FieldState(S_.StepConfig(), device="cuda:0", table_init=0.5, seed=7)
    torch.manual_seed(3)
    with torch.no_grad():
        st.params[2048:3072].mul_(8.0)
        st.occ.normal_(0, 2)
    st.refresh_shadow()
    K = np.array([[40.0, 0, (W - 1) / 2], [0, 40.0, (H - 1) / 2], [0, 0, 1]])
    dirs = C.pinhole_directions(W, H, K)
    yy, xx = np.mgrid[0:H, 0:W]
    imgs, poses = [], []
    for k in range(n_kf):
        img = np.stack([0.5 + 0.4 * np.sin(xx / 7.0 + k), 0.5 + 0.4 * np.cos(yy / 5.0), 0.3 + 0.2 * (xx > W / 2)], -1)
        imgs.append(img.reshape(-1, 3).astype(np.float32))
        a = 0.3 * k
        poses.append(np.array([[np.cos(a), 0, np.sin(a), 0.5 * k], [0, 1, 0, 0], [-np.sin(a), 0, np.cos(a), 0]]))
    cube = dict(scale_factor=20.0, shift=[0.0, 0.0, 0.0])
    fr = C.CameraFrames(dirs, W, H, imgs, poses, cube, (0.5, 40.0), n_rays_per_kf=n_per_kf, seed=seed,
                        device="cuda:0")
    cs = C.ColorState(4, device="cuda:0", seed=5)
    eng = C.CameraStepEngine(st, cs, n_rays=n_kf * n_per_kf, n_samples=128, lr=0.01, seed=seed, skip_zero=skip_zero)
    return fr, cs, eng


def test_camera_step_learns_and_is_deterministic(L):
    fr, cs, eng = _camera_setup()
    R = fr.n_rays(1)
    rays = torch.empty(R, 13, device="cuda:0")
    inten = torch.empty(R, 3, device="cuda:0")
    losses = []
    for rep in range(25):
        for it in range(fr.n_iter):
            n = fr.build(it, rays, inten)
            losses.append(float(eng.step(rays[:n], inten[:n]).item()))
    assert np.isfinite(losses).all()
    assert np.mean(losses[-6:]) < 0.5 * np.mean(losses[:6]), (losses[:6], losses[-6:])
    assert torch.isfinite(cs.params).all()
    # same seed, same inputs -> the same parameters bit for bit
    fr2, cs2, eng2 = _camera_setup()
    fr3, cs3, eng3 = _camera_setup()
    for it in range(3):
        n = fr2.build(it, rays, inten)
        eng2.step(rays[:n], inten[:n])
        eng3.step(rays[:n], inten[:n])
    assert torch.equal(cs2.params, cs3.params)


@pytest.mark.parametrize("skip_zero", [True, False])
def test_camera_two_shards_match_single_batch(L, skip_zero):
    """Data-parallel camera phase: two engines on the two halves of the rays (draws keyed by global
    ray index, loss normalised by the global ray count, one gradient all-reduce) reproduce the
    single-engine iteration, and both replicas hold identical parameters after Adam; with the default
    zero-weight skipping and with the exact full path (skip_zero=False: every sample's records)."""
    import threading
    from loner_amd import camera as C
    fr, cs_ref, eng_ref = _camera_setup(skip_zero=skip_zero)
    R = fr.n_rays(1)
    rays = torch.empty(R, 13, device="cuda:0")
    inten = torch.empty(R, 3, device="cuda:0")
    fr.build(1, rays, inten)
    loss_ref = float(eng_ref.step(rays, inten, global_step=7).item())
    g_ref = host(cs_ref.grad).copy()

    bar = threading.Barrier(2)
    slots = [None, None]

    def make_allreduce(rank):
        def allreduce(t):
            torch.cuda.synchronize()
            slots[rank] = t
            bar.wait()
            if rank == 0:
                tot = slots[0] + slots[1]
                slots[0].copy_(tot)
                slots[1].copy_(tot)
                torch.cuda.synchronize()
            bar.wait()
        return allreduce

    states = [_camera_setup()[1], _camera_setup()[1]]
    field = eng_ref.field
    losses = [None, None]

    def run(rank):
        s0, s1 = (0, R // 2) if rank == 0 else (R // 2, R)
        eng = C.CameraStepEngine(field, states[rank], n_rays=s1 - s0, n_samples=128, lr=0.01, seed=0,
                                 allreduce=make_allreduce(rank), ray_offset=s0, skip_zero=skip_zero)
        losses[rank] = float(eng.step(rays[s0:s1].contiguous(), inten[s0:s1].contiguous(), global_step=7,
                                      n_rays_global=R).item())

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert losses[0] + losses[1] == pytest.approx(loss_ref, rel=1e-5)
    g = host(states[0].grad)
    assert _rel(g, g_ref) < 1e-5
    assert torch.equal(states[0].params, states[1].params)


def test_camera_skip_zero_matches_default(L):
    """CameraStepEngine(skip_zero=True, the default) (zero-weight samples: no colour gathers, backward counts
    only non-zero d_enc) gives the full path's gradient bit for bit: the skipped samples contribute exactly 0, and
    the backward's fixed-point unit depends on the sample count alone, not on how many records it places."""
    from loner_amd import camera as C
    fr, cs_a, eng_def = _camera_setup()
    eng_a = C.CameraStepEngine(eng_def.field, cs_a, n_rays=eng_def.R, n_samples=128, lr=0.01, seed=0, skip_zero=False)
    _, cs_b, eng_ref = _camera_setup()
    eng_b = C.CameraStepEngine(eng_ref.field, cs_b, n_rays=eng_ref.R, n_samples=128, lr=0.01, seed=0, skip_zero=True)
    R = fr.n_rays(1)
    rays = torch.empty(R, 13, device="cuda:0")
    inten = torch.empty(R, 3, device="cuda:0")
    fr.build(1, rays, inten)
    la = float(eng_a.step(rays, inten, global_step=5).item())
    lb = float(eng_b.step(rays, inten, global_step=5).item())
    assert la == lb
    assert float((eng_b.weights[:R] == 0).float().mean()) > 0.05  # the path is exercised
    assert torch.equal(cs_a.grad, cs_b.grad)


def test_camera_live_count_matches_backward_count(L, monkeypatch):
    """skip_zero with the records counted by the live colour encode (lnr_hashgrid_fwd_rays_live_ws, the
    default) against counted by the backward's own pass (LONER_CAM_LIVE_COUNT=0): the same records, so the
    same gradient bit for bit (no live sample of this batch has a zero d_enc), and the same Adam step."""
    from loner_amd import camera as C
    fr, cs_a, eng_def = _camera_setup()
    monkeypatch.setenv("LONER_CAM_LIVE_COUNT", "0")
    eng_a = C.CameraStepEngine(eng_def.field, cs_a, n_rays=eng_def.R, n_samples=128, lr=0.01, seed=0, skip_zero=True)
    monkeypatch.setenv("LONER_CAM_LIVE_COUNT", "1")
    _, cs_b, eng_ref = _camera_setup()
    eng_b = C.CameraStepEngine(eng_ref.field, cs_b, n_rays=eng_ref.R, n_samples=128, lr=0.01, seed=0, skip_zero=True)
    assert not eng_a.live_count and eng_b.live_count
    R = fr.n_rays(1)
    rays = torch.empty(R, 13, device="cuda:0")
    inten = torch.empty(R, 3, device="cuda:0")
    fr.build(1, rays, inten)
    for it in range(2):
        la = float(eng_a.step(rays, inten, global_step=5 + it).item())
        lb = float(eng_b.step(rays, inten, global_step=5 + it).item())
        assert la == lb
        assert torch.equal(cs_a.grad, cs_b.grad)
    assert torch.equal(cs_a.params, cs_b.params)
