"""Edge cases of the C ABI on the GPU: empty batches, sizes the kernels do not support (error
codes + messages, no launch), ragged sample counts (S not a power of two / not a multiple of 64)
through the full step, and the tcnn-style RuntimeError surface."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import _lib
    _lib.lib()
    return _lib


def test_empty_batches_are_noops(L):
    s = L.stream()
    z = torch.empty(0, dtype=torch.float32, device="cuda")
    d = L.grid_desc()
    assert L.lib().lnr_sample_ogm(None, 0, 512, None, 100, 1.0, None, None, 0, 0, None, None, s) == 0
    assert L.lib().lnr_hashgrid_fwd_rays(L.ctypes.byref(d), None, None, 0, 512, None, None, 0, None, 0, s) == 0
    assert L.lib().lnr_hashgrid_bwd_rays(L.ctypes.byref(d), None, None, 0, 512, None, 0, None, None, None, None, 0, 0,
                                        s) == 0
    assert L.lib().lnr_field_render(None, None, 0, None, None, 0, 512, 0, 1.0, None, 0, 0, None, None, None, None,
                                    s) == 0
    assert L.lib().lnr_rgb_render(None, 4, None, 0, None, None, 0, 512, None, s) == 0
    assert L.lib().lnr_adam_step(None, None, None, None, None, 0, 1, 0.01, 0.9, 0.999, 1e-8, None, s) == 0
    L.call("lnr_count_opaque", z, 0, 1.0, None, torch.zeros(1, device="cuda"), s)
    torch.cuda.synchronize()


def test_zero_ray_step_writes_zero_gradient_and_loss(L):
    """A step over an empty batch (one rank's share of a tiny global batch, or a compacted batch with no
    valid ray) stores a zero gradient and finalizes the loss scalars: nothing of the previous step's
    MLP or table gradient survives into Adam (lnr_field_train with LNR_LP_DW_OVERWRITE, the hash-grid
    backward's overwrite contract at N = 0)."""
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    cfg = S_.StepConfig(n_samples=64)
    st = S_.FieldState(cfg, device="cuda:0", table_init=0.5)
    win = syn.make_window("quad", 1, seed=2)
    rays, dgt = syn.build_batch(win, "quad", 64, 0, "RANDOM", seed=4)
    rays, dgt = rays.cuda(), dgt.cuda()
    eng = S_.StepEngine(st, rays.shape[0], seed=1)
    eng.step(rays, dgt, global_step=1, scale=121.426537, far_ref=float(rays[0, 12]))
    torch.cuda.synchronize()
    assert float(st.grad.abs().max()) > 0 and float(eng.loss_out[0]) != 0
    eng.step(rays[:0], dgt[:0], global_step=2, scale=121.426537, far_ref=float(rays[0, 12]),
             n_rays_global=rays.shape[0])
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(st.grad)) == 0
    assert float(eng.loss_out[0]) == 0.0 and float(eng.loss_out[5]) == 0.0


def test_unsupported_sizes_raise(L):
    s = L.stream()
    rays = torch.zeros(4, 13, device="cuda")
    zz = torch.zeros(4, 100, device="cuda")
    out = torch.zeros(4, device="cuda")
    with pytest.raises(RuntimeError, match="multiple of 64"):
        L.call("lnr_field_render", torch.zeros(3072, dtype=torch.float16, device="cuda"),
               torch.zeros(16, 400, dtype=torch.int32, device="cuda"), 400, rays, zz, 4, 100, 0, 1.0, None, 0, 0, out,
               out, out, None, s)
    with pytest.raises(RuntimeError, match="render strategy"):
        L.call("lnr_field_render", torch.zeros(3072, dtype=torch.float16, device="cuda"),
               torch.zeros(16, 512, dtype=torch.int32, device="cuda"), 512, rays, torch.zeros(4, 128, device="cuda"), 4,
               128, 7, 1.0, None, 0, 0, out, out, out, None, s)
    with pytest.raises(RuntimeError, match="n_hidden_layers"):
        L.call("lnr_rgb_render", None, 6, None, 0, rays, None, 4, 128, None, s)
    with pytest.raises(RuntimeError, match="n_samples"):
        L.call("lnr_sample_ogm", rays, 4, 7, torch.zeros(8, device="cuda"), 2, 1.0, None, None, 0, 0, zz, None, s)
    from loner_amd import rendering
    with pytest.raises(ValueError, match="render strategy"):
        from loner_amd import evaluate as E
        from loner_amd import step as S_
        E.DepthRenderer(S_.FieldState(S_.StepConfig(), device="cuda:0"), n_samples=64, chunk=4).render(
            rays, 0, "threshold")
    del rendering


@pytest.mark.parametrize("S", [64, 192, 320])
def test_ragged_sample_counts_step(L, S):
    """S/2 not a multiple of 64 (block sampler), S not a power of two (padded sort): the whole step
    runs, its loss is finite and the gradient is deterministic.  (The fused field kernels take S in
    multiples of 64, one wave per 64 samples; other S raise, see test_unsupported_sizes_raise.)"""
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    win = syn.make_window("quad", 1, seed=3)
    rays, dgt = syn.build_batch(win, "quad", 40, 0, "RANDOM", seed=2)
    rays, dgt = rays.cuda(), dgt.cuda()
    grads = []
    for _ in range(2):
        st = S_.FieldState(S_.StepConfig(n_samples=S), device="cuda:0", table_init=0.3)
        eng = S_.StepEngine(st, rays.shape[0], seed=4)
        out = eng.step(rays, dgt, global_step=1, scale=syn.CUBES["quad"][0], far_ref=float(rays[0, -1]))
        torch.cuda.synchronize()
        assert np.isfinite(out.cpu().numpy()[0])
        grads.append(st.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_status_flags_replace_the_nan_assert(L):
    """The device status word: a clean step leaves it 0; a NaN loss sets LNR_STATUS_NAN_LOSS and
    check_status raises the reference's "NaN Loss Encountered" (optimizer.py:854); an infinite
    sigma sets LNR_STATUS_SIGMA_CLIPPED and warns once (nerf_tcnn.py:74-78) without failing."""
    import warnings
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    win = syn.make_window("quad", 1, seed=3)
    rays, dgt = syn.build_batch(win, "quad", 40, 0, "RANDOM", seed=2)
    rays, dgt = rays.cuda(), dgt.cuda()
    sc, far = syn.CUBES["quad"][0], float(rays[0, -1])
    st = S_.FieldState(S_.StepConfig(n_samples=64), device="cuda:0", table_init=0.3)
    eng = S_.StepEngine(st, rays.shape[0], seed=4)
    eng.step(rays, dgt, global_step=1, scale=sc, far_ref=far)
    assert eng.check_status() == 0
    eng.step(rays, dgt, global_step=2, scale=float("nan"), far_ref=far)
    with pytest.raises(RuntimeError, match="NaN Loss Encountered"):
        eng.check_status()
    assert eng.check_status() == 0  # cleared by the read
    st2 = S_.FieldState(S_.StepConfig(n_samples=64), device="cuda:0", table_init=0.3)
    with torch.no_grad():
        st2.params[:2048].fill_(1e4)  # fp16 hidden activations overflow -> sigma inf -> clipped
        st2.params[2048:3072].fill_(1e4)
    st2.refresh_shadow()
    eng2 = S_.StepEngine(st2, rays.shape[0], seed=4)
    eng2.step(rays, dgt, global_step=1, scale=sc, far_ref=far)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        bits = eng2.check_status()
    assert bits & L.STATUS_SIGMA_CLIPPED
    assert any("Clipping infinite outputs" in str(x.message) for x in w)


def test_status_scan_flags_nonfinite(L):
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    x = torch.ones(100000, device="cuda")
    L.call("lnr_status_scan", x, x.numel(), L.STATUS_NONFINITE_OUTPUT, st, L.stream())
    assert int(st.item()) == 0
    x[77777] = float("inf")
    L.call("lnr_status_scan", x, x.numel(), L.STATUS_NONFINITE_OUTPUT, st, L.stream())
    assert int(st.item()) == L.STATUS_NONFINITE_OUTPUT
    x[77777] = float("nan")
    st.zero_()
    L.call("lnr_status_scan", x, x.numel(), 1, st, L.stream())
    assert int(st.item()) == 1
