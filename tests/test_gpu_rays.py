"""On-device ray selection + building (lnr_build_lidar_rays, loner_amd.rays.RayWindow) against the
numpy oracle (oracle/rays.py), and the optimiser step driven by it (GPU only).

Reference behaviour restated: Optimizer._do_iterate_optimizer's selection (src/mapping/optimizer.py:
363-386), KeyFrame.build_lidar_rays (src/mapping/keyframe.py:75-105), LidarRayDirections.build_lidar_rays
+ get_far_val (src/common/ray_utils.py:31-60, 269-322)."""
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


def _window(kind, n_kf, seed):
    from loner_amd import synthetic as syn
    return syn.make_window(kind, n_kf, seed=seed), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"]


def _oracle(scans, wc, rr, strategy, n_lidar, n_sky, key):
    sel = orays.select_window(scans, strategy, n_lidar, n_sky, key)
    poses = [s["pose"].numpy() for s in scans]
    rays, dep, valid = orays.build_window(scans, poses, sel, rr, float(wc.scale_factor[0]), wc.shift.numpy())
    idx = np.concatenate([np.concatenate([li, si]) for li, si in sel])
    return rays, dep, valid, idx


@pytest.mark.parametrize("kind,strategy,n_sky", [("quad", "RANDOM", 0), ("forest", "MASK", 64), ("quad", "MASK", 16)])
def test_build_matches_oracle(L, kind, strategy, n_sky):
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window(kind, 3, seed=11)
    win = RayWindow(scans, wc, rr, n_lidar=512, n_sky=n_sky, strategy=strategy)
    key = L.step_key(5, 17)
    pidx = torch.empty(win.n_slots, dtype=torch.int32, device="cuda")
    rays, dep, valid, _, far = win.build(key, point_index=pidx)
    o_rays, o_dep, o_valid, o_idx = _oracle(scans, wc, rr, strategy, 512, n_sky, key)
    assert win.n_slots == len(o_idx)
    np.testing.assert_array_equal(host(pidx), o_idx)              # selection: bit-exact
    np.testing.assert_array_equal(host(valid).astype(bool), o_valid)
    np.testing.assert_allclose(host(rays), o_rays, rtol=2e-6, atol=2e-7)  # fp32 matmul order (BLAS) only
    np.testing.assert_array_equal(host(dep), o_dep)                # range / scale: one division
    assert host(far)[0] == pytest.approx(o_rays[np.flatnonzero(o_valid)[0], 12], rel=1e-6)
    if strategy == "MASK":  # distinct points per keyframe part (randperm prefix: no repeats)
        off = win.ray_off_host
        sel = host(win.n_sel)
        for k in range(win.n_kf):
            li = o_idx[off[k]:off[k] + sel[k]]
            assert len(np.unique(li)) == len(li)


def test_mask_short_trunk_counts(L):
    """A keyframe with fewer trunk points than int(0.75 n) keeps all of them (randperm prefix of a
    shorter list, optimizer.py:377-378): the batch shrinks exactly as the reference's does."""
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("quad", 2, seed=3)
    s0 = dict(scans[0])
    z = (s0["directions"] * s0["distances"])[2]
    trunk = torch.nonzero((0.5 < z) & (z < 8)).reshape(-1)
    other = torch.nonzero(~((0.5 < z) & (z < 8))).reshape(-1)
    keep = torch.cat([trunk[:100], other[:2000]])
    s0["directions"], s0["distances"] = s0["directions"][:, keep].contiguous(), s0["distances"][keep].contiguous()
    scans = [s0, scans[1]]
    win = RayWindow(scans, wc, rr, n_lidar=512, strategy="MASK")
    assert host(win.n_sel)[0] == min(100, len(trunk)) + 128
    key = L.step_key(1, 2)
    pidx = torch.empty(win.n_slots, dtype=torch.int32, device="cuda")
    win.build(key, point_index=pidx)
    o_idx = _oracle(scans, wc, rr, "MASK", 512, 0, key)[3]
    np.testing.assert_array_equal(host(pidx), o_idx)


def test_sharded_build_equals_unsharded(L):
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("forest", 4, seed=2)
    win = RayWindow(scans, wc, rr, n_lidar=512, n_sky=64, strategy="MASK")
    key = L.step_key(9, 3)
    full = [host(t) for t in win.build(key)[:3]]
    half = win.n_slots // 2 + 7
    a = [host(t) for t in win.build(key, 0, half)[:3]]
    b = [host(t) for t in win.build(key, half, win.n_slots - half)[:3]]
    for f, x, y in zip(full, a, b):
        np.testing.assert_array_equal(f, np.concatenate([x, y]))


def test_invalid_rays_are_dropped(L):
    """A pose close to the world-cube face: rays leaving the cube within 1 m are invalid
    (ray_utils.py:319-322); the window notices and step_window compacts them away."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("quad", 2, seed=4)
    scale, shift = float(wc.scale_factor[0]), wc.shift.numpy()
    s1 = dict(scans[1])
    pose = s1["pose"].clone()
    pose[0, 3] = float(0.9995 * scale - shift[0])  # origin x just inside the +x face
    s1["pose"] = pose
    scans = [scans[0], s1]
    win = RayWindow(scans, wc, rr, n_lidar=256, strategy="RANDOM")
    assert not win.all_valid
    key = L.step_key(3, 1)
    _, _, valid, _, _ = win.build(key)
    o_valid = _oracle(scans, wc, rr, "RANDOM", 256, 0, key)[2]
    np.testing.assert_array_equal(host(valid).astype(bool), o_valid)
    assert 0 < o_valid.sum() < len(o_valid)
    cfg = S_.StepConfig(n_samples=64)
    st = S_.FieldState(cfg, device="cuda:0")
    eng = S_.StepEngine(st, win.n_slots, seed=3)
    out = host(eng.step_window(win, global_step=1))
    assert np.isfinite(out[0])


def test_step_window_equals_step_on_built_rays(L):
    """The step driven by on-device ray building is the step on the same rays built outside it."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("forest", 2, seed=8)
    win = RayWindow(scans, wc, rr, n_lidar=128, n_sky=16, strategy="MASK")
    assert win.all_valid
    cfg = S_.StepConfig(n_samples=128)
    outs, grads = [], []
    for mode in ("window", "rays"):
        st = S_.FieldState(cfg, device="cuda:0", table_init=0.5)
        eng = S_.StepEngine(st, win.n_slots, seed=21)
        if mode == "window":
            out = eng.step_window(win, global_step=4)
        else:
            rays, dgt, _, _, far = win.build(L.step_key(21, 4))
            out = eng.step(rays, dgt, global_step=4, scale=win.scale, far_ref=float(host(far)[0]))
        outs.append(host(out).copy())
        grads.append(host(st.grad).copy())
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(grads[0], grads[1])


def test_prefetched_compaction_equals_synchronous(L):
    """step_window on a window with invalid rays: the next step's build + compaction prefetched on a
    side stream (double-buffered) gives bitwise the synchronous path's losses and parameters, over
    consecutive steps, a skipped step (the prefetch is discarded) and an OGM step."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("quad", 2, seed=4)
    scale, shift = float(wc.scale_factor[0]), wc.shift.numpy()
    s1 = dict(scans[1])
    pose = s1["pose"].clone()
    pose[0, 3] = float(0.9995 * scale - shift[0])
    s1["pose"] = pose
    win = RayWindow([scans[0], s1], wc, rr, n_lidar=256, strategy="RANDOM")
    assert not win.all_valid
    res = []
    for prefetch in (True, False):
        st = S_.FieldState(S_.StepConfig(n_samples=64, occ_lr=1e-3), device="cuda:0", table_init=0.5)
        eng = S_.StepEngine(st, win.n_slots, seed=3)
        eng.prefetch = prefetch
        outs = [host(eng.step_window(win, global_step=g)).copy() for g in (8, 9, 10, 12, 13)]
        torch.cuda.synchronize()
        res.append((outs, host(st.params).copy(), host(st.occ).copy()))
    for a, b in zip(res[0][0], res[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][2], res[1][2])


def test_pipelined_build_and_sampling_equals_plain(L):
    """step_window's pipeline (step k + 1's ray build and sampling enqueued on a side stream after
    step k, double-buffered; no sampling prefetch after an OGM step) gives bitwise the plain path's
    losses, parameters, occupancy grid and last samples, across OGM steps (global steps 10, 20) and a
    skipped step (the prefetch is discarded)."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow
    scans, wc, rr = _window("forest", 2, seed=8)
    win = RayWindow(scans, wc, rr, n_lidar=128, n_sky=16, strategy="MASK")
    assert win.all_valid
    res = []
    for pipeline in (False, True):
        st = S_.FieldState(S_.StepConfig(n_samples=128, occ_lr=1e-3), device="cuda:0", table_init=0.5)
        eng = S_.StepEngine(st, win.n_slots, seed=7)
        eng.pipeline = pipeline
        outs = [eng.step_window(win, global_step=g).clone() for g in (8, 9, 10, 11, 13, 14, 19, 20, 21)]
        torch.cuda.synchronize()
        res.append(([host(o) for o in outs], host(st.params).copy(), host(st.occ).copy(), host(eng.z).copy(),
                    host(eng.rays).copy()))
    for r in res[1:]:
        for a, b in zip(res[0][0], r[0]):
            np.testing.assert_array_equal(a, b)
        for a, b in zip(res[0][1:], r[1:]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("all_valid", [True, False])
def test_prefetch_across_windows_equals_plain(L, all_valid):
    """Back-to-back windows (a new RayWindow per window, the old one released, consecutive global steps,
    as Optimizer._run_config does): a prefetch built from the previous window is never used for the new
    one (it is matched by the window object, not its id(), which CPython may hand to the next window),
    so the pipelined (all-valid windows) / prefetched (windows with invalid rays) path equals the plain
    path bit for bit."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow

    def make(seed):
        scans, wc, rr = _window("forest" if all_valid else "quad", 2, seed=seed)
        if all_valid:
            return RayWindow(scans, wc, rr, n_lidar=128, n_sky=16, strategy="MASK")
        scale, shift = float(wc.scale_factor[0]), wc.shift.numpy()
        s1 = dict(scans[1])
        pose = s1["pose"].clone()
        pose[0, 3] = float(0.9995 * scale - shift[0])
        s1["pose"] = pose
        return RayWindow([scans[0], s1], wc, rr, n_lidar=128, strategy="RANDOM")

    res = []
    for fast in (False, True):
        st = S_.FieldState(S_.StepConfig(n_samples=64, occ_lr=1e-3), device="cuda:0", table_init=0.5)
        eng = None
        outs, g = [], 31
        for seed in (8, 9, 10, 11):
            win = make(seed)
            assert win.all_valid == all_valid
            if eng is None:
                eng = S_.StepEngine(st, win.n_slots, seed=5)
                eng.pipeline = eng.prefetch = fast
            for _ in range(3):
                outs.append(host(eng.step_window(win, global_step=g)).copy())
                g += 1
            del win  # the next window may reuse its address
        torch.cuda.synchronize()
        res.append((outs, host(st.params).copy(), host(st.occ).copy()))
    for a, b in zip(res[0][0], res[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][2], res[1][2])


@pytest.mark.parametrize("zero", [None, (1, 4)])
def test_graph_replay_equals_eager(L, zero):
    """step_window as a replayed HIP graph (per-step key, decaying los_lambda, los_eps, Adam coefficients
    and the ExponentialLR factor read from device memory, set by one launch per step) gives bitwise the
    eager path's losses, parameters, moments, occupancy grid and samples, across OGM steps (their own
    graph), a skipped global step, a changed iteration index / learning-rate factor and a second window
    (the graphs are re-captured), against the eager path with and without its pipelined prefetch; also with
    the sharded optimiser's one-rank share (bench --shard-of)."""
    from loner_amd import step as S_
    from loner_amd.rays import RayWindow
    loss = S_.LossConfig.from_dict(dict(loss_selection="L1_LOS", decay_los_lambda=True, los_lambda=1000.0,
                                        los_lambda_decay_rate=1e-4, los_lambda_decay_steps=30))
    res = []
    for graph, pipe in ((False, True), (False, False), (True, True)):
        st = S_.FieldState(S_.StepConfig(n_samples=64, occ_lr=1e-3, loss=loss), device="cuda:0", table_init=0.5)
        eng = None
        outs = []
        for seed, steps in ((8, (8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 19, 20, 21, 22, 23)), (9, (24, 25, 30, 31, 32))):
            scans, wc, rr = _window("forest", 2, seed=seed)
            win = RayWindow(scans, wc, rr, n_lidar=128, n_sky=16, strategy="MASK")
            if eng is None:
                eng = S_.StepEngine(st, win.n_slots, seed=4, zero=zero)
                eng.use_graph, eng.pipeline = graph, pipe
            st.reset_optimizer()
            for it, g in enumerate(steps):
                eng.lr_factor = 0.97 ** it
                outs.append(host(eng.step_window(win, global_step=g, iteration_idx=it)).copy())
            if graph:  # at least the OGM and the plain step of this window (times parities and prefetch states)
                assert len(eng._graphs) >= 2
        torch.cuda.synchronize()
        res.append((outs, host(st.params).copy(), host(st.m).copy(), host(st.v).copy(), host(st.occ).copy(),
                    host(eng.z).copy(), st.adam_step))
    for r in res[1:]:
        for a, b in zip(res[0][0], r[0]):
            np.testing.assert_array_equal(a, b)
        for a, b in zip(res[0][1:], r[1:]):
            np.testing.assert_array_equal(a, b)


# Every accumulate version the fused Adam epilogue runs in (the switches are read at every launch): the
# whole-bucket kernel (the default at this size), the unit work list with its cut buckets finished by the
# last piece or by k_bwd_finalize_units, and the record-balanced split with k_bwd_finalize or in-kernel
# finishing.  A bucket finished twice would apply Adam twice: bitwise equality with the separate Adam
# pins each of them.
_FUSED_PATHS = {
    "buckets": {},
    "units_finish": {"LONER_ACCUM_UNITS": "1", "LONER_UNITS_FINISH": "1"},
    "units_finalize": {"LONER_ACCUM_UNITS": "1", "LONER_UNITS_FINISH": "0"},
    "balanced_finalize": {"LONER_ACCUM_UNITS": "0", "LONER_ACCUM_BUCKETS_MAX_N": "0", "LONER_ACCUM_FINISH": "0"},
    "balanced_finish": {"LONER_ACCUM_UNITS": "0", "LONER_ACCUM_BUCKETS_MAX_N": "0", "LONER_ACCUM_FINISH": "1"},
}


def _fused_adam_run(fused, graph):
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    st = S_.FieldState(S_.StepConfig(n_samples=64, occ_lr=1e-3), device="cuda:0", table_init=0.5)
    scans, wc, rr = _window("forest", 2, seed=8)
    win = RayWindow(scans, wc, rr, n_lidar=128, n_sky=16, strategy="MASK")
    eng = S_.StepEngine(st, win.n_slots, seed=4)
    eng.fused_adam, eng.use_graph = fused, graph
    outs = []
    for it, g in enumerate((8, 9, 10, 11, 12, 13)):
        eng.lr_factor = 0.97 ** it
        outs.append(host(eng.step_window(win, global_step=g, iteration_idx=it)).copy())
    st.reset_optimizer()
    for it, g in enumerate((14, 15)):
        outs.append(host(eng.step_window(win, global_step=g, iteration_idx=it)).copy())
    # an empty batch: zero gradient everywhere, Adam still steps every parameter
    w2 = syn.make_window("quad", 1, seed=2)
    rays, dgt = syn.build_batch(w2, "quad", 64, 0, "RANDOM", seed=4)
    rays, dgt = rays.cuda(), dgt.cuda()
    eng.step(rays[:0], dgt[:0], global_step=16, scale=121.426537, far_ref=float(rays[0, 12]), n_rays_global=64)
    torch.cuda.synchronize()
    # a fused step never stores the table gradient, and says so (FieldState.table_gradient)
    assert st.grad_table_current is (not fused)
    if fused:
        with pytest.raises(RuntimeError, match="fused"):
            st.table_gradient()
    return (outs, host(st.params).copy(), host(st.m).copy(), host(st.v).copy(),
            host(st.shadow).view(np.uint16).copy(), host(st.occ).copy(), st.adam_step)


@pytest.mark.parametrize("path", sorted(_FUSED_PATHS))
def test_fused_adam_equals_separate(L, path, monkeypatch):
    """The table's Adam fused into the hash-grid backward (lnr_hashgrid_bwd_rays_jac_adam: each entry's
    gradient updates its parameter where the accumulation finishes it; the MLP's Adam separate) gives
    bitwise the separate lnr_adam_step's parameters, moments, fp16 shadow, losses and occupancy grid:
    eager and graph-replayed steps, OGM steps, a changed learning-rate factor, a new optimiser, and an
    empty batch (Adam with a zero gradient), in every accumulate version the epilogue runs in
    (``_FUSED_PATHS``; the batch of 288 rays x 64 samples has cut buckets in the split versions)."""
    ref = _fused_adam_run(False, False)
    for k, v in _FUSED_PATHS[path].items():
        monkeypatch.setenv(k, v)
    res = [_fused_adam_run(True, False)]
    if path == "buckets":
        res.append(_fused_adam_run(True, True))
    for r in res:
        for a, b in zip(ref[0], r[0]):
            np.testing.assert_array_equal(a, b)
        for a, b in zip(ref[1:], r[1:]):
            np.testing.assert_array_equal(a, b)
