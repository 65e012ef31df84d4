"""The live hash-grid backward (LNR_BWD_LIVE) on a trained field (GPU only).

A sample whose dL/dsigma is exactly 0 (alpha = 1 - exp(-delta relu(sigma + n)) with sigma + n <= 0,
/root/reference/src/models/rendering_tcnn.py:252,260) adds exactly 0 to every gradient.  On a field trained
through the north-star driver's windowed schedule (examples/fdt_optimize_implicit_map.py:576-616: shuffled
keyframe windows, a new Adam per window, src/mapping/optimizer.py:255-265, the OGM on) most samples are such.
The live backward skips them: its records, and the MLP backward's dead tile pairs.  These tests pin that the
step's table gradient, MLP gradient, Adam state, shadow and occupancy grid are BITWISE those of the full
backward, over steps that include an OGM update, with the table's Adam separate and fused."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_KF, PER_KF, S = 4, 512, 512  # 2048 rays x 512 samples: 2048 histogram rows, the level-looped scatter


@pytest.fixture(scope="module")
def trained():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    cfg = S_.StepConfig(n_samples=S)
    state = S_.FieldState(cfg, device=dev)
    pool = syn.make_window("quad", 12, seed=2000)
    rng = np.random.default_rng(3)
    R = N_KF * PER_KF
    eng = S_.StepEngine(state, R, seed=5)
    eng.live_bwd, eng._live = False, False
    g = 1
    for _ in range(8):  # the driver's shuffled windows, 32 iterations each
        idx = rng.choice(len(pool), N_KF, replace=False)
        win = RayWindow([pool[i] for i in idx], syn.world_cube("quad"), syn.SENSORS["quad"]["ray_range"],
                        n_lidar=PER_KF, device=dev)
        state.reset_optimizer()
        for it in range(32):
            eng.step_window(win, global_step=g, iteration_idx=it)
            g += 1
        eng.release()
    window = RayWindow(syn.make_window("quad", N_KF, seed=1000), syn.world_cube("quad"),
                       syn.SENSORS["quad"]["ray_range"], n_lidar=PER_KF, device=dev)
    torch.cuda.synchronize()
    g = (g // 10 + 1) * 10 - 1  # the second of the three compared steps updates the OGM
    return cfg, state.state_dict(), window, g


def _records(L, eng):
    """Records the last backward placed (the segment starts' last entry)."""
    st = eng.state
    nb = sum((int(st.desc.size[l]) + 4095) // 4096 for l in range(st.desc.n_levels))
    p = L.lib().lnr_hashgrid_bwd_seg_start(L.ctypes.byref(st.desc), eng.N, L.ptr(eng.bwd_ws))
    off = p - eng.bwd_ws.data_ptr()
    return int(eng.bwd_ws[off:off + 8 * (nb + 1)].view(torch.int64)[nb].item())


@pytest.mark.parametrize("fused", [False, True])
def test_live_backward_bitwise_on_trained_field(trained, fused):
    """Full backward without early ray termination (the reference's arithmetic) against the live backward, early ray
    termination (LONER_ERT, csrc/field.hip kErtTMin: the rays whose transmittance fell below 1e-100 skip the encode
    and sigma of their later samples) and both, eager and graph-replayed: bitwise equal."""
    from loner_amd import _lib as L
    from loner_amd import step as S_
    cfg, sd, window, g = trained
    out = {}
    for live, ert, graph in ((False, False, False), (True, False, False), (False, True, False), (True, True, False),
                             (True, True, True)):
        st = S_.FieldState(cfg, device="cuda")
        st.load_state_dict(sd)
        st.reset_optimizer()
        eng = S_.StepEngine(st, window.n_slots, seed=9)
        eng.live_bwd, eng._live = live, live
        eng.ert = ert
        eng.fused_adam = fused
        eng.pipeline, eng.use_graph = False, graph
        recs, zero, alive = [], [], []
        for k in range(3):
            eng.step_window(window, global_step=g + k, iteration_idx=k)
            torch.cuda.synchronize()
            recs.append(_records(L, eng))
            zero.append(float((eng.d_sigma() == 0).float().mean()))
            alive.append(eng.ert_alive_last())
        eng.finish()
        torch.cuda.synchronize()
        o = {k: getattr(st, k).clone() for k in ("params", "m", "v", "shadow", "occ")}
        o["grad_mlp"] = st.grad_mlp.clone()
        o["loss"] = eng.loss_out.clone()
        o["depth"] = eng.depth[:window.n_slots].clone()
        if not fused and not graph:
            o["grad_table"] = st.table_gradient().clone()
        out[(live, ert, graph)] = (o, recs, zero, alive)
    full, rec_full, zero_full, _ = out[(False, False, False)]
    assert min(zero_full) > 0.5, f"the pre-trained field should leave most samples dead: {zero_full}"
    for key, (o, recs, zero, alive) in out.items():
        assert zero == zero_full, key
        for k in o:
            assert torch.equal(full[k], o[k]), f"{k} differs between the full step and {key} (live, ert, graph)"
        if key[0]:  # the live backward placed far fewer records (its histogram counts live samples only)
            for rf, rl in zip(rec_full, recs):
                assert rl < 0.6 * rf, (key, rec_full, recs)
        if key[1]:  # early ray termination stopped rays before their last phase
            assert min(alive) < 1.0, (key, alive)


def test_live_probe_switches_modes(trained):
    """LONER_LIVE_BWD=auto: the probe turns the live backward on for the trained field and off again for a
    freshly initialised one (all samples live after its first steps)."""
    from loner_amd import step as S_
    cfg, sd, window, g = trained
    st = S_.FieldState(cfg, device="cuda")
    st.load_state_dict(sd)
    eng = S_.StepEngine(st, window.n_slots, seed=9)
    eng.live_bwd, eng._live = "auto", False
    for k in range(4):
        eng.step_window(window, global_step=g + k, iteration_idx=k)
        torch.cuda.synchronize()
    assert eng._live
    fresh = S_.FieldState(cfg, device="cuda")
    eng2 = S_.StepEngine(fresh, window.n_slots, seed=9)
    eng2.live_bwd, eng2._live, eng2.live_probe_every = "auto", True, 1
    for k in range(40):
        eng2.step_window(window, global_step=1 + k, iteration_idx=k)
        torch.cuda.synchronize()
    assert not eng2._live


def test_ert_auto_plans_from_termination_counts(trained, monkeypatch):
    """LONER_ERT=auto: the compositing's termination counts (lnr_loss_params.dev_term_hist) reach the planner
    without a host sync; on the trained field it picks phases, every ray is counted once per step, and the steps
    stay bitwise those without termination; on a fresh field (no ray terminates) it picks none.  (This batch,
    2048 rays, is too small for the fitted fixed costs to let phases pay: the test lowers them.)"""
    from loner_amd import step as S_
    monkeypatch.setattr(S_, "ERT_FIXED_US", 2.0)
    monkeypatch.setattr(S_, "ERT_PHASE_US", 2.0)
    cfg, sd, window, g = trained
    outs = []
    for mode in (False, "auto"):
        st = S_.FieldState(cfg, device="cuda")
        st.load_state_dict(sd)
        st.reset_optimizer()
        eng = S_.StepEngine(st, window.n_slots, seed=9)
        eng.live_bwd, eng._live = True, True
        eng.ert = mode
        eng.pipeline, eng.use_graph = False, False
        plans = []
        for k in range(6):
            eng.step_window(window, global_step=g + k, iteration_idx=k)
            torch.cuda.synchronize()
            plans.append(eng.ert_bounds())
        eng.finish()
        torch.cuda.synchronize()
        outs.append({k: getattr(st, k).clone() for k in ("params", "m", "v", "shadow", "occ")})
        if mode == "auto":
            assert int(eng.term_hist.sum()) == 6 * window.n_slots
            assert plans[0] is None and plans[-1] is not None, plans  # off until the first counts arrive
            alive = S_.ert_alive(eng.term_hist.long().sum(0).cpu().numpy(), S)
            assert alive[-1] < 0.9, alive
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
    fresh = S_.FieldState(cfg, device="cuda")
    eng2 = S_.StepEngine(fresh, window.n_slots, seed=9)
    eng2.ert = "auto"
    for k in range(4):
        eng2.step_window(window, global_step=1 + k, iteration_idx=k)
        torch.cuda.synchronize()
    assert eng2.ert_bounds() is None


def test_ert_plan_change_waits_for_window(trained, monkeypatch):
    """LONER_ERT=auto under HIP-graph replay: the first plan is taken at once, a later one waits for the window's
    end (release()), where the graphs are captured anew anyway, instead of an eager step and a capture mid-window."""
    from loner_amd import step as S_
    cfg, sd, window, g = trained
    plans = [[0, S // 2, S], [0, S // 4, S // 2, S]]
    pick = [plans[0]]
    monkeypatch.setattr(S_, "ert_plan", lambda *a, **k: list(pick[0]))
    st = S_.FieldState(cfg, device="cuda")
    st.load_state_dict(sd)
    st.reset_optimizer()
    eng = S_.StepEngine(st, window.n_slots, seed=9)
    eng.ert, eng.use_graph, eng.live_probe_every = "auto", True, 2
    for k in range(3):
        eng.step_window(window, global_step=g + k, iteration_idx=k)
        torch.cuda.synchronize()
    assert eng.ert_bounds() == plans[0]
    pick[0] = plans[1]
    for k in range(3, 8):
        eng.step_window(window, global_step=g + k, iteration_idx=k)
        torch.cuda.synchronize()
    assert eng.ert_bounds() == plans[0] and eng._ert_next[0] == plans[1]
    eng.finish()
    eng.release()
    assert eng.ert_bounds() == plans[1]


@pytest.mark.parametrize("graph", [False, True])
def test_split_backward_bitwise(trained, graph):
    """The live backward's preparation (histogram, scans, lists) on a side stream beside the MLP backward
    (StepEngine.split_bwd: lnr_field_train's FORWARD_ONLY / BACKWARD_ONLY halves, the backward's PREPARE_ONLY /
    PREPARED halves), eager and as two branches of the captured graph: bitwise the one-stream step, over three
    steps with an OGM update and the table's Adam fused."""
    from loner_amd import step as S_
    cfg, sd, window, g = trained
    outs = []
    for split in (False, True):
        st = S_.FieldState(cfg, device="cuda")
        st.load_state_dict(sd)
        st.reset_optimizer()
        eng = S_.StepEngine(st, window.n_slots, seed=9)
        eng.live_bwd, eng._live = True, True
        eng.ert, eng.fused_adam, eng.split_bwd = True, True, split
        eng.pipeline, eng.use_graph = False, graph
        for k in range(3):
            eng.step_window(window, global_step=g + k, iteration_idx=k)
        eng.finish()
        torch.cuda.synchronize()
        o = {k: getattr(st, k).clone() for k in ("params", "m", "v", "shadow", "occ")}
        o["loss"] = eng.loss_out.clone()
        outs.append(o)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
