"""Early ray termination's planner (loner_amd.step.ert_plan, host only): the phases it picks from a termination
histogram (lnr_loss_params.dev_term_hist) under the cost model fitted to round 6's C2 / C4 traces."""
import numpy as np

from loner_amd import step as S_

S, N = 512, 8192 * 512


def _hist(alive_at):
    """A histogram (bins of 64 samples + never) whose alive shares after samples 64 k are ``alive_at[k]``."""
    a = np.asarray(list(alive_at) + [0.0], dtype=np.float64)
    return np.round((a[:-1] - a[1:]) * 10000).astype(np.int64)


def test_alive_from_histogram():
    h = [10, 0, 0, 0, 20, 30, 0, 0, 40]  # 40 % never terminate
    a = S_.ert_alive(h, S)
    assert np.allclose(a, [1.0, 0.9, 0.9, 0.9, 0.9, 0.7, 0.4, 0.4, 0.4])


def test_no_termination_means_no_phases():
    """The forest (C4) regime: almost no ray terminates, the phases would only add launches."""
    h = _hist([1.0] * 8 + [0.97])
    assert S_.ert_plan(h, S, N) is None
    # and a plan in use is dropped
    assert S_.ert_plan(h, S, N, current=[0, 256, 320, 384, 512]) is None


def test_trained_quad_regime_terminates():
    """The trained C2 field: rays alive 1.0 up to sample 192, then 0.9 / 0.73 / 0.34 / 0.12 / 0.05 at 256 .. 448."""
    h = _hist([1, 1, 1, 0.9, 0.73, 0.34, 0.12, 0.05, 0.02])
    b = S_.ert_plan(h, S, N)
    assert b is not None and b[0] == 0 and b[-1] == S and len(b) >= 3
    full = S_.ert_cost_us(None, S_.ert_alive(h, S), S, N)
    assert S_.ert_cost_us(b, S_.ert_alive(h, S), S, N) < 0.85 * full
    # the modelled encode + sigma of a traced trained C2 step (cuts 192, 320, 384; 461 us measured, gpurun_out r6o)
    assert abs(S_.ert_cost_us([0, 192, 320, 384, 512], S_.ert_alive(_hist([1, 1, .98, .654, .47, .214, .052, .001, 0]),
                                                                     S), S, N) - 461) < 15
    # hysteresis: a plan within the margin of the best stays
    assert S_.ert_plan(h, S, N, current=b) == b


def test_small_batches_and_short_rays():
    """Fixed costs dominate a small batch (a shard, C1): no phases; 64 samples per ray cannot be phased."""
    h = _hist([1, 1, 1, 0.9, 0.73, 0.34, 0.12, 0.05, 0.02])
    assert S_.ert_plan(h, S, 64 * 512) is None
    assert S_.ert_plan([5, 5], 64, 1 << 22) is None
