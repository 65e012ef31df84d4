"""The north-star driver's LiDAR-phase schedule (loner_amd/driver.py) against the reference script's
statements (examples/fdt_optimize_implicit_map.py).  The script itself imports rosbag and cannot be
imported here, so its numpy statements are restated below verbatim in meaning, on numpy's legacy
global generator exactly as the script uses it; the literal index lists pin numpy's stream."""
import math

import numpy as np
import pytest

from loner_amd import driver as D


def _reference_draws(n_scans, reps, start=0, end=120, n_eval=6, skip=1):
    """fdt_optimize_implicit_map.py:427-431, :496, :578 on np.random's global state."""
    np.random.seed(8)
    n = len(list(range(n_scans))[start:end])
    test = np.random.choice(n, n_eval, replace=False)
    train = [i for i in range(n) if i not in test]
    ev = np.random.choice(len(train), n_eval, replace=False)
    m = len(train[::skip])
    shuffles = [np.random.choice(m, m, replace=False) for _ in range(reps)]
    return test.tolist(), train, ev.tolist(), [s.tolist() for s in shuffles]


@pytest.mark.parametrize("n_scans", [120, 300, 40])
def test_split_and_shuffles_match_reference_stream(n_scans):
    cfg = D.DriverSettings()
    rng = np.random.RandomState(cfg.seed)
    test, train, ev = D.split_indices(n_scans, cfg, rng)
    wins = [D.repetition_windows(len(train), cfg, rng) for _ in range(3)]
    r_test, r_train, r_ev, r_sh = _reference_draws(n_scans, 3)
    assert test == r_test and train == r_train and ev == r_ev
    for w, sh in zip(wins, r_sh):
        assert [i for win in w for i in win] == sh
        assert all(len(x) == cfg.max_window_length for x in w[:-1]) and 0 < len(w[-1]) <= cfg.max_window_length


def test_reference_stream_literals():
    # np.random.seed(8) as the driver does, over its default END_STEP_LIDAR = 120 scans
    cfg = D.DriverSettings()
    rng = np.random.RandomState(8)
    test, train, ev = D.split_indices(500, cfg, rng)
    assert test == [101, 29, 17, 57, 87, 103]
    assert ev == [109, 16, 23, 59, 30, 53]
    assert len(train) == 114
    assert D.repetition_windows(len(train), cfg, rng)[0][:10] == [87, 15, 80, 107, 20, 72, 25, 24, 96, 37]


def test_windows_skip_and_no_shuffle():
    cfg = D.DriverSettings(shuffle=False, skip_step=3, max_window_length=4)
    w = D.repetition_windows(20, cfg, np.random.RandomState(0))
    assert w == [[0, 1, 2, 3], [4, 5, 6]]  # positions into keyframes[::3] (7 of them)


def _run_rule(means, reps_max=8, thr=1.05):
    rule = D.StopRule(D.DriverSettings(repetitions_max=reps_max, l1_threshold=thr))
    log = []
    step = 0
    for m in means:
        if rule.done:
            break
        step += 10
        log.append(rule.after_repetition(m, step))
    return log


def test_stop_rule_first_repetition_threshold():
    assert _run_rule([1.0, 2.0]) == [(["final.tar"], "threshold")]


def test_stop_rule_second_repetition_never_worse():
    # the first repetition does not record its mean (l1s_mean_prev stays inf): rep 2 cannot be "worse"
    log = _run_rule([2.0, 3.0, 4.0, 1.5])
    assert log == [(["final.tar"], None), (["final_20.tar"], None), ([], "worse_than_previous")]


def test_stop_rule_improving_until_max():
    log = _run_rule([3.0, 2.9, 2.8, 2.7], reps_max=4)
    assert log == [(["final.tar"], None), (["final_20.tar"], None), (["final_30.tar"], None),
                   (["final_40.tar", "final_40.tar"], "max_repetitions")]


def test_stop_rule_threshold_later():
    log = _run_rule([3.0, 2.0, 1.0, 0.5])
    assert log == [(["final.tar"], None), (["final_20.tar"], None), (["final_30.tar"], "threshold")]


def test_stop_rule_single_repetition():
    assert _run_rule([3.0], reps_max=1) == [(["final.tar"], "max_repetitions")]


class _FakeOpt:
    def __init__(self):
        self._global_step = 0
        self._optimization_settings = type("S", (), {})()
        self._keyframe_schedule = [dict(num_keyframes=1, iteration_schedule=[dict(num_iterations=5)])]
        self._settings = dict(rays_selection=dict(strategy="RANDOM"))
        self.windows = []

    def iterate_optimizer(self, window):
        self.windows.append(list(window))
        self._global_step += self._keyframe_schedule[0]["iteration_schedule"][0]["num_iterations"]
        return 1.0


def test_run_lidar_phase_schedule():
    cfg = D.DriverSettings(repetitions_max=3, num_iterations=4)
    opt = _FakeOpt()
    D.configure_optimizer(opt, cfg)
    sched = opt._keyframe_schedule[0]
    assert sched["num_keyframes"] == -1 and sched["iteration_schedule"][0]["freeze_rgb_mlp"] is True
    assert opt._settings["rays_selection"]["strategy"] == "MASK" and opt._rays_strategy == "MASK"
    rng = np.random.RandomState(cfg.seed)
    _, train, _ = D.split_indices(40, cfg, rng)
    kfs = [f"kf{i}" for i in train]  # 34 keyframes: windows of 16, 16, 2
    means = iter([5.0, 4.0, 4.5])
    saved = []
    hist = D.run_lidar_phase(opt, kfs, lambda: [1.0, 2.0], lambda: [next(means)], cfg, rng,
                             save=lambda name, step: saved.append((name, step)))
    assert [h["windows"] for h in hist] == [3, 3, 3]
    assert [len(w) for w in opt.windows] == [16, 16, 2] * 3
    assert sorted(opt.windows[0] + opt.windows[1] + opt.windows[2]) == sorted(kfs)
    assert [h["global_step"] for h in hist] == [12, 24, 36]
    assert saved == [("final.tar", 12), ("final_24.tar", 24), ("final_36.tar", 36)]
    assert hist[-1]["stop"] == "worse_than_previous"  # saved for reaching the maximum, then found worse
    assert hist[0]["l1_test"]["mean"] == 1.5 and math.isclose(hist[0]["l1_test"]["rmse"], math.sqrt(2.5))
