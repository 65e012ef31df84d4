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


def test_metric_files_in_reference_format(tmp_path):
    """The files fdt_optimize_implicit_map.py:548-562,645-677 writes: both CSVs created with their
    header before the loop, one row per repetition, and a YAML per (kind, global step) holding the
    0-d tensors' format (the float32 value, in Python's repr), without a trailing newline."""
    import csv

    import torch

    from loner_amd.metrics import L1MetricsLog
    cfg = D.DriverSettings(repetitions_max=2, num_iterations=4)
    opt = _FakeOpt()
    D.configure_optimizer(opt, cfg)
    rng = np.random.RandomState(cfg.seed)
    _, train, _ = D.split_indices(40, cfg, rng)
    log = L1MetricsLog(tmp_path)
    for kind in ("test", "eval"):
        assert (tmp_path / "metrics" / f"l1_{kind}.csv").read_text() == "global_step,min,max,mean,rmse\n"
    evals = iter([[torch.tensor([1.5, 2.5])], [torch.tensor([0.25]), torch.tensor([0.75])]])
    hist = D.run_lidar_phase(opt, [f"kf{i}" for i in train], lambda: torch.tensor([1.0, 2.0, 4.0]),
                             lambda: next(evals), cfg, rng, metrics=log)
    assert [h["global_step"] for h in hist] == [12, 24]
    t = torch.tensor([1.0, 2.0, 4.0])
    rmse = torch.sqrt(torch.mean(t ** 2))
    assert (tmp_path / "metrics_test" / "l1_12.yaml").read_text() == \
        f"min: {t.min()}\nmax: {t.max()}\nmean: {t.mean()}\nrmse: {rmse}"
    assert (tmp_path / "metrics_test" / "l1_12.yaml").read_text().startswith("min: 1.0\nmax: 4.0\nmean: 2.3333332538604736")
    rows = list(csv.reader(open(tmp_path / "metrics" / "l1_test.csv")))
    assert rows[0] == ["global_step", "min", "max", "mean", "rmse"]
    assert [r[0] for r in rows[1:]] == ["12", "24"]
    assert rows[1][1:4] == ["1.0", "4.0", str(np.float32(7.0 / 3.0))]
    ev = list(csv.reader(open(tmp_path / "metrics" / "l1_eval.csv")))
    assert ev[2][1:4] == ["0.25", "0.75", "0.5"]  # the per-scan tensors joined (torch.hstack)
    assert hist[1]["l1_eval"]["mean"] == 0.5


def _rand_transforms(rng, n):
    from scipy.spatial.transform import Rotation
    T = np.tile(np.eye(4), (n, 1, 1))
    T[:, :3, :3] = Rotation.from_rotvec(rng.normal(0, 0.4, (n, 3))).as_matrix()
    T[:, :3, 3] = np.cumsum(rng.normal(0, 1.0, (n, 3)), axis=0)
    return T


def test_pose_interpolator():
    """fdt_optimize_implicit_map.py:370-425,768-783: relative to the first pose (not for submaps), exact
    at the ground-truth stamps, linear translation / slerp rotation between them, the scan-period rule
    for which scans and images are kept, [start:end:skip] of the images."""
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(3)
    ts = 100.0 + np.cumsum(rng.uniform(0.05, 0.15, 30))
    T = _rand_transforms(rng, 30)
    pi = D.PoseInterpolator(ts, T)
    rel = np.linalg.inv(T[0]) @ T
    P = D.pose6_to_matrix(pi.at(ts - ts[0]))
    np.testing.assert_allclose(P, rel, atol=2e-6)
    assert P.dtype == np.float32
    np.testing.assert_allclose(D.pose6_to_matrix(D.PoseInterpolator(ts, T, submap=True).at(ts - ts[0])), T, atol=2e-5)
    mid = 0.5 * (ts[4] + ts[5]) - ts[0]
    p = pi.at([mid])[0]
    np.testing.assert_allclose(p[:3], 0.5 * (rel[4, :3, 3] + rel[5, :3, 3]), atol=1e-9)
    r4, r5 = Rotation.from_matrix(rel[4, :3, :3]), Rotation.from_matrix(rel[5, :3, :3])
    half = r4 * Rotation.from_rotvec(0.5 * (r4.inv() * r5).as_rotvec())
    np.testing.assert_allclose(Rotation.from_rotvec(p[3:]).as_matrix(), half.as_matrix(), atol=1e-9)
    lidar_ts = np.arange(ts[0] - 0.3, ts[-1] + 0.3, 0.1)
    out = pi.lidar(lidar_ts)
    assert out["scan_time"] == np.round((lidar_ts[-1] - lidar_ts[0]) / len(lidar_ts), 2)
    st = out["scan_time"]
    keep = lidar_ts[(lidar_ts - st >= ts[0]) & (lidar_ts <= ts[-1])]
    np.testing.assert_allclose(out["ts"], keep - ts[0])
    np.testing.assert_allclose(out["poses_motion_comp"], pi.at(keep - ts[0] - st))
    cam_ts = np.arange(ts[0] - 0.2, ts[-1] + 0.2, 0.07)
    cts, cposes = pi.camera(cam_ts, st, start=1, end=None, skip=2)
    inside = cam_ts[(cam_ts >= ts[0]) & (cam_ts <= ts[-1] - st)] - ts[0]
    np.testing.assert_allclose(cts, inside[1::2])
    np.testing.assert_allclose(cposes, pi.at(inside)[1::2])


def test_camera_phase():
    """:736-757 schedule edits; :834-887 windows of 6 closed at the order's last image, one
    iterate_optimizer_camera per window, `reiterate_camera_<step>.tar` at the end; off by default."""
    cfg = D.CameraPhaseSettings(iterate=True, repetitions=2, num_iterations=3)
    opt = _FakeOpt()
    opt._optimization_settings = type("S", (), {})()
    D.configure_optimizer_camera(opt, cfg)
    s = opt._optimization_settings
    assert (s.freeze_poses, s.freeze_sigma_mlp, s.freeze_rgb_mlp, s.lidar_only, s.num_iterations) == \
        (True, True, False, False, 3)
    assert opt._use_gt_poses and opt._settings["rays_selection"]["strategy"] == "FIXED"
    it = opt._keyframe_schedule[0]["iteration_schedule"][0]
    assert opt._keyframe_schedule[0]["num_keyframes"] == -1 and it["freeze_sigma_mlp"] and not it["freeze_rgb_mlp"]
    rng = np.random.RandomState(8)
    wins = D.camera_windows(15, cfg, np.random.RandomState(8))
    assert [len(w) for w in wins] == [6, 6, 3] and sorted(sum(wins, [])) == list(range(15))
    calls, saved = [], []

    def cam(frames):
        calls.append(frames)
        opt._global_step += 3
        return 0.5

    opt.iterate_optimizer_camera = cam
    losses = D.run_camera_phase(opt, lambda w: list(w), 15, cfg, rng, save=lambda n, st: saved.append(n))
    assert [len(x) for x in losses] == [3, 3] and len(calls) == 6
    assert saved == [f"reiterate_camera_{opt._global_step}.tar"]
    assert D.run_camera_phase(opt, list, 15, D.CameraPhaseSettings()) == []  # ITERATE_CAMERA = False
