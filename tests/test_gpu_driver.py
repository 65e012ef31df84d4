"""The north-star driver's LiDAR phase (loner_amd/driver.py, examples/fdt_optimize_implicit_map.py
:427-727) end to end on the GPU path: scans split into test / train / eval, the driver's optimiser
edits, shuffled MASK windows through Optimizer.iterate_optimizer, compute_l1_depth on the held-out
and training scans after every repetition, and the reference-format checkpoints the stop rule
writes (reloaded bit-exactly).  Synthetic scans (no datasets here)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_lidar_phase_on_gpu(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from loner_amd import checkpoint as ckp
    from loner_amd import driver as D
    from loner_amd import evaluate as E
    from loner_amd import synthetic as syn
    from loner_amd.optimizer import Optimizer

    kind = "quad"
    cube, rr = syn.world_cube(kind), syn.SENSORS[kind]["ray_range"]
    scans = syn.make_window(kind, 14, seed=21)
    cfg = D.DriverSettings(n_eval=2, max_window_length=4, repetitions_max=2, num_iterations=3, l1_threshold=0.0)
    rng = np.random.RandomState(cfg.seed)
    test, train, ev = D.split_indices(len(scans), cfg, rng)
    assert len(test) == 2 and len(train) == 12 and not set(test) & set(train)
    settings = dict(num_samples=dict(lidar=64, sky=0), rays_selection=dict(strategy="RANDOM"),
                    samples_selection=dict(strategy="OGM"), skip_pose_refinement=True, freeze_poses=False,
                    keyframe_schedule=[dict(num_keyframes=1, iteration_schedule=[dict(
                        num_iterations=100, freeze_poses=False, freeze_sigma_mlp=False, freeze_rgb_mlp=True)])],
                    model_config=dict(model=dict(ray_range=list(rr), render=dict(N_samples_train=128, perturb=1.0,
                                                                                 raw_noise_std=1.0),
                                                 occ_model=dict(voxel_size=100, lr=1e-4, N_iters_acc=10)),
                                      train=dict(lrate_sigma_mlp=0.01, lrate_gamma=1.0)))
    opt = Optimizer(settings, None, cube, "cuda:0", seed=3)
    D.configure_optimizer(opt, cfg)
    assert opt._rays_strategy == "MASK"
    rend = E.DepthRenderer(opt.state, n_samples=256, chunk=4096)

    def sub(s):  # every 9th point keeps the evaluation short
        k = torch.arange(0, s["distances"].shape[0], 9)
        return dict(directions=s["directions"][:, k].contiguous(), distances=s["distances"][k].contiguous(),
                    pose=s["pose"])

    test_scans = [sub(scans[i]) for i in test]
    eval_scans = [sub(scans[train[i]]) for i in ev]

    def l1s(group):
        return [float(E.compute_l1_depth(rend, s, s["pose"], cube, rr, key=7).item()) for s in group]

    saved = {}

    def save(name, step):
        path = os.path.join(tmp_path, name)
        ckp.save_checkpoint(path, opt.state, step)
        saved[name] = path

    hist = D.run_lidar_phase(opt, [scans[i] for i in train], lambda: l1s(test_scans), lambda: l1s(eval_scans),
                             cfg, rng, save=save)
    # 12 keyframes in windows of 4: 3 windows x 3 iterations per repetition, 2 repetitions
    assert [h["windows"] for h in hist] == [3, 3]
    assert [h["global_step"] for h in hist] == [9, 18] and opt._global_step == 18
    assert all(np.isfinite(h["loss"]).all() for h in hist)
    for h in hist:
        for k in ("l1_test", "l1_eval"):
            assert np.isfinite(h[k]["mean"]) and h[k]["min"] <= h[k]["mean"] <= h[k]["max"]
    assert sorted(saved) == ["final.tar", "final_18.tar"]
    ck = torch.load(saved["final_18.tar"], map_location="cpu", weights_only=True)
    assert int(ck["global_step"]) == 18
    st2 = type(opt.state)(opt.cfg, device="cuda:0", seed=99)
    ckp.load_checkpoint(saved["final_18.tar"], st2, load_optimizer=False)
    # the reference format stores tcnn's fp16 params: the reloaded field's fp16 operand is the same bits
    assert torch.equal(st2.shadow, opt.state.shadow)
    assert torch.equal(st2.occ, opt.state.occ)
