"""loner_amd.optimizer.Optimizer: the reference's Optimizer.iterate_optimizer surface on the fused
path (GPU only): schedule selection, a new Adam per iteration config, global-step bookkeeping and the
OGM cadence, RANDOM / MASK / FIXED ray selection; equivalence with StepEngine driven by hand."""
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


def _settings(strategy="RANDOM", n_it=4, sky=0, schedule=None):
    return dict(
        num_samples=dict(lidar=64, sky=sky), rays_selection=dict(strategy=strategy),
        samples_selection=dict(strategy="OGM"), skip_pose_refinement=True, freeze_poses=False,
        keyframe_schedule=schedule or [dict(num_keyframes=-1, iteration_schedule=[dict(
            num_iterations=n_it, freeze_poses=True, freeze_sigma_mlp=False, freeze_rgb_mlp=True)])],
        model_config=dict(model=dict(ray_range=[1.0, 75.0], render=dict(N_samples_train=128, perturb=1.0,
                                                                         raw_noise_std=1.0),
                                     occ_model=dict(voxel_size=100, lr=1e-4, N_iters_acc=10)),
                          train=dict(lrate_sigma_mlp=0.01, lrate_gamma=1.0)))


def _window(kind="quad", n=3):
    from loner_amd import synthetic as syn
    return syn.make_window(kind, n, seed=4), syn.world_cube(kind)


def test_iterate_optimizer_matches_step_engine(L):
    from loner_amd import step as S_
    from loner_amd.optimizer import Optimizer
    from loner_amd.rays import RayWindow
    scans, cube = _window()
    opt = Optimizer(_settings(n_it=5), None, cube, "cuda:0", seed=2)
    loss = opt.iterate_optimizer(scans)
    assert np.isfinite(loss) and opt._global_step == 5 and opt._keyframe_count == 1
    # the same five steps by hand
    st = S_.FieldState(opt.cfg, device="cuda:0", seed=2)
    win = RayWindow(scans, cube, (1.0, 75.0), n_lidar=64, device="cuda:0")
    eng = S_.StepEngine(st, win.n_slots, seed=2)
    for i in range(5):
        out = eng.step_window(win, global_step=i, iteration_idx=i)
    # every step is bitwise reproducible (int64 fixed-point table gradient and OGM splat, fixed-order
    # MLP reductions), so the two routes give the same bits
    assert float(out[0].item()) == loss
    assert torch.equal(st.params, opt.state.params) and torch.equal(st.occ, opt.state.occ)
    # second window: global step continues, a new Adam (moments restart)
    opt.iterate_optimizer(scans)
    assert opt._global_step == 10 and opt.state.adam_step == 5


def test_schedule_selection_and_skips(L):
    from loner_amd.optimizer import Optimizer
    scans, cube = _window()
    sched = [dict(num_keyframes=1, iteration_schedule=[dict(num_iterations=3, freeze_poses=True,
                                                            freeze_sigma_mlp=False, freeze_rgb_mlp=True)]),
             dict(num_keyframes=-1, iteration_schedule=[
                 dict(num_iterations=7, freeze_poses=False, latest_kf_only=True, freeze_sigma_mlp=True,
                      freeze_rgb_mlp=True),
                 dict(num_iterations=2, freeze_poses=True, freeze_sigma_mlp=False, freeze_rgb_mlp=True)])]
    opt = Optimizer(_settings(schedule=sched), None, cube, "cuda:0")
    opt.iterate_optimizer(scans)           # first keyframe: 3 iterations
    assert opt._global_step == 3
    opt.iterate_optimizer(scans)           # then: tracking config skipped (skip_pose_refinement), 2 mapping its
    assert opt._global_step == 5
    opt._settings["skip_pose_refinement"] = False
    opt.iterate_optimizer(scans)           # pose tracking (7, map frozen) then mapping (2): tests/test_gpu_pose.py
    assert opt._global_step == 14


def test_joint_pose_config_fixed_poses_opt_in(L):
    """The reference's default mapper schedule optimises poses and map jointly (cfg/defaults.yaml:93-97,
    optimizer.py:258-262): the fused Optimizer does so (tests/test_gpu_pose.py), and moves the poses.
    fixed_poses=True opts out (a warning, then the map optimised exactly as with freeze_poses: True);
    use_gt_poses freezes them as the reference does."""
    import warnings
    from loner_amd.optimizer import Optimizer
    scans, cube = _window()
    joint = [dict(num_keyframes=-1, iteration_schedule=[dict(num_iterations=3, freeze_poses=False,
                                                             freeze_sigma_mlp=False, freeze_rgb_mlp=True)])]
    p0 = [s["pose"].clone() for s in scans]
    loss_joint = Optimizer(_settings(schedule=joint), None, cube, "cuda:0", seed=2).iterate_optimizer(scans)
    assert np.isfinite(loss_joint) and all(not torch.equal(s["pose"], p) for s, p in zip(scans, p0))
    scans, cube = _window()
    with pytest.warns(UserWarning, match="fixed_poses=True"):
        loss_fixed = Optimizer(_settings(schedule=joint), None, cube, "cuda:0", seed=2,
                               fixed_poses=True).iterate_optimizer(scans)
    frozen = [dict(num_keyframes=-1, iteration_schedule=[dict(num_iterations=3, freeze_poses=True,
                                                              freeze_sigma_mlp=False, freeze_rgb_mlp=True)])]
    loss_frozen = Optimizer(_settings(schedule=frozen), None, cube, "cuda:0", seed=2).iterate_optimizer(scans)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        loss_gt = Optimizer(_settings(schedule=joint), None, cube, "cuda:0", seed=2,
                            use_gt_poses=True).iterate_optimizer(scans)
    assert loss_fixed == loss_frozen == loss_gt
    assert all(torch.equal(s["pose"], p) for s, p in zip(scans, p0))


@pytest.mark.parametrize("strategy,sky", [("MASK", 8), ("FIXED", 0), ("FIXED", 8)])
def test_strategies_run(L, strategy, sky):
    from loner_amd.optimizer import Optimizer
    scans, cube = _window("forest", 2)
    opt = Optimizer(_settings(strategy, n_it=3, sky=sky), None, cube, "cuda:0")
    loss = opt.iterate_optimizer(scans)
    assert np.isfinite(loss)
    if strategy == "FIXED":  # num_iterations = floor(max scan length / n) (optimizer.py:288)
        assert opt._global_step == max(int(s["distances"].numel()) for s in scans) // 64
    else:
        assert opt._global_step == 3


def test_camera_phase_and_checkpoint(L, tmp_path):
    """iterate_optimizer_camera trains the colour head with the sigma head frozen; the checkpoint
    carries both branches under the reference's module paths and restores them."""
    from loner_amd import camera as C
    from loner_amd import checkpoint as ckp
    from loner_amd.optimizer import Optimizer
    scans, cube = _window("quad", 2)
    opt = Optimizer(_settings(n_it=3), None, cube, "cuda:0")
    opt.iterate_optimizer(scans)
    sigma_before = opt.state.params.clone()
    W, H = 32, 24
    dirs = C.pinhole_directions(W, H, np.array([[30.0, 0, 15.5], [0, 30.0, 11.5], [0, 0, 1]]))
    imgs = [np.full((W * H, 3), 0.3, np.float32)]
    pose = scans[0]["pose"].numpy()[:3]
    fr = C.CameraFrames(dirs, W, H, imgs, [pose], cube, (1.0, 75.0), n_rays_per_kf=128, device="cuda:0")
    l0 = opt.iterate_optimizer_camera(fr)
    assert np.isfinite(l0) and opt.color.adam_step == fr.n_iter
    assert torch.equal(opt.state.params, sigma_before)  # the sigma head is frozen in the camera phase
    path = tmp_path / "ck.tar"
    ckp.save_checkpoint(str(path), opt.state, opt._global_step, other_params=ckp.color_params(opt.color))
    ck = torch.load(str(path), map_location="cpu", weights_only=True)
    assert set(ck["network_state_dict"]) >= {ckp.SIGMA_KEY, ckp.COLOR_GRID_KEY, ckp.COLOR_MLP_KEY, ckp.DIR_ENC_KEY}
    cs2 = C.ColorState(device="cuda:0", seed=99)
    ckp.load_color(ck, cs2)
    assert torch.equal(cs2.shadow, opt.color.shadow)  # fp16 round trip of the fp16 shadow


def _dp_window(strategy):
    """The DP test's window; FIXED runs floor(points / 64) iterations, so its scans are cut to 300
    points (4 iterations): long runs amplify summation-order differences through Adam."""
    scans, cube = _window("forest", 2)
    if strategy == "FIXED":
        scans = [dict(s, directions=s["directions"][:, :300].contiguous(), distances=s["distances"][:300].contiguous())
                 for s in scans]
    return scans, cube


def _dp_worker(rank, world, port, out, strategy="MASK"):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from loner_amd.optimizer import Optimizer
    scans, cube = _dp_window(strategy)

    def allreduce(t, async_op=False):
        return dist.all_reduce(t, async_op=async_op)

    opt = Optimizer(_settings(strategy, n_it=4, sky=8), None, cube, "cuda:0", seed=2, allreduce=allreduce, rank=rank,
                    world=world)
    opt.iterate_optimizer(scans)
    torch.cuda.synchronize()
    np.save(os.path.join(out, f"p{rank}.npy"), opt.state.params.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("strategy", ["MASK", "FIXED"])
def test_optimizer_data_parallel_gloo(L, tmp_path, strategy):
    """Optimizer(allreduce, rank, world): two gloo ranks on the window's two ray shards give the same
    map on both replicas, and the single-GPU map to a tolerance (summation order, OGM atomics).
    FIXED: each rank takes its slice of the iteration's FIXED batch (optimizer.py:269,380)."""
    import socket
    import torch.multiprocessing as mp
    from loner_amd.optimizer import Optimizer
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, str(tmp_path), strategy)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=150)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    assert np.array_equal(p0, p1)
    scans, cube = _dp_window(strategy)
    opt = Optimizer(_settings(strategy, n_it=4, sky=8), None, cube, "cuda:0", seed=2)
    opt.iterate_optimizer(scans)
    ref = opt.state.params.cpu().numpy()
    assert opt._global_step == 4
    assert np.linalg.norm(p0 - ref) / np.linalg.norm(ref) < 1e-4
