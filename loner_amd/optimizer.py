"""``Optimizer``: the reference's mapping optimiser surface (src/mapping/optimizer.py:60-511) on the
fused path, for the sigma field.

    opt = Optimizer(settings, calibration, world_cube, device)   # settings = mapper.optimizer
    loss = opt.iterate_optimizer(keyframe_window)                # one window, its iteration schedule

The schedule logic follows the reference:
* the keyframe schedule picks the iteration schedule by the running keyframe count (:141-152);
* ``skip_pose_refinement`` drops the first iteration config when there are several (:218-219);
* a fresh Adam (``lrate_sigma_mlp``, ExponentialLR ``lrate_gamma`` stepped every iteration) per
  iteration config (:255-265);
* RANDOM / MASK / FIXED ray selection with sky rays (:279-424);
* the OGM update when ``global_step % N_iters_acc == 0``, checked before the increment (:466-469).

Rays are selected and built on the device from the window held in HBM (``RayWindow``). Each
iteration is ``StepEngine.step``: no host synchronisation until the window's final loss is read.

Poses (optimizer.py:235-262): an iteration config with ``freeze_poses: False`` optimises the pose
tensors [t, axis-angle] of the active window's un-anchored keyframes (a window of one keyframe anchors
it, :196-197) in an Adam at ``lrate_pose`` beside the map's, with the same ExponentialLR; the joint
config of the default mapper schedule (cfg/defaults.yaml:93-97) and pose tracking (both heads frozen,
:252-257: the map's Adam steps at lr 0) both run on the fused step (``loner_amd.pose``: the step writes
dL/d{ray} and dL/dpos, chained to the poses on the device).  The optimised poses are written back into
the keyframes (scan dicts: ``pose6`` and ``pose``; objects: their pose tensor).  ``fixed_poses=True``
keeps the poses fixed instead (a map-only run of such configs, with a warning); ``use_gt_poses=True``
(the north-star driver, fdt_optimize_implicit_map.py:355) freezes them as the reference does.

The colour head trains in the camera phase: ``iterate_optimizer_camera(frames)`` over a
``loner_amd.camera.CameraFrames`` window (``loner_amd.camera``).

Keyframes are ``loner_amd`` scan dicts (``directions`` (3,P), ``distances`` (P,), optional
``sky_directions`` (3,Q), ``pose`` (4,4)), or objects with the reference's KeyFrame accessors
(``get_lidar_scan()`` with ``ray_directions``, ``distances`` and ``sky_rays``, and
``get_lidar_pose().get_transformation_matrix()``).
"""
import warnings
from dataclasses import dataclass

import torch

from . import _lib as L
from .rays import RayWindow
from .step import FieldState, LossConfig, StepConfig, StepEngine


def _g(obj, key, default=None):
    """settings[key] for dicts, getattr for Settings-like objects."""
    if obj is None:
        return default
    if isinstance(obj, dict):
        return obj.get(key, default)
    return getattr(obj, key, default)


@dataclass
class OptimizationSettings:
    """optimizer.py:41-58."""
    num_iterations: int = 1
    freeze_poses: bool = False
    latest_kf_only: bool = False
    freeze_sigma_mlp: bool = False
    freeze_rgb_mlp: bool = False

    @staticmethod
    def from_dict(d):
        return OptimizationSettings(d.get("num_iterations", 1), d.get("freeze_poses", False),
                                    d.get("latest_kf_only", False), d.get("freeze_sigma_mlp", False),
                                    d.get("freeze_rgb_mlp", False))


def _kf_time(kf):
    t = kf.get("time") if isinstance(kf, dict) else getattr(kf, "get_time", lambda: None)()
    return None if t is None else float(t)


def _is_anchored(kf):
    return bool(kf.get("anchored", False)) if isinstance(kf, dict) else bool(getattr(kf, "is_anchored", False))


def _set_anchored(kf):
    if isinstance(kf, dict):
        kf["anchored"] = True
    else:
        kf.is_anchored = True


def _pose6_of(kf, scan):
    """The keyframe's pose tensor [t, axis-angle] (Pose.get_pose_tensor), or transform_to_tensor of its matrix."""
    from .pose import matrix_to_pose6
    if isinstance(kf, dict):
        if kf.get("pose6") is not None:
            return torch.as_tensor(kf["pose6"], dtype=torch.float32).reshape(6).cpu()
        return matrix_to_pose6(scan["pose"])
    p = kf.get_lidar_pose()
    if hasattr(p, "get_pose_tensor") and p.get_pose_tensor() is not None:
        return p.get_pose_tensor().detach().float().reshape(6).cpu()
    return matrix_to_pose6(scan["pose"])


def _write_poses(keyframes, scans, pw):
    """The optimised poses back into their keyframes (the reference's pose tensors change in place):
    scan dicts get ``pose6`` and ``pose`` (4x4), objects with a pose tensor get it overwritten."""
    p6 = pw.p6.detach().cpu()
    M = pw.matrices()
    moved = pw.optimise.cpu().tolist()
    for k, (kf, sc) in enumerate(zip(keyframes, scans)):
        if not moved[k]:
            continue  # an anchored keyframe keeps its pose as it was
        if isinstance(kf, dict):
            kf["pose6"] = p6[k].clone()
            kf["pose"] = M[k].clone()
        else:
            p = kf.get_lidar_pose()
            if hasattr(p, "get_pose_tensor") and p.get_pose_tensor() is not None:
                with torch.no_grad():
                    p.get_pose_tensor().copy_(p6[k].to(p.get_pose_tensor().device))


def _scan_dict(kf):
    if isinstance(kf, dict):
        return kf
    scan = kf.get_lidar_scan()
    d = dict(directions=scan.ray_directions, distances=scan.distances,
             pose=kf.get_lidar_pose().get_transformation_matrix().detach())
    sky = getattr(scan, "sky_rays", None)
    if sky is not None and sky.numel() > 0:
        d["sky_directions"] = sky
    return d


class Optimizer:
    def __init__(self, settings, calibration=None, world_cube=None, device="cuda", use_gt_poses=False,
                 lidar_only=True, enable_sky_segmentation=True, seed=0, allreduce=None, rank=0, world=1,
                 fixed_poses=False):
        """``allreduce`` / ``rank`` / ``world``: data-parallel over ranks (one process per GPU):
        rank r optimises the contiguous slice ``shard_range(window slots, r, world)`` of every
        window's rays; the opaque count and the gradients are summed with ``allreduce(t,
        async_op=...)`` (e.g. ``torch.distributed.all_reduce``), so every rank holds the same map.
        ``fixed_poses``: run joint pose + map iteration configs as map-only ones with the poses held
        fixed (otherwise they raise NotImplementedError; see the module docstring)."""
        if world_cube is None:
            raise ValueError("Optimizer needs the world cube")
        self._settings = settings
        self._calibration = calibration
        self._device = torch.device(device)
        self._use_gt_poses = use_gt_poses
        self._lidar_only = lidar_only
        self._enable_sky_segmentation = enable_sky_segmentation
        self._world_cube = world_cube
        mc = _g(settings, "model_config")
        model = _g(mc, "model")
        render = _g(model, "render")
        occ = _g(model, "occ_model")
        train = _g(mc, "train")
        self._ray_range = tuple(float(x) for x in _g(model, "ray_range", _g(_g(mc, "data"), "ray_range", (1.0, 75.0))))
        self._samples_strategy = _g(_g(settings, "samples_selection"), "strategy", "OGM")
        if self._samples_strategy not in ("OGM", "UNIFORM"):
            raise RuntimeError(f"Can't find samples_selection strategy: {self._samples_strategy}")
        self._rays_strategy = _g(_g(settings, "rays_selection"), "strategy", "RANDOM")
        if self._rays_strategy not in ("RANDOM", "MASK", "FIXED"):
            raise RuntimeError(f"Can't find rays_selection strategy: {self._rays_strategy}")
        ns = _g(settings, "num_samples")
        self._num_lidar_samples = int(_g(ns, "lidar", 512))
        self._num_sky_samples = int(_g(ns, "sky", 0))
        loss = _g(mc, "loss")
        self.cfg = StepConfig(
            n_samples=int(_g(render, "N_samples_train", 512)), perturb=float(_g(render, "perturb", 1.0)),
            raw_noise_std=float(_g(render, "raw_noise_std", 1.0)), lr=float(_g(train, "lrate_sigma_mlp", 0.01)),
            occ_res=int(_g(occ, "voxel_size", 100)), occ_lr=float(_g(occ, "lr", 1e-4)),
            n_iters_acc=int(_g(occ, "N_iters_acc", 10)), sampler=self._samples_strategy,
            loss=LossConfig.from_dict(dict(loss)) if loss is not None else LossConfig())
        self._lr_gamma = float(_g(train, "lrate_gamma", 1.0))
        self._lr_pose = float(_g(train, "lrate_pose", 0.001))
        self.state = FieldState(self.cfg, device=self._device, seed=seed)
        self._seed = int(seed)
        self._allreduce, self._rank, self._world = allreduce, int(rank), int(world)
        if self._world > 1 and allreduce is None:
            raise ValueError("world > 1 needs an allreduce")
        self._engine = None
        self._keyframe_schedule = _g(settings, "keyframe_schedule") or [
            dict(num_keyframes=-1, iteration_schedule=[dict(num_iterations=1, freeze_poses=True,
                                                            freeze_sigma_mlp=False, freeze_rgb_mlp=True)])]
        self._optimization_settings = OptimizationSettings()
        self._keyframe_count = 0
        self._global_step = 0
        self._fixed_poses = bool(fixed_poses)
        self._warned_poses = False
        self._fixed_gen = torch.Generator(device="cpu").manual_seed(seed)

    # ------------------------------------------------------------------ schedule
    def _iteration_schedule(self):
        """optimizer.py:141-152."""
        cumulative = 0
        schedule = None
        for item in self._keyframe_schedule:
            kf_count = item["num_keyframes"]
            schedule = item["iteration_schedule"]
            cumulative += kf_count
            if cumulative >= self._keyframe_count + 1 or kf_count == -1:
                break
        return schedule

    def _engine_for(self, n_slots):
        """The engine for a window of n_slots rays and this rank's slot range [s0, s1) of it (all of
        them on one GPU).  The engine is reused while its capacity suffices; its ray_offset (the
        global index of its first ray, which keys the draws) follows the window."""
        from .shard import shard_range
        s0, s1 = shard_range(n_slots, self._rank, self._world)
        e = self._engine
        if e is None or e.n_rays < s1 - s0:
            e = StepEngine(self.state, s1 - s0, seed=self._seed, allreduce=self._allreduce, ray_offset=s0)
            self._engine = e
        e.ray_offset = s0
        return e, s1 - s0

    def iterate_optimizer(self, keyframe_window, optimizer_settings: OptimizationSettings = None) -> float:
        schedule = self._iteration_schedule()
        result = self._do_iterate_optimizer(keyframe_window, schedule, optimizer_settings)
        self._keyframe_count += 1
        return result

    def _do_iterate_optimizer(self, keyframe_window, iteration_schedule, optimizer_settings=None) -> float:
        if len(keyframe_window) == 1:
            _set_anchored(keyframe_window[0])  # optimizer.py:196-197 (persists on the keyframe)
        if len(iteration_schedule) > 1 and _g(self._settings, "skip_pose_refinement", False):
            iteration_schedule = iteration_schedule[1:]
        if optimizer_settings is not None:
            iteration_schedule = [None]
        loss = None
        for config in iteration_schedule:
            os_ = optimizer_settings if config is None else OptimizationSettings.from_dict(config)
            freeze_poses = os_.freeze_poses or bool(_g(self._settings, "freeze_poses", False)) or self._use_gt_poses
            if not freeze_poses and self._fixed_poses:
                if not self._warned_poses:
                    self._warned_poses = True
                    warnings.warn("fixed_poses=True: the config's poses stay fixed and only the map is optimised")
                freeze_poses = True
            # optimizer.py:252-253: poses free with both heads frozen is pose tracking (the map's Adam
            # steps at lr 0 here: the map does not move)
            tracking = (not freeze_poses) and os_.freeze_sigma_mlp and os_.freeze_rgb_mlp
            if os_.freeze_sigma_mlp and not tracking:
                continue  # nothing of the map or the poses to optimise in this config
            # the active window (optimizer.py:237-246): the most recent keyframe only, or all of them
            active = list(keyframe_window)
            if os_.latest_kf_only and len(active) > 1:
                active = [max(active, key=_kf_time)] if all(_kf_time(k) is not None for k in active) else active[-1:]
            self.state.reset_optimizer()  # a new torch.optim.Adam per iteration config (:255-265)
            loss = self._run_config(active, int(os_.num_iterations), optimise_poses=not freeze_poses,
                                    tracking=tracking)
        return float(loss[0].item()) if loss is not None else float("nan")

    def _run_config(self, keyframes, num_iterations, optimise_poses=False, tracking=False):
        scans = [_scan_dict(kf) for kf in keyframes]
        n_sky = self._num_sky_samples if self._enable_sky_segmentation else 0
        fixed = self._rays_strategy == "FIXED"
        window = RayWindow(scans, self._world_cube, self._ray_range, n_lidar=self._num_lidar_samples, n_sky=n_sky,
                           strategy="RANDOM" if fixed else self._rays_strategy, device=self._device)
        eng, n_local = self._engine_for(window.n_slots)
        out = None
        if fixed:
            given, num_iterations = self._fixed_schedule(scans, window)
        pw = None
        if optimise_poses:
            # joint pose + map (optimizer.py:258-262) or tracking (:255-257): the un-anchored keyframes' pose
            # tensors in an Adam at lrate_pose beside the map's, same ExponentialLR (loner_amd.pose)
            from .pose import PoseWindow
            p6 = [_pose6_of(kf, sc) for kf, sc in zip(keyframes, scans)]
            pw = PoseWindow(window, [not _is_anchored(kf) for kf in keyframes], self._lr_pose,
                            pose6=torch.stack(p6), allreduce=self._allreduce if self._world > 1 else None,
                            n_iter=num_iterations, lr_gamma=self._lr_gamma)
            eng.set_poses(pw)
            eng.map_frozen = bool(tracking)
        try:
            for it in range(num_iterations):
                eng.lr_factor = self._lr_gamma ** it  # ExponentialLR stepped after every iteration
                if fixed:
                    out = self._fixed_step(eng, window, given, it)
                else:
                    out = eng.step_window(window, global_step=self._global_step, iteration_idx=it,
                                          n_rays_global=window.n_slots, n_slots=n_local)
                self._global_step += 1
        finally:
            eng.lr_factor = 1.0
            if pw is not None:
                eng.set_poses(None)
                eng.map_frozen = False
        if pw is not None:
            _write_poses(keyframes, scans, pw)
        eng.release()  # the next window is a new object: this one's prefetched step and graphs are dropped
        return out

    # ------------------------------------------------------------------ camera phase
    def iterate_optimizer_camera(self, frames, color=None, n_samples=None) -> float:
        """Optimizer.iterate_optimizer_camera (optimizer.py:517-688) for one camera window
        (``loner_amd.camera.CameraFrames``): the sigma head frozen, a new Adam over the colour head
        at ``lrate_rgb`` with ExponentialLR ``lrate_gamma``, ``frames.n_iter`` iterations.  The colour
        head (``loner_amd.camera.ColorState``) is created on first use and kept in ``self.color``."""
        from .camera import CameraStepEngine, ColorState
        train = _g(_g(self._settings, "model_config"), "train")
        if color is not None:
            self.color = color
        elif getattr(self, "color", None) is None:
            self.color = ColorState(device=self._device, seed=self._seed + 1)
        S = int(n_samples or self.cfg.n_samples)
        n_max = max(frames.n_rays(it) for it in range(frames.n_iter)) if frames.n_iter else 0
        eng = getattr(self, "_camera_engine", None)
        if eng is None or eng.R < n_max or eng.S != S or eng.color is not self.color:
            eng = CameraStepEngine(self.state, self.color, n_rays=max(n_max, 1), n_samples=S,
                                   perturb=self.cfg.perturb, raw_noise_std=self.cfg.raw_noise_std,
                                   lr=float(_g(train, "lrate_rgb", 0.01)),
                                   gamma=float(_g(train, "lrate_gamma", 1.0)), seed=self._seed)
            self._camera_engine = eng
        self.color.reset_optimizer()  # torch.optim.Adam over the colour parameters (:576)
        rays = torch.empty(max(n_max, 1), 13, dtype=torch.float32, device=self._device)
        inten = torch.empty(max(n_max, 1), 3, dtype=torch.float32, device=self._device)
        loss = None
        for it in range(frames.n_iter):
            n = frames.build(it, rays, inten)
            loss = eng.step(rays[:n], inten[:n], global_step=self._global_step)
            self._global_step += 1
        self._keyframe_count += 1
        return float(loss.item()) if loss is not None else float("nan")

    # ------------------------------------------------------------------ FIXED ray selection
    def _fixed_schedule(self, scans, window):
        """optimizer.py:279-299: every keyframe's points in a random order, padded to the longest scan
        with a permutation of its first points; num_iterations = floor(max length / n)."""
        n = self._num_lidar_samples
        lengths = [int(s["distances"].numel()) for s in scans]
        max_len = max(lengths)
        n_iter = max_len // n
        full = torch.zeros(len(scans), max_len, dtype=torch.int64)
        for k, P in enumerate(lengths):
            idx = torch.arange(P)
            pad = max_len - P
            full[k] = torch.cat((idx[torch.randperm(P, generator=self._fixed_gen)],
                                 idx[torch.randperm(pad, generator=self._fixed_gen)]))
        return full, n_iter

    def _fixed_step(self, eng, window, full, it):
        """Iteration it: keyframe k's points full[k, max(n it - 1, 0) : min(n (it + 1) - 1, n_iter n)]
        (optimizer.py:302-317) plus its sky draws, as GIVEN indices into the window's slots."""
        n = self._num_lidar_samples
        n_iter = full.shape[1] // n
        lo, hi = max(n * it - 1, 0), min(n * (it + 1) - 1, n_iter * n)
        K = full.shape[0]
        given = torch.zeros(window.n_slots, dtype=torch.int32)
        keep = torch.zeros(window.n_slots, dtype=torch.bool)
        ray_off, n_sel = window.ray_off_host, window.n_sel_host
        for k in range(K):
            base = int(ray_off[k])
            m = hi - lo
            given[base:base + m] = full[k, lo:hi].to(torch.int32)
            keep[base:base + m] = True
            n_sky_k = int(ray_off[k + 1]) - base - int(n_sel[k])
            if n_sky_k > 0:
                q = int(window.sky_count_host[k])
                given[base + int(n_sel[k]):base + int(n_sel[k]) + n_sky_k] = torch.randint(
                    0, q, (n_sky_k,), generator=self._fixed_gen, dtype=torch.int64).to(torch.int32)
                keep[base + int(n_sel[k]):base + int(n_sel[k]) + n_sky_k] = True
        dev = self._device
        key = L.step_key(eng.seed, self._global_step)
        rays, depth, valid, _, far_ref = window.build(key, 0, window.n_slots, given=given.to(dev))
        sel = keep.to(dev) & valid.bool()
        rays, depth = rays[sel], depth[sel]
        n_glob = rays.shape[0]
        if self._world > 1:
            # data parallel: every rank builds the same FIXED batch (one generator, one seed), so its
            # size is known everywhere; all-reducing [n, n^2] checks that, and rank r steps the
            # contiguous slice shard_range(n, r, world) with its draws keyed by global ray index.
            # world * sum(n^2) == sum(n)^2 holds iff every rank's n is equal (Cauchy-Schwarz), and every
            # rank evaluates it on the same sums, so all ranks reach the same verdict (none is left
            # waiting in a later collective)
            from .shard import shard_range
            cnt = torch.tensor([float(n_glob), float(n_glob) ** 2], dtype=torch.float64, device=dev)
            self._allreduce(cnt)
            s1_, s2_ = (float(v) for v in cnt.cpu())
            if s2_ * self._world != s1_ * s1_:
                raise RuntimeError("FIXED ray selection diverged across ranks")
            s0, s1 = shard_range(n_glob, self._rank, self._world)
            rays, depth = rays[s0:s1], depth[s0:s1]
            eng.ray_offset = s0
        out = eng.step(rays.contiguous(), depth.contiguous(), self._global_step, it, scale=window.scale,
                       far_ref=far_ref, n_rays_global=n_glob)
        if eng.poses is not None:
            slots = torch.nonzero(sel).squeeze(1)  # (FIXED: one host sync per step already, above)
            if self._world > 1:
                slots = slots[s0:s1]
            eng.poses.step(eng, rays, slots.contiguous(), eng.lr_factor)
        return out
