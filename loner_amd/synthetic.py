"""Synthetic LiDAR workloads for the benchmark configurations C1-C5.

No datasets are reachable (no network, no ROS bags), so every config is an analytic scene
ray-cast with the sensor model of the reference's config:
  quad    Newer College quad-easy: OS0-128, 128 beams over +-45 deg (cfg/newer_college/quad.yaml:26),
          ranges [1, 75] m (:19), courtyard walls + ground + boxes, loop inside the bbox
          x[-5,50] y[-25,15] z[-3,10] (:8-14); world cube = compute_world_cube(bbox, padding 0.3)
  forest  haveri_hpk: QT64-like, 64 beams over +-52.1 deg (cfg/haveri_hpk/02_02_04.yaml:116),
          ranges [2.5, 45] m (:60), tree trunks + ground, poses = the reference's shipped keyframe
          trajectory (gazebo/example_implicit_map/trajectory/keyframe_trajectory.txt, stored as a
          fixture), world cube from gazebo/example_implicit_map/world_cube.yaml
  canteen Fusion Portable canteen: OS1-128 +-22.5 deg (cfg/fusion_portable/canteen.yaml:28),
          [1, 50] m (:19), indoor hall with pillars
Ray batches follow Optimizer._do_iterate_optimizer's selection (optimizer.py:363-424):
RANDOM (randint) or MASK (75 % "trunk" points 0.5 < z_sensor < 8 m), plus sky rays at r_max + 1.
All host-side numpy/torch; generated once, then resident on the GPU for the timed region.
"""
import os

import numpy as np
import torch

from . import rays as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SENSORS = {
    "quad": dict(n_beams=128, fov=(-45.0, 45.0), n_az=1024, ray_range=(1.0, 75.0)),
    "forest": dict(n_beams=64, fov=(-52.1, 52.1), n_az=600, ray_range=(2.5, 45.0)),
    "canteen": dict(n_beams=128, fov=(-22.5, 22.5), n_az=1024, ray_range=(1.0, 50.0)),
}
CUBES = {
    "quad": (121.426537, (-22.5, 5.0, -3.5)),          # SURVEY §8(c) / compute_world_cube(bbox, 0.3)
    "forest": (116.75345611572266, (-10.527198791503906, 89.2310791015625, 4.763427734375)),
    "canteen": (85.761414, (7.5, 5.0, 0.0)),
}


def sensor_directions(n_beams, fov, n_az):
    el = np.deg2rad(np.linspace(fov[0], fov[1], n_beams))
    az = np.linspace(-np.pi, np.pi, n_az, endpoint=False)
    E, A = np.meshgrid(el, az, indexing="ij")
    d = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)]).reshape(3, -1)
    return d.astype(np.float64)


class Scene:
    def __init__(self, ground_z, boxes=(), cylinders=None, cyl_height=12.0):
        self.ground_z = ground_z
        self.boxes = [np.asarray(b, np.float64) for b in boxes]  # (lo(3), hi(3)) as (2,3)
        self.cyl = np.zeros((0, 3)) if cylinders is None else np.asarray(cylinders, np.float64)  # x, y, r
        self.cyl_height = cyl_height

    def cast(self, o, d, r_max):
        """Distance along unit directions d (P,3) from o (3,) to the first hit, inf if none."""
        t = np.full(d.shape[0], np.inf)
        with np.errstate(divide="ignore", invalid="ignore"):
            tg = (self.ground_z - o[2]) / d[:, 2]
            t = np.where((tg > 0) & (tg < t), tg, t)
            for b in self.boxes:
                t0 = (b[0] - o) / d
                t1 = (b[1] - o) / d
                tn = np.nanmax(np.minimum(t0, t1), axis=1)
                tf = np.nanmin(np.maximum(t0, t1), axis=1)
                hit = (tf >= np.maximum(tn, 0)) & (tn > 0)
                t = np.where(hit & (tn < t), tn, t)
            if len(self.cyl):
                near = np.hypot(self.cyl[:, 0] - o[0], self.cyl[:, 1] - o[1]) < r_max + self.cyl[:, 2]
                for cx, cy, cr in self.cyl[near]:
                    px, py = o[0] - cx, o[1] - cy
                    a = d[:, 0] ** 2 + d[:, 1] ** 2
                    bq = 2 * (px * d[:, 0] + py * d[:, 1])
                    c = px * px + py * py - cr * cr
                    disc = bq * bq - 4 * a * c
                    tc = (-bq - np.sqrt(np.maximum(disc, 0))) / (2 * a)
                    zc = o[2] + tc * d[:, 2]
                    hit = (disc > 0) & (tc > 0) & (zc > self.ground_z) & (zc < self.ground_z + self.cyl_height)
                    t = np.where(hit & (tc < t), tc, t)
        return t


def make_scene(kind, rng):
    if kind == "quad":
        walls = [((-12, -22, -3), (52, -20, 12)), ((-12, 18, -3), (52, 20, 12)), ((-12, -22, -3), (-10, 20, 12)),
                 ((50, -22, -3), (52, 20, 12))]
        boxes = [((x, y, -1.5), (x + rng.uniform(1, 4), y + rng.uniform(1, 4), -1.5 + rng.uniform(0.5, 3)))
                 for x, y in rng.uniform((-5, -15), (45, 12), (25, 2))]
        return Scene(-1.5, walls + boxes)
    if kind == "forest":
        xy = rng.uniform((-80, -260), (100, 80), (3500, 2))
        r = rng.uniform(0.12, 0.45, (3500, 1))
        return Scene(-1.8, cylinders=np.concatenate([xy, r], 1))
    if kind == "canteen":
        walls = [((-25, -15, -1), (40, -14, 6)), ((-25, 24, -1), (40, 25, 6)), ((-25, -15, -1), (-24, 25, 6)),
                 ((39, -15, -1), (40, 25, 6)), ((-25, -15, 5), (40, 25, 6))]
        pillars = [((x, y, -1), (x + 0.6, y + 0.6, 5)) for x in range(-20, 36, 8) for y in range(-10, 22, 8)]
        return Scene(-1.0, walls + pillars)
    raise ValueError(kind)


def _yaw_pose(x, y, z, yaw):
    p = np.eye(4)
    c, s = np.cos(yaw), np.sin(yaw)
    p[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    p[:3, 3] = (x, y, z)
    return p


def _quat_pose(t, q):
    x, y, z, w = q
    Rm = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                   [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                   [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    p = np.eye(4)
    p[:3, :3] = Rm
    p[:3, 3] = t
    return p


def keyframe_poses(kind, n_kf, rng, start=0):
    if kind == "forest":
        tum = np.load(os.path.join(ROOT, "tests", "golden", "haveri_keyframe_trajectory.npz"))["tum"]
        idx = (start + np.arange(n_kf) * 3) % len(tum)
        return [_quat_pose(tum[i, 1:4], tum[i, 4:8]) for i in idx]
    if kind == "quad":
        ang = 2 * np.pi * (start + np.arange(n_kf)) / 48.0
        return [_yaw_pose(22 + 18 * np.cos(a), -3 + 12 * np.sin(a), 0.0, a + np.pi / 2) for a in ang]
    ang = 2 * np.pi * (start + np.arange(n_kf)) / 32.0
    return [_yaw_pose(7 + 12 * np.cos(a), 5 + 8 * np.sin(a), 0.5, a) for a in ang]


def make_window(kind, n_kf=16, seed=0, dropout=0.05, start=0, poses=None):
    """A keyframe window: list of dicts with sensor-frame directions (3,P), distances (P,),
    sky directions (3,Q) and the lidar pose (4,4), all torch float32 on the CPU.  ``poses``: explicit
    keyframe poses (4,4) instead of the config's trajectory."""
    rng = np.random.default_rng(seed)
    sc = SENSORS[kind]
    scene = make_scene(kind, np.random.default_rng(1234))
    dirs = sensor_directions(sc["n_beams"], sc["fov"], sc["n_az"])
    window = []
    for pose in (keyframe_poses(kind, n_kf, rng, start) if poses is None else poses):
        dw = (pose[:3, :3] @ dirs).T
        t = scene.cast(pose[:3, 3], dw, sc["ray_range"][1])
        hit = np.isfinite(t) & (t >= sc["ray_range"][0]) & (t < sc["ray_range"][1]) & (rng.uniform(size=t.shape) > dropout)
        sky = ~np.isfinite(t) & (dirs[2] > 0.05)
        window.append(dict(directions=torch.from_numpy(dirs[:, hit].astype(np.float32)),
                           distances=torch.from_numpy(t[hit].astype(np.float32)),
                           sky_directions=torch.from_numpy(dirs[:, sky].astype(np.float32)),
                           pose=torch.from_numpy(pose.astype(np.float32))))
    return window


def submap_window(part_id, n_kf=16, seed=0):
    """C5: the haveri trajectory split into <= 50 m submaps with +-30-pose padding as
    examples/fdt_segment_and_optimize_submaps.py does (loner_amd.submaps), submap part_id mod the part
    count: n_kf keyframes evenly spread over its padded pose range and its own world cube
    (compute_world_cube of all the padded range's poses, pose_utils.py:285-314).  Returns (scans, WorldCube, info dict)."""
    from . import submaps as SM
    tum = np.load(os.path.join(ROOT, "tests", "golden", "haveri_keyframe_trajectory.npz"))["tum"]
    parts = SM.split_trajectory(tum[:, 1:4])
    ranges = SM.padded_ranges(parts, len(tum))
    k = part_id % len(parts)
    lo, hi = ranges[k]
    idx = np.round(np.linspace(lo, hi, n_kf)).astype(int)
    poses = [_quat_pose(tum[i, 1:4], tum[i, 4:8]) for i in idx]
    scale, shift = SM.world_cube_from_poses(SM.poses_from_tum(tum[lo:hi + 1]), SENSORS["forest"]["ray_range"])
    wc = R.WorldCube(torch.tensor([scale], dtype=torch.float32), torch.from_numpy(shift))
    info = dict(part=k, n_parts=len(parts), core=list(parts[k]), padded=[lo, hi], cube_scale=scale)
    return make_window("forest", n_kf, seed=seed, poses=poses), wc, info


def world_cube(kind):
    s, sh = CUBES[kind]
    return R.WorldCube(torch.tensor([s], dtype=torch.float32), torch.tensor(sh, dtype=torch.float32))


def select_indices(scan, n, strategy, rng):
    P = scan["distances"].shape[0]
    if strategy == "MASK":
        xyz_z = (scan["directions"][2] * scan["distances"]).numpy()
        trunk = np.flatnonzero((0.5 < xyz_z) & (xyz_z < 8))
        other = np.flatnonzero(~((0.5 < xyz_z) & (xyz_z < 8)))
        nt = int(n * 0.75)
        sel = np.concatenate([rng.permutation(trunk)[:nt], rng.permutation(other)[:n - nt]])
        return torch.from_numpy(sel)
    return torch.from_numpy(rng.integers(0, P, n))


def build_batch(window, kind, rays_per_kf=512, sky_per_kf=0, strategy="RANDOM", seed=0, ray_range=None):
    """One optimiser step's (rays (R,13), depths (R,)) from a window (optimizer.py:363-424)."""
    rng = np.random.default_rng(seed)
    rr = torch.tensor(ray_range or SENSORS[kind]["ray_range"], dtype=torch.float32)
    wc = world_cube(kind)
    all_r, all_d = [], []
    for kf in window:
        li = select_indices(kf, rays_per_kf, strategy, rng)
        si = None
        if sky_per_kf > 0 and kf["sky_directions"].shape[1] > 0:
            si = torch.from_numpy(rng.integers(0, kf["sky_directions"].shape[1], sky_per_kf))
        r, d = R.build_keyframe_rays(kf, kf["pose"], li, rr, wc, si)
        all_r.append(r)
        all_d.append(d)
    return torch.cat(all_r).float().contiguous(), torch.cat(all_d).float().contiguous()


CONFIGS = {
    # name: (scene, n_kf, rays_per_kf, sky_per_kf, strategy, n_samples, loss preset)
    "C1": ("quad", 1, 512, 0, "RANDOM", 64, "default"),
    "C2": ("quad", 16, 512, 0, "RANDOM", 512, "default"),
    "C3": ("canteen", 8, 512, 0, "RANDOM", 2048, "default"),
    "C4": ("forest", 16, 512, 64, "MASK", 512, "haveri"),
    # C5 submaps: C4-like independent single-GPU jobs, one per GPU, no collectives
    # (examples/fdt_segment_and_optimize_submaps.py:24,86-109); each rank its own trajectory segment
    "C5": ("forest", 16, 512, 64, "MASK", 512, "haveri"),
}
