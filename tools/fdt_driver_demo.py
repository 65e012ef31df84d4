"""The north-star driver's flow (examples/fdt_optimize_implicit_map.py) on synthetic data, through
the reference-shaped surface only (GPU box):

  1. per-keyframe preprocessing: sky rays (lnr_sky_rays) for each scan;
  2. sliding keyframe windows, each optimised by ``Optimizer.iterate_optimizer`` with the driver's
     schedule edits (_keyframe_count = 1, NUM_ITERATIONS = 32 per window, freeze_poses, :529-541);
  3. compute_l1_depth on a held-out scan after every few windows (:595-612 / utils :260-282);
  4. the camera phase (ITERATE_CAMERA, :826-873): ``iterate_optimizer_camera`` over synthetic
     images;
  5. the final checkpoint in the reference's format (:619-624), reloaded.

    python tools/fdt_driver_demo.py [--kind quad] [--keyframes 24] [--window 8]
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NUM_ITERATIONS = 2 ** 5


def settings(kind):
    import bench
    from loner_amd import synthetic as syn
    preset = "haveri" if kind == "forest" else "default"
    sched = dict(num_keyframes=1, iteration_schedule=[dict(num_iterations=1000, freeze_poses=True,
                                                           freeze_sigma_mlp=False, freeze_rgb_mlp=True)])
    return dict(num_samples=dict(lidar=512, sky=64 if kind == "forest" else 0),
                rays_selection=dict(strategy="MASK" if kind == "forest" else "RANDOM"),
                samples_selection=dict(strategy="OGM"), skip_pose_refinement=True, freeze_poses=False,
                keyframe_schedule=[sched],
                model_config=dict(model=dict(ray_range=list(syn.SENSORS[kind]["ray_range"]),
                                             render=dict(N_samples_train=512, perturb=1.0, raw_noise_std=1.0),
                                             occ_model=dict(voxel_size=100, lr=1e-3 if preset == "haveri" else 1e-4,
                                                            N_iters_acc=10)),
                                  train=dict(lrate_sigma_mlp=0.01, lrate_rgb=0.01, lrate_gamma=1.0),
                                  loss=bench.LOSS_PRESETS[preset]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="quad")
    ap.add_argument("--keyframes", type=int, default=24)
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from loner_amd import camera as C
    from loner_amd import checkpoint as ckp
    from loner_amd import evaluate as E
    from loner_amd import preprocess as P
    from loner_amd import synthetic as syn
    from loner_amd.optimizer import Optimizer
    kind = args.kind
    dev = torch.device("cuda", 0)
    wc, rr = syn.world_cube(kind), syn.SENSORS[kind]["ray_range"]
    scans = syn.make_window(kind, args.keyframes, seed=2000)
    t_pre = time.perf_counter()
    for s in scans:  # 1. sky rays from each scan's own directions (compute_sky_rays)
        sky = P.sky_rays(s["directions"].T.contiguous().to(dev), s["pose"])  # (Q, 3), pose-rotated as the reference
        s["sky_directions"] = sky.T.contiguous().cpu() if sky.numel() else torch.zeros(3, 0)
    t_pre = time.perf_counter() - t_pre
    held = syn.make_window(kind, 1, seed=77, start=3)[0]
    sub = torch.arange(0, held["distances"].shape[0], 7)
    held = dict(directions=held["directions"][:, sub].contiguous(), distances=held["distances"][sub].contiguous(),
                pose=held["pose"])

    opt = Optimizer(settings(kind), None, wc, dev, seed=3)
    # the driver's schedule edits (fdt_optimize_implicit_map.py:529-541)
    opt._optimization_settings.num_iterations = NUM_ITERATIONS
    opt._keyframe_count = 1
    empty = copy.deepcopy(opt._keyframe_schedule[0])
    empty["num_keyframes"] = -1
    empty["iteration_schedule"][0].update(num_iterations=NUM_ITERATIONS, freeze_poses=True, freeze_sigma_mlp=False,
                                          freeze_rgb_mlp=True)
    opt._keyframe_schedule = [empty]
    rend = E.DepthRenderer(opt.state, n_samples=512, chunk=8192)

    def l1():
        return float(E.compute_l1_depth(rend, held, held["pose"], wc, rr, key=1).item())

    rec = dict(kind=kind, keyframes=args.keyframes, window=args.window, iterations_per_window=NUM_ITERATIONS,
               sky_rays_s=t_pre, l1_m=[[0, l1()]], loss=[])
    t0 = time.perf_counter()
    w = 0
    for k0 in range(0, args.keyframes - args.window + 1, 2):  # sliding windows, 2 new keyframes each
        loss = opt.iterate_optimizer(scans[k0:k0 + args.window])
        w += 1
        rec["loss"].append([opt._global_step, loss])
        if w % 3 == 0:
            rec["l1_m"].append([opt._global_step, l1()])
            print(f"window {w}: step {opt._global_step} loss {loss:.4f} l1 {rec['l1_m'][-1][1]:.3f} m", flush=True)
    torch.cuda.synchronize()
    rec["map_s"] = time.perf_counter() - t0
    rec["l1_m"].append([opt._global_step, l1()])

    # 4. camera phase on synthetic images seen from the keyframe poses (camera z = lidar x)
    W, H = 320, 180
    dirs = C.pinhole_directions(W, H, np.array([[160.0, 0, (W - 1) / 2], [0, 160.0, (H - 1) / 2], [0, 0, 1]]))
    l2c = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=np.float64)
    yy, xx = np.mgrid[0:H, 0:W]
    imgs, poses = [], []
    for s in scans[:6]:
        Pc = s["pose"].numpy().astype(np.float64)
        Pc[:3, :3] = Pc[:3, :3] @ l2c
        poses.append(Pc[:3])
        imgs.append(np.stack([0.5 + 0.4 * np.sin(xx / 17.0), 0.5 + 0.4 * np.cos(yy / 11.0),
                              0.4 + 0.2 * (xx > W / 2)], -1).reshape(-1, 3).astype(np.float32))
    frames = C.CameraFrames(dirs, W, H, imgs, poses, wc, rr, n_rays_per_kf=512, seed=0, device=dev)
    t1 = time.perf_counter()
    cam_losses = [opt.iterate_optimizer_camera(frames) for _ in range(3)]
    rec["camera_s"] = time.perf_counter() - t1
    rec["camera_loss_per_repetition"] = cam_losses

    # 5. checkpoint round trip
    import tempfile
    path = os.path.join(tempfile.mkdtemp(), "fdt_demo_ckpt.tar")
    ckp.save_checkpoint(path, opt.state, opt._global_step, other_params=ckp.color_params(opt.color))
    ck = torch.load(path, map_location="cpu", weights_only=True)
    rec["checkpoint_keys"] = sorted(ck["network_state_dict"])
    rec["global_step"] = int(ck["global_step"])
    print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
