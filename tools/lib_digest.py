"""Digest of a few training steps (C2 shape: 16 keyframes x 512 rays x 512 samples, synthetic quad
window): sha256 of the fp32 parameters, the Adam moments and the last step's loss after K steps.  Run
once per library build (LONER_AMD_LIB=...) to check that an experiment variant changes no bit.  With
``cam``: the same over K camera-phase iterations (bench.py --config CAM's shape: colour parameters, moments,
loss).

    LONER_AMD_LIB=loner_amd/_lib/variants/x.so python tools/lib_digest.py [steps] [cam]
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loner_amd import _lib as L  # noqa: E402
from loner_amd import step as S_  # noqa: E402
from loner_amd import synthetic as syn  # noqa: E402
from loner_amd.rays import RayWindow  # noqa: E402


def sha(t):
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]


def camera(steps):
    import numpy as np
    from loner_amd import camera as C
    dev = torch.device("cuda", 0)
    n_kf, per_kf, S, W, H = 6, 512, 512, 320, 180
    kind = "forest"
    K = np.array([[160.0, 0, (W - 1) / 2], [0, 160.0, (H - 1) / 2], [0, 0, 1]])
    dirs = C.pinhole_directions(W, H, K)
    lidar_to_cam = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=np.float64)
    poses, imgs = [], []
    yy, xx = np.mgrid[0:H, 0:W]
    for k, P in enumerate(syn.keyframe_poses(kind, n_kf, np.random.default_rng(0))):
        Pc = np.array(P, dtype=np.float64)
        Pc[:3, :3] = Pc[:3, :3] @ lidar_to_cam
        poses.append(Pc[:3])
        imgs.append(np.stack([0.5 + 0.4 * np.sin(xx / 37.0 + k), 0.5 + 0.4 * np.cos(yy / 23.0),
                              0.3 + 0.2 * np.sin((xx + yy) / 50.0)], -1).reshape(-1, 3).astype(np.float32))
    fr = C.CameraFrames(dirs, W, H, imgs, poses, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                        n_rays_per_kf=per_kf, seed=0, device=dev)
    state = S_.FieldState(S_.StepConfig(n_samples=S), device=dev)
    color = C.ColorState(4, device=dev)
    R = n_kf * per_kf
    eng = C.CameraStepEngine(state, color, n_rays=R, n_samples=S, seed=0)
    rays = torch.empty(R, 13, dtype=torch.float32, device=dev)
    inten = torch.empty(R, 3, dtype=torch.float32, device=dev)
    loss = None
    for i in range(steps):
        fr.build(1 + i % (fr.n_iter - 1), rays, inten)
        loss = eng.step(rays, inten, global_step=i + 1)
    torch.cuda.synchronize()
    print(json.dumps(dict(lib=os.path.basename(L.LIB_PATH), camera_steps=steps, params=sha(color.params),
                          m=sha(color.m), v=sha(color.v), loss=sha(loss))))


def main(steps=3, mode="lidar"):
    steps = int(steps)
    if mode == "cam":
        return camera(steps)
    scans = syn.make_window("quad", 16, seed=1)
    win = RayWindow(scans, syn.world_cube("quad"), syn.SENSORS["quad"]["ray_range"], n_lidar=512, strategy="RANDOM")
    st = S_.FieldState(S_.StepConfig(n_samples=512), device="cuda:0")
    eng = S_.StepEngine(st, win.n_slots, seed=3)
    loss = None
    for g in range(1, steps + 1):
        loss = eng.step_window(win, global_step=g)
    eng.drop_prefetch()
    torch.cuda.synchronize()
    print(json.dumps(dict(lib=os.path.basename(L.LIB_PATH), steps=steps, params=sha(st.params), m=sha(st.m),
                          v=sha(st.v), loss=sha(loss) if torch.is_tensor(loss) else None)))


if __name__ == "__main__":
    main(*sys.argv[1:])
