"""Fractions of zero-weight samples and zero colour gradients in one CAM-shaped camera iteration
(GPU box): the inputs behind the camera phase's skip_zero measurement.

    python tools/zero_fraction.py
"""
import sys, torch, numpy as np
sys.path.insert(0, '.')
from loner_amd import camera as C, step as S_, synthetic as syn
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
n_kf, per_kf, S, W, H = 6, 512, 512, 1280, 720
K = np.array([[640.0, 0, (W - 1) / 2], [0, 640.0, (H - 1) / 2], [0, 0, 1]])
dirs = C.pinhole_directions(W, H, K)
l2c = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=np.float64)
poses, imgs = [], []
for k, P in enumerate(syn.keyframe_poses("forest", n_kf, np.random.default_rng(0))):
    Pc = np.array(P, dtype=np.float64); Pc[:3, :3] = Pc[:3, :3] @ l2c; poses.append(Pc[:3])
    imgs.append(np.full((W * H, 3), 0.5, np.float32))
fr = C.CameraFrames(dirs, W, H, imgs, poses, syn.world_cube("forest"), syn.SENSORS["forest"]["ray_range"], n_rays_per_kf=per_kf, device=dev)
st = S_.FieldState(S_.StepConfig(n_samples=S), device=dev)
cs = C.ColorState(4, device=dev)
R = n_kf * per_kf
eng = C.CameraStepEngine(st, cs, n_rays=R, n_samples=S)
rays = torch.empty(R, 13, device=dev); inten = torch.empty(R, 3, device=dev)
n = fr.build(1, rays, inten)
eng.step(rays[:n], inten[:n])
torch.cuda.synchronize()
w = eng.weights[:n]
print("w==0 frac", float((w == 0).float().mean()))
de = eng.denc_f32()[:, :n * S]
print("d_enc zero frac per level", [round(float(((de[l] == 0).all(-1)).float().mean()), 3) for l in range(16)])
tiles = (w.reshape(-1, 16) == 0).all(-1).float().mean()
print("all-zero 16-tiles", float(tiles))
