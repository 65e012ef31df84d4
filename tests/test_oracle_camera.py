"""oracle/camera.py's hand-written colour-loss backward pinned against torch autograd (CPU, fp64).

The autograd graph mirrors compute_loss_camera (optimizer.py:861-894) on DecoupledNeRF's colour
branch: FullyFusedMLP (no biases, ReLU, output padded to 16) -> sigmoid -> weights-composited rgb +
white background -> l1_loss over 3 x rays.  The fp16 roundings of the oracle's forward enter the
graph as straight-through values (x + (round(x) - x).detach()), so both sides differentiate the same
function at the same point and must agree to fp64 rounding."""
import numpy as np
import torch

from oracle import camera as ocam
from oracle import mlp as omlp


def _st16(x):
    return x + (x.to(torch.float16).to(torch.float64) - x).detach()


def test_rgb_train_backward_matches_autograd():
    rng = np.random.default_rng(0)
    R, S, nh = 6, 32, 3
    N = R * S
    enc = rng.uniform(-1, 1, (N, 32)).astype(np.float16)
    o = rng.uniform(-0.5, 0.5, (R, 3))
    d = rng.normal(size=(R, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, -d, np.zeros((R, 4))], 1).astype(np.float32)
    w = (rng.dirichlet(np.full(S, 0.5), R) * 0.8).astype(np.float32)
    mats = [rng.uniform(-0.3, 0.3, s).astype(np.float16) for s in omlp.layer_shapes(48, 3, 64, nh)]
    rgb0, x, _, _ = ocam.rgb_forward(enc, rays, w, mats, S)
    gt = rgb0 + rng.choice([-1, 1], rgb0.shape) * 0.1
    ref = ocam.rgb_train(enc, rays, w, gt, mats, S)

    X = torch.tensor(x.astype(np.float64), requires_grad=True)
    Ws = [torch.tensor(m.astype(np.float64), requires_grad=True) for m in mats]
    h = X
    for i, Wl in enumerate(Ws):
        h = h @ Wl.T
        if i < len(Ws) - 1:
            h = _st16(torch.relu(h))
    hc = _st16(h[:, :3])
    # torch.sigmoid on the reference's fp16 tensor: SigmoidBackward uses the fp16 OUTPUT y, y(1 - y)
    y = torch.sigmoid(hc).to(torch.float16).to(torch.float64).detach()
    col = y + (hc - hc.detach()) * (y * (1 - y))
    wt = torch.tensor(w.astype(np.float64))
    rgb = (wt[..., None] * col.reshape(R, S, 3)).sum(1) + (1 - wt.sum(1, keepdim=True))
    loss = torch.nn.functional.l1_loss(rgb.reshape(-1, 1), torch.tensor(gt).reshape(-1, 1))
    loss.backward()
    np.testing.assert_allclose(rgb.detach().numpy(), ref["rgb"], rtol=0, atol=1e-12)
    assert abs(loss.item() - ref["loss"]) < 1e-12
    np.testing.assert_allclose(X.grad.numpy()[:, :32], ref["d_enc"], rtol=1e-9, atol=1e-15)
    got = np.concatenate([Wl.grad.numpy().reshape(-1) for Wl in Ws])
    np.testing.assert_allclose(got, ref["d_w"], rtol=1e-9, atol=1e-15)


def test_camera_rays_oracle_matches_reference_formula():
    """CameraRayDirections.build_rays (ray_utils.py:175-212) written with torch ops as the reference
    does (homogeneous origin, directions @ R^T, get_far_val) against the oracle's fp32 restatement."""
    rng = np.random.default_rng(1)
    W, H = 8, 6
    dirs = np.concatenate([rng.uniform(-0.5, 0.5, (W * H, 2)), np.ones((W * H, 1))], 1).astype(np.float32)
    pose = np.eye(4, dtype=np.float32)
    a = 0.7
    pose[:3, :3] = [[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]]
    pose[:3, 3] = [2.0, -1.0, 0.5]
    scale, shift, r_min = 10.0, np.array([0.5, 0.5, -0.25], np.float32), 1.0
    pix = rng.choice(W * H, 20, replace=False)
    img = rng.uniform(0, 1, (W * H, 3)).astype(np.float32)
    rays, inten = ocam.build_camera_rays(dirs, img, pix, pose[:3], scale, shift, r_min, W)
    T = torch.tensor(pose)
    T[:3, 3] = (T[:3, 3] + torch.tensor(shift)) / scale
    dt = torch.tensor(dirs)[pix] @ T[:3, :3].T
    dt = dt / torch.norm(dt, dim=-1, keepdim=True)
    ot = torch.cat([torch.zeros_like(dt), torch.ones_like(dt[:, :1])], -1) @ T[:3, :].T
    far = torch.stack([torch.clamp((-1 - ot) / (dt + 1e-15), min=0), torch.clamp((1 - ot) / (dt + 1e-15), min=0)],
                      0).max(0).values.min(1).values
    np.testing.assert_allclose(rays[:, 0:3], ot.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rays[:, 3:6], dt.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rays[:, 6:9], -dt.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(rays[:, 9], pix % W)
    np.testing.assert_array_equal(rays[:, 10], pix // W)
    np.testing.assert_allclose(rays[:, 11], r_min / scale)
    np.testing.assert_allclose(rays[:, 12], far.numpy(), rtol=1e-5)
    np.testing.assert_array_equal(inten, img[pix])
