"""Camera phase (colour-head training) restated in numpy -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this package.

* ``build_camera_rays``: KeyFrame.build_camera_rays -> CameraRayDirections.build_rays
  (src/mapping/keyframe.py:108-127, src/common/ray_utils.py:175-212), fp32.
* ``rgb_train``: compute_loss_camera (src/mapping/optimizer.py:861-894) with detached compositing
  weights: rgb = sum_i w_i sigmoid(h_c,i) + 1 - sum_i w_i (rendering_tcnn.py:283-289), loss =
  l1_loss over 3 x rays; its autograd restated by hand: dL/drgb = sign(rgb - gt) / (3R),
  dL/dcolor_i = w_i dL/drgb, sigmoid backward, then the FullyFusedMLP backward (oracle/mlp.py) in
  fp64 from the fp16 activations.  tcnn's own backward arithmetic (fp16 with loss scaling) is not
  vendored: parity for the gradients is unpinned, checked against this fp64 restatement with the
  tolerance written in the test.
"""
import numpy as np

from . import mlp as omlp
from .render import sh4


def get_far_val(o, d):
    """ray_utils.get_far_val(no_nan=True), fp32 (as oracle.rays.get_far_val)."""
    dd = d + np.float32(1e-15)
    t0 = np.maximum((np.float32(-1) - o) / dd, np.float32(0))
    t1 = np.maximum((np.float32(1) - o) / dd, np.float32(0))
    return np.maximum(t0, t1).min(axis=1)


def build_camera_rays(dirs, image, pixels, pose3x4, scale, shift, r_min, width):
    dirs = np.asarray(dirs, np.float32)
    P = np.asarray(pose3x4, np.float32)
    sc = np.float32(scale)
    o = ((P[:, 3] + np.asarray(shift, np.float32)) / sc).astype(np.float32)
    dp = dirs[pixels]
    d = ((dp[:, 0:1] * P[None, :, 0] + dp[:, 1:2] * P[None, :, 1]) + dp[:, 2:3] * P[None, :, 2]).astype(np.float32)
    nrm = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
    d = (d / nrm[:, None]).astype(np.float32)
    n = len(pixels)
    O = np.repeat(o[None], n, 0)
    far = get_far_val(O, d)
    rays = np.concatenate([O, d, -d, (pixels % width)[:, None].astype(np.float32),
                           (pixels // width)[:, None].astype(np.float32),
                           np.full((n, 1), np.float32(r_min) / sc, np.float32), far[:, None]], 1).astype(np.float32)
    inten = np.asarray(image, np.float32)[pixels]
    return rays, inten


def composite_rgb(weights, col):
    """raw2outputs' colour map with white background (rendering_tcnn.py:283-289):
    rgb = sum_i w_i c_i + 1 - sum_i w_i; weights (R,S), col (R,S,3) -> (R,3) fp64."""
    w = np.asarray(weights, np.float64)
    return (w[..., None] * np.asarray(col, np.float64)).sum(1) + (1 - w.sum(1, keepdims=True))


def rgb_loss_grad(rgb, gt, weights, n_rays):
    """compute_loss_camera (optimizer.py:861-894): l1_loss over 3 x n_rays colour values, and its
    gradient with respect to each sample's colour, w_i sign(rgb - gt) / (3 n) -> (loss, (R,S,3))."""
    diff = np.asarray(rgb, np.float64) - np.asarray(gt, np.float64)
    g = np.sign(diff) / (3.0 * n_rays)
    return np.abs(diff).sum() / (3.0 * n_rays), np.asarray(weights, np.float64)[..., None] * g[:, None, :]


def rgb_forward(enc32, rays, weights, mats_f16, S):
    """enc32 (N, 32) fp16 colour-grid features, rays (R, 13), weights (R, S) -> (rgb (R,3) fp64,
    x (N,48) fp16, hidden list, col (N,3) fp64)."""
    R = rays.shape[0]
    d01 = ((rays[:, 6:9] + np.float32(1)) / np.float32(2)).astype(np.float32)
    h_d = np.repeat(sh4(d01), S, axis=0)
    x = np.concatenate([np.asarray(enc32, np.float16), h_d], 1)
    out16, hidden = omlp.forward(x, mats_f16)
    col = (1 / (1 + np.exp(-out16[:, :3].astype(np.float32)))).astype(np.float16).astype(np.float64)
    rgb = composite_rgb(np.asarray(weights, np.float64).reshape(R, S), col.reshape(R, S, 3))
    return rgb, x, hidden, col


def rgb_train(enc32, rays, weights, gt, mats_f16, S, n_rays_global=None):
    """-> dict(rgb, loss, d_enc (N,32), d_w (flat, tcnn layer order)) in fp64."""
    R = rays.shape[0]
    rgb, x, hidden, col = rgb_forward(enc32, rays, weights, mats_f16, S)
    n = R if n_rays_global is None else n_rays_global
    loss, dcol = rgb_loss_grad(rgb, gt, np.asarray(weights, np.float64).reshape(R, S), n)
    dcol = dcol.reshape(-1, 3)
    dlogit = dcol * col * (1 - col)
    d_out = np.zeros((x.shape[0], mats_f16[-1].shape[0]))
    d_out[:, :3] = dlogit
    d_x, dws = omlp.backward(x, mats_f16, hidden, d_out)
    return dict(rgb=rgb, loss=loss, d_enc=d_x[:, :32],
                d_w=np.concatenate([dw.reshape(-1) for dw in dws]))
