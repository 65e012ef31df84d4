"""Optimiser restatements in numpy — TEST INFRASTRUCTURE ONLY.

adam_step  ``torch.optim.Adam`` (defaults betas (0.9, 0.999), eps 1e-8, no weight decay) as built
           per window at ``src/mapping/optimizer.py:255-265`` and stepped at ``:460``; torch 2.x
           single-tensor update: m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2; p -= lr/bc1 * m /
           (sqrt(v)/sqrt(bc2) + eps).
ogm_step   ``Optimizer._step_occupancy_grid`` ``src/mapping/optimizer.py:897-908``: grid_sample
           backward of the per-sample logit "gradient" (``losses.py:54-62``) then SGD.
"""
import numpy as np

from . import render, loss

F32 = np.float32


def adam_step(p, g, m, v, step, lr, b1=0.9, b2=0.999, eps=1e-8):
    """In-place fp32 Adam; ``step`` is the 1-based step count after increment."""
    g = g.astype(F32)
    m += (F32(1 - b1) * (g - m)).astype(F32)
    v *= F32(b2)
    v += (F32(1 - b2) * g * g).astype(F32)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    step_size = F32(lr / bc1)
    denom = (np.sqrt(v) / F32(np.sqrt(bc2)) + F32(eps)).astype(F32)
    p -= (step_size * (m / denom)).astype(F32)
    return p, m, v


def ogm_step(grid, rays, z, depth_gt, scale, lr):
    """grid (D,H,W) fp32 updated in place; returns the fp64 gradient."""
    pts = (rays[:, None, 0:3] + rays[:, None, 3:6] * z[:, :, None]).astype(F32)
    lg = loss.logits_grad((z * F32(scale)).astype(F32), (depth_gt * F32(scale)).astype(F32))
    gr = render.grid_sample_3d_backward(grid.shape, pts, lg)
    grid -= (F32(lr) * gr).astype(F32)
    return gr
