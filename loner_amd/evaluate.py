"""Inference / evaluation path on the fused HIP kernels.

    DepthRenderer      Model.forward(testing=True, camera=False) for depth: OGM sampler with
                       N_samples_test samples and no jitter (model_tcnn.py:77-81), sigma field,
                       'default' or 'adjusted' (peak) compositing (rendering_tcnn.py:70-295), with
                       the reference's test-time quirks: sigma noise stays on (raw_noise_std) and
                       the importance draws stay random (sample_pdf det=False).
    compute_l1_depth   examples/fdt_optimize_implicit_map_utils.py:260-282 and
                       analysis/compute_l1_depth.py:42-64: mean |depth * scale - range| over the
                       scan points with r_min < range < r_max - 0.25 m.

Rays of a whole scan are built on the device (``lnr_build_lidar_rays``, every point in order), so a
scan's evaluation is: one ray build, then per chunk one sampler, one hash-grid encode and one fused
render launch; the L1 reduction stays on the device.  The reference renders in chunks of 2^8 or 2^12 rays; chunks here only bound the
encoding workspace (``chunk`` rays x n_samples x 64 B).

Deviations: the reference's ``compute_l1_depth`` in examples/ passes render_strategy='threshold',
which its own render_rays rejects (rendering_tcnn.py:394-404, ValueError), so 'default' is used, as
analysis/compute_l1_depth.py does.  Rays failing the 1 m validity filter (ray_utils.py:319-322) are
dropped by the reference before rendering, which misaligns its chunk writes; here they are simply
excluded from the mean.
"""
import torch

from . import _lib as L
from .rays import RayWindow

_STRATEGY = {"default": 0, "adjusted": 1}


class DepthRenderer:
    """Forward-only depth rendering of a ``loner_amd.step.FieldState``."""

    def __init__(self, state, n_samples=2048, chunk=8192, raw_noise_std=1.0, sampler="OGM"):
        if n_samples % 64:
            raise ValueError(f"n_samples={n_samples} must be a multiple of 64")
        self.state = state
        self.S = int(n_samples)
        self.chunk = int(chunk)
        self.noise_std = float(raw_noise_std)
        self.sampler = sampler
        dev = state.device
        self.z = torch.empty(self.chunk, self.S, dtype=torch.float32, device=dev)
        self.enc = torch.empty(state.cfg.n_levels, self.chunk * self.S, dtype=torch.int32, device=dev)

    def render(self, rays, key, strategy="default", depth=None, opacity=None, variance=None, ray_offset=0):
        """rays (R,13) on the GPU -> depth, opacity, variance (R,) normalised units (device)."""
        if strategy not in _STRATEGY:
            raise ValueError(f"Unknown render strategy: {strategy}")  # rendering_tcnn.py:404
        st = self.state
        dev = st.device
        R = rays.shape[0]
        depth = torch.empty(R, dtype=torch.float32, device=dev) if depth is None else depth
        opacity = torch.empty(R, dtype=torch.float32, device=dev) if opacity is None else opacity
        variance = torch.empty(R, dtype=torch.float32, device=dev) if variance is None else variance
        s = L.stream(dev)
        stride = self.chunk * self.S
        for r0 in range(0, R, self.chunk):
            n = min(self.chunk, R - r0)
            rc = rays[r0:r0 + n]
            off = ray_offset + r0
            if self.sampler == "OGM":
                L.call("lnr_sample_ogm", rc, n, self.S, st.occ, st.cfg.occ_res, 0.0, None, None, key, off, self.z, s)
            else:
                L.call("lnr_sample_uniform", rc, n, self.S, 0.0, None, key, off, self.z, s)
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rc, self.z, n, self.S, st.table_f16, self.enc,
                   stride, None, 0, s)
            L.call("lnr_field_render", st.mlp_f16, self.enc, stride, rc, self.z, n, self.S, _STRATEGY[strategy],
                   self.noise_std, None, key, off, depth[r0:r0 + n], opacity[r0:r0 + n], variance[r0:r0 + n], None, s)
        return depth, opacity, variance


def scan_window(scan, pose, world_cube, ray_range, device):
    """A one-keyframe RayWindow over a whole scan (LidarRayDirections over every point)."""
    s = dict(directions=scan["directions"], distances=scan["distances"], pose=pose)
    return RayWindow([s], world_cube, ray_range, n_lidar=1, strategy="RANDOM", device=device)


def compute_l1_depth(renderer, scan, pose, world_cube, ray_range, key=0, strategy="default"):
    """L1 depth error (metres) of one scan; returns a 0-d device tensor.  The only host
    synchronisation is the scan window's one-off validity check (RayWindow)."""
    win = scan_window(scan, pose, world_cube, ray_range, renderer.state.device)
    rays, _, valid = win.build_all()
    depth, _, _ = renderer.render(rays, key, strategy)
    scale = win.scale
    rng_m = win.dists  # the scan's ranges in metres, in slot order
    good = (rng_m > float(ray_range[0])) & (rng_m < float(ray_range[1]) - 0.25) & valid.bool()
    err = (depth * scale - rng_m).abs()
    return (err * good).sum() / good.sum().clamp(min=1)
