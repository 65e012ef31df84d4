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


class ColorHead:
    """The colour branch of DecoupledNeRF (nerf_tcnn.py:40-52,80-95) for rendering: the T=2^19
    colour HashGrid table and the 48 -> 64 x n_hidden_layers -> 3 FullyFusedMLP, both fp16 on the
    GPU in tcnn's flat layouts.  ``table`` / ``mlp`` are the ``params`` of the reference's
    ``_pos_encoding`` and ``_model_intensity`` modules (or of loner_amd.tcnn's), in any float dtype."""

    def __init__(self, table, mlp, n_hidden_layers=4, n_levels=16, log2_hashmap_size=19, base_resolution=16,
                 device="cuda"):
        self.desc = L.grid_desc(n_levels, 2, log2_hashmap_size, base_resolution, 2.0)
        self.n_hidden_layers = int(n_hidden_layers)
        n_mlp = 64 * 48 + (self.n_hidden_layers - 1) * 64 * 64 + 16 * 64
        if table.numel() != 2 * self.desc.n_entries or mlp.numel() != n_mlp:
            raise RuntimeError(f"colour head sizes: table {table.numel()} (want {2 * self.desc.n_entries}), "
                               f"mlp {mlp.numel()} (want {n_mlp})")
        self.table = table.detach().reshape(-1).to(device, torch.float16).contiguous()
        self.mlp = mlp.detach().reshape(-1).to(device, torch.float16).contiguous()
        self.n_levels = n_levels

    @staticmethod
    def init(n_hidden_layers=4, seed=1337, device="cuda"):
        """tcnn-style initialisation: table U(-1e-4, 1e-4), Xavier-uniform layers (counter-based draws)."""
        import math
        desc = L.grid_desc(16, 2, 19, 16, 2.0)
        dev = torch.device(device)
        s = L.stream(dev)
        table = torch.empty(2 * desc.n_entries, dtype=torch.float32, device=dev)
        L.call("lnr_fill_uniform", table, table.numel(), seed, -1e-4, 1e-4, 0, s)
        shapes = [(64, 48)] + [(64, 64)] * (n_hidden_layers - 1) + [(16, 64)]
        parts = []
        for k, (o, i) in enumerate(shapes):
            a = math.sqrt(6.0 / (o + i))
            w = torch.empty(o * i, dtype=torch.float32, device=dev)
            L.call("lnr_fill_uniform", w, o * i, seed + 1 + k, -a, a, 0, s)
            parts.append(w)
        return ColorHead(table, torch.cat(parts), n_hidden_layers, device=dev)


class DepthRenderer:
    """Forward-only rendering of a ``loner_amd.step.FieldState``: depth / opacity / variance, and
    the colour map when a ``ColorHead`` is given (Model.forward(testing=True, camera=True))."""

    def __init__(self, state, n_samples=2048, chunk=8192, raw_noise_std=1.0, sampler="OGM", color=None):
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
        self.color = color
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)  # LNR_STATUS_* bits (DEBUG scan)
        if color is not None:
            if self.S % 16:
                raise ValueError("colour rendering needs n_samples % 16 == 0")
            self.enc_rgb = torch.empty(color.n_levels, self.chunk * self.S, dtype=torch.int32, device=dev)
            self.weights = torch.empty(self.chunk, self.S, dtype=torch.float32, device=dev)

    def render(self, rays, key, strategy="default", depth=None, opacity=None, variance=None, ray_offset=0,
               rgb=None):
        """rays (R,13) on the GPU -> depth, opacity, variance (R,) normalised units (device).  With a
        colour head, ``rgb`` (R,3) receives the white-background colour map."""
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
                L.call("lnr_sample_ogm", rc, n, self.S, st.occ, st.cfg.occ_res, 0.0, None, None, key, off, self.z, None, s)
            else:
                L.call("lnr_sample_uniform", rc, n, self.S, 0.0, None, key, off, self.z, None, s)
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rc, self.z, n, self.S, st.table_f16, self.enc,
                   stride, None, 0, s)
            cw = self.color is not None and rgb is not None
            L.call("lnr_field_render", st.mlp_f16, self.enc, stride, rc, self.z, n, self.S, _STRATEGY[strategy],
                   self.noise_std, None, key, off, depth[r0:r0 + n], opacity[r0:r0 + n], variance[r0:r0 + n],
                   self.weights if cw else None, s)
            if cw:
                c = self.color
                # zero-weight samples cannot change rgb: no colour-grid gathers for them
                L.call("lnr_hashgrid_fwd_rays_live", L.ctypes.byref(c.desc), rc, self.z, n, self.S, c.table,
                       self.weights, self.enc_rgb, stride, s)
                L.call("lnr_rgb_render", c.mlp, c.n_hidden_layers, self.enc_rgb, stride, rc, self.weights, n, self.S,
                       rgb[r0:r0 + n], s)
        for t in (depth, opacity, variance) + ((rgb,) if rgb is not None else ()):
            L.call("lnr_status_scan", t, t.numel(), L.STATUS_NONFINITE_OUTPUT, self.status, s)
        return depth, opacity, variance

    def check_status(self, clear=True):
        """Model.forward's DEBUG scan (rendering_tcnn.py:419-424) without a per-render sync: prints the
        reference's message when any rendered output held nan/inf since the last check."""
        bits = int(self.status.item())
        if clear:
            self.status.zero_()
        if bits & L.STATUS_NONFINITE_OUTPUT:
            print("! [Numerical Error] a rendered output contains nan or inf.")
        return bits


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
