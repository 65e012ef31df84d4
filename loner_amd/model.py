"""Model / OccupancyGridModel with the reference's interface (src/models/model_tcnn.py:24-134),
built on the HIP DecoupledNeRF and render_rays of this package.  ``cfg`` may be the reference's
AttrDict or any mapping (attribute or key access)."""
from collections import defaultdict

import torch
import torch.nn as nn

from .nerf import DecoupledNeRF
from .rendering import inference, render_rays


class _Cfg:
    """Attribute view over a mapping (AttrDict-compatible)."""

    def __init__(self, d):
        self._d = d

    def __getattr__(self, k):
        d = object.__getattribute__(self, "_d")
        v = getattr(d, k) if hasattr(d, k) and not isinstance(d, dict) else d[k]
        return _Cfg(v) if isinstance(v, dict) else v

    def __getitem__(self, k):
        return self._d[k]


def _cfg(c):
    return c if isinstance(c, _Cfg) else _Cfg(c)


class Model(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        self.cfg = _cfg(cfg)
        if self.cfg.model_type == 'nerf_decoupled':
            nc = self.cfg.nerf_config
            self.nerf_model = DecoupledNeRF(nc._d if isinstance(nc, _Cfg) else nc, self.cfg.num_colors, device=device)
        else:
            raise NotImplementedError()

    def get_rgb_parameters(self, ignore_requires_grad=False):
        m = self.nerf_model
        params = list(m._model_intensity.parameters()) + list(m._pos_encoding.parameters()) + \
            ([] if m._dir_encoding is None else list(m._dir_encoding.parameters()))
        return params if ignore_requires_grad else [p for p in params if p.requires_grad]

    def get_rgb_mlp_parameters(self):
        return list(self.nerf_model._model_intensity.parameters())

    def get_rgb_feature_parameters(self):
        m = self.nerf_model
        params = list(m._pos_encoding.parameters()) + \
            ([] if m._dir_encoding is None else list(m._dir_encoding.parameters()))
        return [p for p in params if p.requires_grad]

    def get_sigma_parameters(self, ignore_requires_grad=False):
        params = list(self.nerf_model._model_sigma.parameters())
        return params if ignore_requires_grad else [p for p in params if p.requires_grad]

    def freeze_sigma_head(self, should_freeze=True):
        for p in self.get_sigma_parameters(True):
            p.requires_grad = not should_freeze

    def freeze_rgb_head(self, should_freeze=True):
        for p in self.get_rgb_parameters(True):
            p.requires_grad = not should_freeze

    def inference_points(self, xyz_, dir_, sigma_only):
        return inference(self.nerf_model, xyz_, dir_, netchunk=0, sigma_only=sigma_only, meshing=True)

    def forward(self, rays, ray_sampler, scale_factor, testing=False, camera=True, detach_sigma=True,
                return_variance=False, render_strategy='default'):
        """model_tcnn.py:70-108: chunked render_rays, results concatenated per key."""
        r = self.cfg.render
        if testing:
            n_samples, perturb = r.N_samples_test, 0.
        else:
            n_samples, perturb = r.N_samples_train, r.perturb
        results = defaultdict(list)
        for i in range(0, rays.shape[0], r.chunk):
            out = render_rays(rays[i:i + r.chunk, :], ray_sampler, self.nerf_model, self.cfg.ray_range, scale_factor,
                              N_samples=n_samples, retraw=r.retraw, perturb=perturb, white_bkgd=True,
                              raw_noise_std=r.raw_noise_std, netchunk=r.netchunk, num_colors=self.cfg.num_colors,
                              sigma_only=(not camera), DEBUG=True, detach_sigma=detach_sigma,
                              return_variance=return_variance, render_strategy=render_strategy)
            for k, v in out.items():
                results[k] += [v]
        for k, v in results.items():
            results[k] = torch.cat(v, 0)
        return results


class _GridSample3d(torch.autograd.Function):
    """grid_sample on a (1, 1, R, R, R) grid at (..., 3) points on the HIP path (lnr_grid_sample3d and
    its deterministic backward): the values, and the grid's gradient on backward."""

    @staticmethod
    def forward(ctx, grid, pts):
        from . import _lib as L
        R = grid.shape[-1]
        p = pts.detach().reshape(-1, 3).contiguous()
        out = torch.empty(p.shape[0], dtype=torch.float32, device=grid.device)
        L.call("lnr_grid_sample3d", grid.detach().contiguous(), R, p, p.shape[0], out, L.stream(grid.device))
        ctx.save_for_backward(p)
        ctx.res = R
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import _lib as L
        if ctx.needs_input_grad[1]:
            raise NotImplementedError("OccupancyGridModel.interpolate: no gradient for the points "
                                      "(the reference's points are detached)")
        (p,) = ctx.saved_tensors
        R = ctx.res
        ws = torch.empty(int(L.lib().lnr_grid_sample3d_bwd_workspace_words(R)), dtype=torch.float32, device=p.device)
        dgrid = torch.empty(1, 1, R, R, R, dtype=torch.float32, device=p.device)
        L.call("lnr_grid_sample3d_bwd", p, dout.reshape(-1).contiguous().float(), p.shape[0], R, dgrid, ws, ws.numel(),
               L.stream(p.device))
        return dgrid, None


class OccupancyGridModel(nn.Module):
    """model_tcnn.py:111-134.  ``interpolate`` runs lnr_grid_sample3d (forward) and
    lnr_grid_sample3d_bwd (the grid's gradient, what _step_occupancy_grid backpropagates,
    optimizer.py:897-908); the sampler's own lookup is fused into the HIP sampler kernel."""

    def __init__(self, cfg, device=None):
        super().__init__()
        self.cfg = _cfg(cfg)
        v = self.cfg.voxel_size
        self.occupancy_grid = nn.Parameter(torch.zeros(1, 1, v, v, v, device=device))

    def forward(self):
        return self.occupancy_grid

    @staticmethod
    def interpolate(occupancy_grid, ray_bin_centers, mode='bilinear'):
        """grid_sample(occupancy_grid, points, mode, align_corners=False) -> (n_rays, n_bins), for a
        (1, 1, R, R, R) fp32 device grid and (n_rays, n_bins, 3) points; ``mode`` 'bilinear' (the
        reference's only use).  Anything else raises: there is no host fallback."""
        n_rays, n_bins, _ = ray_bin_centers.shape
        g = occupancy_grid
        if mode != 'bilinear':
            raise NotImplementedError(f"OccupancyGridModel.interpolate: mode={mode!r} (only 'bilinear')")
        if not (g.is_cuda and ray_bin_centers.is_cuda and g.dtype == torch.float32 and
                ray_bin_centers.dtype == torch.float32 and g.dim() == 5 and g.shape[:2] == (1, 1) and
                g.shape[2] == g.shape[3] == g.shape[4]):
            raise ValueError("OccupancyGridModel.interpolate: needs a (1, 1, R, R, R) fp32 device grid and "
                             "fp32 device points")
        return _GridSample3d.apply(g, ray_bin_centers).reshape(n_rays, n_bins)
