"""Volume rendering on the HIP kernels, with the reference's call surface
(src/models/rendering_tcnn.py): ``render_rays``, ``inference``, ``raw2outputs``,
``raw2outputs_adjusted``.

Differences from the reference, all deliberate:
  * compositing runs in one HIP kernel per ray (lnr_composite) and its autograd backward in
    another (lnr_composite_bwd: the reverse affine scan of DESIGN.md) instead of ~40 torch ops
    that save every intermediate;
  * random draws (sample jitter, sigma noise) come from the counter-based generator keyed by
    ``loner_amd.random.next_key()`` rather than torch.rand/randn, so they are reproducible
    and regenerated in the backward instead of stored;
  * ``inference(netchunk > 0)`` evaluates each chunk once (the reference re-evaluates the whole
    input per chunk, rendering_tcnn.py:326-329; LONER configures netchunk = 0);
  * the DEBUG NaN/inf scan (rendering_tcnn.py:419-424) costs one host sync per key and is only
    run when ``DEBUG`` is True, as in the reference.
"""
import torch

from . import _lib as L
from . import random as R

_STRATEGY = {"default": 0, "adjusted": 1}


def _rays13(rays_d, far, rays_o=None):
    """The kernels read direction and far from the (R, 13) ray layout (ray_utils.py:314-317)."""
    n = rays_d.shape[0]
    r = torch.zeros(n, 13, dtype=torch.float32, device=rays_d.device)
    if rays_o is not None:
        r[:, 0:3] = rays_o
    r[:, 3:6] = rays_d
    if far is not None:
        r[:, 12] = far.reshape(n)
    return r


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigmas, z_vals, rays13, strategy, noise_std, key):
        n, s = z_vals.shape
        dev = z_vals.device
        sig = sigmas.detach().float().contiguous()
        z = z_vals.detach().float().contiguous()
        w = torch.empty(n, s, dtype=torch.float32, device=dev)
        depth = torch.empty(n, dtype=torch.float32, device=dev)
        opacity = torch.empty(n, dtype=torch.float32, device=dev)
        var = torch.empty(n, dtype=torch.float32, device=dev)
        rays13 = rays13.detach().contiguous()
        L.call("lnr_composite", rays13, z, sig, n, s, strategy, noise_std, None, key, 0, w, depth, opacity, var,
               L.stream(dev))
        ctx.save_for_backward(sig, z, rays13)
        ctx.cfg = (strategy, noise_std, key, sigmas.dtype)
        return w, depth, opacity, var

    @staticmethod
    def backward(ctx, g_w, g_depth, g_opacity, g_var):
        sig, z, rays13 = ctx.saved_tensors
        strategy, noise_std, key, dtype = ctx.cfg
        n, s = z.shape
        d_sigma = torch.empty(n, s, dtype=torch.float32, device=z.device)

        def c(t):
            return None if t is None else t.float().contiguous()

        want_ray = ctx.needs_input_grad[2]
        d_ray = torch.empty(n, 2, dtype=torch.float32, device=z.device) if want_ray else None
        L.call("lnr_composite_bwd", rays13, z, sig, n, s, strategy, noise_std, None, key, 0, c(g_w), c(g_depth),
               c(g_opacity), c(g_var), d_sigma, d_ray, L.stream(z.device))
        d_rays13 = None
        if want_ray:
            # rays that require grad (poses under optimisation): the deltas' direction norm
            # (rendering_tcnn.py:248) and the far term of the default depth (:274-278)
            d = rays13[:, 3:6]
            d_rays13 = torch.zeros_like(rays13)
            d_rays13[:, 3:6] = d_ray[:, 0:1] * d / d.norm(dim=-1, keepdim=True)
            d_rays13[:, 12] = d_ray[:, 1]
        return d_sigma.to(dtype), None, d_rays13, None, None, None


def _composite(raw, z_vals, rays_d, raw_noise_std, white_bkgd, sigma_only, num_colors, far, ret_var, strategy,
               softplus, rays_o=None):
    if softplus:
        raise NotImplementedError("loner_amd: softplus density activation is not implemented (LONER uses relu)")
    n, s = z_vals.shape
    if s < 2 or s > 4096:
        raise ValueError(f"loner_amd: N_samples={s} outside [2, 4096]")
    sigmas = raw[..., 0] if sigma_only else raw[..., num_colors]
    noise_std = float(raw_noise_std) if (raw_noise_std > 0 and strategy == 0) else 0.0
    key = R.next_key() if noise_std > 0 else 0
    weights, depth, opacity, var = _Composite.apply(sigmas, z_vals, _rays13(rays_d, far, rays_o), strategy,
                                                    noise_std, key)
    if sigma_only:
        rgb = torch.tensor([-1.])
    else:
        rgb = torch.sum(weights.unsqueeze(-1) * raw[..., :num_colors], -2)
        if white_bkgd:
            rgb = rgb + 1 - weights.sum(-1, keepdim=True)
    return rgb, depth, weights, opacity, (var if ret_var else None)


def raw2outputs(raw, z_vals, rays_d, raw_noise_std=0, white_bkgd=False, sigma_only=False, num_colors=3,
                softplus=False, far=None, ret_var=False):
    """rendering_tcnn.py:219-295: (rgb, depth, weights, opacity, variance|None)."""
    return _composite(raw, z_vals, rays_d, raw_noise_std, white_bkgd, sigma_only, num_colors, far, ret_var, 0,
                      softplus)


def raw2outputs_adjusted(raw, z_vals, rays_o, rays_d, raw_noise_std=0, white_bkgd=False, sigma_only=False,
                         num_colors=3, softplus=False, far=None, ret_var=True):
    """rendering_tcnn.py:70-214: depth = z at the first T <= 0.5 crossing (0 if none); noise is
    forced off (:104); the peak/prominence overrides of :136-199 write into copies and have no
    effect in the reference, so they are not reproduced."""
    return _composite(raw, z_vals, rays_d, 0.0, white_bkgd, sigma_only, num_colors, None, ret_var, 1, softplus,
                      rays_o)


def inference(model, xyz_, dir_, sigma_only=False, netchunk=32768, detach_sigma=True, meshing=False):
    """rendering_tcnn.py:297-335."""
    n_rays, n_samples = xyz_.shape[0:2]
    xyz_ = xyz_.reshape(-1, 3).contiguous()
    if sigma_only:
        dir_ = None
    else:
        dir_ = torch.repeat_interleave(dir_, repeats=n_samples, dim=0).contiguous()
    B = xyz_.shape[0]
    if netchunk == 0 or netchunk >= B:
        out = model(xyz_, dir_, sigma_only, detach_sigma)
    else:
        out = torch.cat([model(xyz_[i:i + netchunk], None if dir_ is None else dir_[i:i + netchunk], sigma_only,
                               detach_sigma) for i in range(0, B, netchunk)], 0)
    if meshing:
        return out
    return out.view(n_rays, n_samples, -1)


def render_rays(rays, ray_sampler, nerf_model, ray_range, scale_factor, N_samples=64, retraw=False, perturb=0,
                white_bkgd=False, raw_noise_std=0., netchunk=32768, num_colors=3, sigma_only=False, DEBUG=True,
                detach_sigma=True, return_variance=False, render_strategy='default'):
    """rendering_tcnn.py:340-425 — same arguments, same result keys."""
    if render_strategy not in _STRATEGY:
        raise ValueError(f"Unknown render strategy: {render_strategy}")
    rays_o, rays_d = rays[:, 0:3], rays[:, 3:6]
    viewdirs = rays[:, 6:9]
    far = rays[:, -1:]
    z_vals = ray_sampler.get_samples(rays, N_samples, perturb)
    xyz_samples = rays_o.unsqueeze(1) + rays_d.unsqueeze(1) * z_vals.unsqueeze(2)
    raw = inference(nerf_model, xyz_samples, viewdirs, netchunk=netchunk, sigma_only=sigma_only,
                    detach_sigma=detach_sigma)
    if render_strategy == 'default':
        rgb, depth, weights, opacity, variance = raw2outputs(
            raw, z_vals, rays_d, raw_noise_std, white_bkgd, sigma_only=sigma_only, num_colors=num_colors, far=far,
            ret_var=return_variance)
    else:
        rgb, depth, weights, opacity, variance = raw2outputs_adjusted(
            raw, z_vals, rays_o, rays_d, raw_noise_std, white_bkgd, sigma_only=sigma_only, num_colors=num_colors,
            far=far, ret_var=return_variance)
    result = {'rgb_fine': rgb, 'depth_fine': depth, 'weights_fine': weights, 'opacity_fine': opacity}
    if return_variance:
        result["variance"] = variance
    if retraw:
        result['samples_fine'] = z_vals
        result['points_fine'] = xyz_samples
    if DEBUG:
        result['raw_fine'] = raw
        for k in result:
            if torch.isnan(result[k]).any() or torch.isinf(result[k]).any():
                print(f"! [Numerical Error] {k} contains nan or inf.")
    return result
