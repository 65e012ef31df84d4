"""Ray samplers with the reference's interface (src/models/ray_sampling.py:18-92), one HIP
kernel each (lnr_sample_uniform / lnr_sample_ogm: linspace + jitter, occupancy-grid trilinear
lookup, inverse-CDF importance sampling and the per-ray sort, all in registers/LDS).

Jitter and inverse-CDF variates come from the counter-based generator (loner_amd.random) instead
of torch.rand; everything else follows the reference op for op (oracle/render.py restates it and
tests/golden pins it against the reference's own functions)."""
import torch

from . import _lib as L
from . import random as R


def _check_rays(rays, who):
    if not rays.is_cuda:
        raise RuntimeError(f"{who}: rays must be a GPU tensor (the HIP path has no CPU implementation)")
    if rays.dim() != 2 or rays.shape[1] < 13:
        raise RuntimeError(f"{who}: expected rays (N, 13), got {tuple(rays.shape)}")
    return rays.float().contiguous()


class UniformRaySampler():
    def __init__(self):
        print('Initializing a uniform ray sampler')

    def get_samples(self, rays, N_samples, perturb):
        rays = _check_rays(rays, "UniformRaySampler")
        n = rays.shape[0]
        z = torch.empty(n, N_samples, dtype=torch.float32, device=rays.device)
        key = R.next_key() if perturb > 0 else 0
        L.call("lnr_sample_uniform", rays, n, N_samples, float(perturb), None, key, 0, z, None, L.stream(rays.device))
        return z


class OccGridRaySampler():
    def __init__(self):
        self._occ_gamma = None

    def update_occ_grid(self, occ_gamma):
        self._occ_gamma = occ_gamma

    def get_samples(self, rays, N_samples, perturb):
        rays = _check_rays(rays, "OccGridRaySampler")
        if self._occ_gamma is None:
            raise RuntimeError("OccGridRaySampler: update_occ_grid() has not been called")
        occ = self._occ_gamma.detach()
        res = occ.shape[-1]
        if occ.numel() != res ** 3 or not occ.is_cuda:
            raise RuntimeError(f"OccGridRaySampler: expected a cubic GPU grid, got {tuple(occ.shape)}")
        occ = occ.float().contiguous()
        n = rays.shape[0]
        z = torch.empty(n, N_samples, dtype=torch.float32, device=rays.device)
        key = R.next_key()
        L.call("lnr_sample_ogm", rays, n, N_samples, occ, res, float(perturb), None, None, key, 0, z,
               None, L.stream(rays.device))
        return z
