"""DecoupledNeRF on the HIP tcnn-compatible modules (mirrors src/models/nerf_tcnn.py:19-95).

Same constructor (cfg dict with pos_encoding_sigma / sigma_network / pos_encoding_intensity /
dir_encoding_intensity / intensity_network / enable_view_dependence, num_colors) and the same
``forward(pos, dir, sigma_only=False, detach_sigma=True)`` contract: pos in [-1,1]^3 -> sigma
(N,1) fp16 when sigma_only, else cat([sigmoid(colour), sigma]) (N, num_colors+1).

One deliberate deviation: the reference evaluates the colour hash grid (``_pos_encoding``,
2^19-entry table) before its ``sigma_only`` return (nerf_tcnn.py:64,80-81) and discards the
result; that dead encode is skipped here.  No output changes (the colour head is frozen on the
sigma path, so the discarded encode contributes no gradient either) — SURVEY.md §8(a) A8.
"""
import torch
import torch.nn as nn

from . import tcnn


class DecoupledNeRF(nn.Module):
    def __init__(self, cfg, num_colors=3, device=None):
        super().__init__()
        self._num_colors = num_colors
        self.cfg = cfg
        self._enable_view_dependence = cfg["enable_view_dependence"]
        self._model_sigma = tcnn.NetworkWithInputEncoding(n_input_dims=3, n_output_dims=1,
                                                          encoding_config=cfg["pos_encoding_sigma"],
                                                          network_config=cfg["sigma_network"], device=device)
        self._pos_encoding = tcnn.Encoding(3, cfg["pos_encoding_intensity"], device=device)
        if self._enable_view_dependence:
            self._dir_encoding = tcnn.Encoding(3, cfg["dir_encoding_intensity"], device=device)
            n_in = self._pos_encoding.n_output_dims + self._dir_encoding.n_output_dims
        else:
            self._dir_encoding = None
            n_in = self._pos_encoding.n_output_dims
        self._model_intensity = tcnn.Network(n_input_dims=n_in, n_output_dims=num_colors,
                                             network_config=cfg["intensity_network"], device=device)
        self._max_float = torch.finfo(self._model_intensity.dtype).max
        self._min_float = torch.finfo(self._model_intensity.dtype).min
        self._warn_infinite = True

    def forward(self, pos, dir, sigma_only=False, detach_sigma=True):
        pos = (pos + 1) / 2
        if detach_sigma and not sigma_only:
            with torch.no_grad():
                sigma = self._model_sigma(pos)[..., [0]]
        else:
            sigma = self._model_sigma(pos)[..., [0]]
        # nerf_tcnn.py:74-78.  The HIP sigma MLP already clamps non-finite outputs to +-65504
        # (lnr_sigma_mlp_fwd), so this only fires for the generic-network path; no host sync on
        # the fused path.
        if not self._model_sigma._fused and not torch.isfinite(sigma).all():
            if self._warn_infinite:
                print("Warning: Clipping infinite outputs. Will not warn about this again (but it will happen again)")
                self._warn_infinite = False
            sigma = sigma.nan_to_num(posinf=self._max_float, neginf=self._min_float)
        if sigma_only:
            return sigma
        h_x = self._pos_encoding(pos)
        dir = (dir + 1) / 2
        if self._enable_view_dependence:
            h_xd = torch.cat([h_x, self._dir_encoding(dir)], dim=-1)
            h_c = self._model_intensity(h_xd)
        else:
            h_c = self._model_intensity(h_x)
        color = torch.sigmoid(h_c)
        return torch.cat([color, sigma], dim=-1)
