"""tiny-cuda-nn-compatible PyTorch modules backed by the loner_amd HIP library.

Drop-in for the three tcnn classes LONER constructs (src/models/nerf_tcnn.py:35-52):

    tcnn.NetworkWithInputEncoding(n_input_dims=3, n_output_dims=1, encoding_config, network_config)
    tcnn.Encoding(n_input_dims, encoding_config)
    tcnn.Network(n_input_dims, n_output_dims, network_config)

Same constructor dicts (passed verbatim from cfg/nerf_config/default_nerf_hash.yaml), one flat fp32
``params`` Parameter per module (network first, then encoding, as tcnn lays them out), ``dtype`` =
torch.half, ``n_input_dims`` / ``n_output_dims``, fp16 outputs, and a custom autograd Function
whose backward returns the parameter gradient and, when the input requires grad, the input gradient
(tcnn's dL/dx: joint pose + map optimisation differentiates the sample positions through the grid,
src/models/nerf_tcnn.py:63,68-71, src/mapping/optimizer.py:256-262).  Unsupported configurations raise
``RuntimeError`` at construction, like tcnn's CHECK_THROW; CPU inputs raise (there is no CPU path).

Implementation per configuration:
  * HashGrid (n_features_per_level = 2) encode / backward: HIP kernels (lnr_hashgrid_*), the
    table backward is the binned int64-fixed-point scatter, so gradients are
    deterministic; the input gradient is lnr_hashgrid_bwd's d_pos (one fixed-order sum per sample);
  * NetworkWithInputEncoding(HashGrid, FullyFusedMLP 64 neurons x 1 hidden layer, 1 output) — the
    LONER sigma field: HIP hash encode + MFMA sigma MLP (lnr_sigma_mlp_fwd/_bwd);
  * SphericalHarmonics (degree <= 4): HIP kernel forward; its input gradient (the polynomials'
    derivative) as torch ops on the GPU;
  * other FullyFusedMLP shapes (the colour head 48 -> 4x64 -> 3): fp16 GEMMs through hipBLASLt
    (torch.matmul), fp32 accumulate — a plain library GEMM, off the sigma hot path.

Numerics differ from tcnn v1.7 in the backward only in being more precise: tcnn scales the loss
by 128 and accumulates fp16; here gradients are fp32 (hash grid: fp32 records summed in int64
fixed point).  Parameter initialisation follows tcnn's rules (hash table U(-1e-4, 1e-4),
Xavier-uniform MLP layers) with a counter-based generator instead of tcnn's PCG32 — parity
unpinned (no tcnn in this image).
"""
import ctypes
import math

import torch
import torch.nn as nn

from . import _lib as L

__all__ = ["Encoding", "Network", "NetworkWithInputEncoding", "free_temporary_memory"]


def free_temporary_memory():
    """tcnn API; the HIP path holds no temporaries of its own (workspaces come from torch)."""
    torch.cuda.empty_cache()


def _next_multiple(v, m):
    return (v + m - 1) // m * m


def _fill_uniform(n, seed, lo, hi, device, start=0):
    out = torch.empty(n, dtype=torch.float32, device=device)
    if n:
        L.call("lnr_fill_uniform", out, n, seed & 0xFFFFFFFF, lo, hi, start, L.stream(device))
    return out


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("loner_amd.tcnn: no GPU visible; the HIP path has no CPU implementation")
    return torch.device("cuda", torch.cuda.current_device())


def _check_input(x, n_input_dims, who):
    if not x.is_cuda:
        raise RuntimeError(f"{who}: input must be a GPU tensor (the HIP path has no CPU implementation)")
    if x.dim() != 2 or x.shape[1] != n_input_dims:
        raise RuntimeError(f"{who}: expected input of shape (B, {n_input_dims}), got {tuple(x.shape)}")
    return x.float().contiguous()


# ----------------------------------------------------------------------------- hash grid
class _GridSpec:
    """HashGrid config -> lnr_grid_desc (tcnn v1.7 GridEncodingTemplated layout)."""

    def __init__(self, n_input_dims, cfg):
        otype = cfg.get("otype", "")
        if otype not in ("HashGrid", "Grid") or cfg.get("type", "Hash") != "Hash":
            raise RuntimeError(f"loner_amd.tcnn: encoding otype={otype!r} is not a hash grid")
        if n_input_dims != 3:
            raise RuntimeError("loner_amd.tcnn: HashGrid supports n_input_dims=3 only")
        self.n_levels = int(cfg.get("n_levels", 16))
        self.n_features = int(cfg.get("n_features_per_level", 2))
        self.log2_hashmap_size = int(cfg.get("log2_hashmap_size", 19))
        self.base_resolution = int(cfg.get("base_resolution", 16))
        self.per_level_scale = float(cfg.get("per_level_scale", 2.0))
        if cfg.get("interpolation", "Linear") != "Linear":
            raise RuntimeError("loner_amd.tcnn: HashGrid interpolation must be Linear")
        self.desc = L.grid_desc(self.n_levels, self.n_features, self.log2_hashmap_size, self.base_resolution,
                                self.per_level_scale)
        self.n_entries = int(self.desc.n_entries)
        self.n_params = self.n_entries * self.n_features
        self.n_output_dims = self.n_levels * self.n_features


def _grid_backward(spec, pos01, d_enc, n, want_table=True, table16=None):
    """d_enc (L, n, 2) fp32 level-major -> (d_table (n_params) fp32 or None, d_pos01 (n, 3) fp32 or None).
    The table gradient is the binned HIP backward; with ``table16`` (the forward's fp16 table) the input
    gradient dL/dpos01 is computed as well (tcnn returns it when the positions require grad)."""
    dev = pos01.device
    want_pos = table16 is not None
    d_table = torch.empty(spec.n_params, dtype=torch.float32, device=dev) if want_table else None  # overwritten
    d_pos = torch.empty(n, 3, dtype=torch.float32, device=dev) if want_pos else None
    if n == 0 or not (want_table or want_pos):
        return (d_table.zero_() if want_table else None), d_pos
    nbytes = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(spec.desc), n)) if want_table else 0
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev) if want_table else None
    L.call("lnr_hashgrid_bwd", ctypes.byref(spec.desc), pos01, n, d_enc, n, d_table, table16, d_pos, ws, nbytes, 0,
           L.stream(dev))
    return d_table, d_pos


def _grid_forward(spec, pos01, table16, n):
    enc = torch.empty(spec.n_levels, max(n, 1), dtype=torch.int32, device=pos01.device)
    if n:
        L.call("lnr_hashgrid_fwd", ctypes.byref(spec.desc), pos01, n, table16, enc, n, None, 0,
               L.stream(pos01.device))
    return enc


class _EncodingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pos01, params, spec):
        n = pos01.shape[0]
        table16 = params.detach().half().contiguous()
        enc = _grid_forward(spec, pos01, table16, n)
        out = torch.empty(n, spec.n_output_dims, dtype=torch.half, device=pos01.device)
        if n:
            L.call("lnr_enc_to_aos", enc, n, n, spec.n_levels, out, L.stream(pos01.device))
        ctx.spec = spec
        ctx.save_for_backward(pos01, table16)
        return out

    @staticmethod
    def backward(ctx, g):
        pos01, table16 = ctx.saved_tensors
        spec = ctx.spec
        n = pos01.shape[0]
        g = g.contiguous()
        d_enc = torch.empty(spec.n_levels, max(n, 1), 2, dtype=torch.float32, device=pos01.device)
        if n:
            g16 = g if g.dtype == torch.half else None
            g32 = g.float().contiguous() if g16 is None else None
            L.call("lnr_aos_grad_to_enc", g16, g32, n, spec.n_levels, d_enc, n, L.stream(pos01.device))
        d_table, d_pos = _grid_backward(spec, pos01, d_enc, n, want_table=ctx.needs_input_grad[1],
                                        table16=table16 if ctx.needs_input_grad[0] else None)
        return d_pos, d_table, None


def _sh_basis(d01, degree):
    """tcnn SphericalHarmonics basis (degree <= 4) of directions in [0,1]^3 as differentiable torch ops; only
    its derivative is used (the forward values come from lnr_sh_encode)."""
    x, y, z = (d01 * 2 - 1).unbind(-1)
    out = [torch.full_like(x, 0.28209479177387814)]
    if degree > 1:
        out += [-0.48860251190291987 * y, 0.48860251190291987 * z, -0.48860251190291987 * x]
    if degree > 2:
        out += [1.0925484305920792 * x * y, -1.0925484305920792 * y * z, 0.94617469575755997 * z * z - 0.31539156525251999,
                -1.0925484305920792 * x * z, 0.54627421529603959 * (x * x - y * y)]
    if degree > 3:
        out += [0.59004358992664352 * y * (-3 * x * x + y * y), 2.8906114426405538 * x * y * z,
                0.45704579946446572 * y * (1 - 5 * z * z), 0.3731763325901154 * z * (5 * z * z - 3),
                0.45704579946446572 * x * (1 - 5 * z * z), 1.4453057213202769 * z * (x * x - y * y),
                0.59004358992664352 * x * (-x * x + 3 * y * y)]
    return torch.stack(out, -1)


class _SHFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dir01, degree):
        n = dir01.shape[0]
        out = torch.empty(n, degree * degree, dtype=torch.half, device=dir01.device)
        L.call("lnr_sh_encode", dir01, n, degree, out, L.stream(dir01.device))
        ctx.degree = degree
        ctx.save_for_backward(dir01)
        return out

    @staticmethod
    def backward(ctx, g):
        # tcnn's SphericalHarmonics input gradient (the polynomials' derivative, fp32); the encoding has no
        # parameters.  A 16-term polynomial on (n, 3): plain torch ops on the GPU, off the sigma path.
        (dir01,) = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None
        with torch.enable_grad():
            d = dir01.detach().float().requires_grad_()
            (gd,) = torch.autograd.grad(_sh_basis(d, ctx.degree), d, g.float())
        return gd, None


class Encoding(nn.Module):
    """tcnn.Encoding(n_input_dims, encoding_config, seed=1337, dtype=torch.half)."""

    def __init__(self, n_input_dims, encoding_config, seed=1337, dtype=torch.half, device=None):
        super().__init__()
        if dtype not in (torch.half, None):
            raise RuntimeError("loner_amd.tcnn: only fp16 encodings are supported")
        self.n_input_dims = n_input_dims
        self.encoding_config = dict(encoding_config)
        self.seed = seed
        self.dtype = torch.half
        device = device or _default_device()
        otype = encoding_config.get("otype", "")
        if otype == "SphericalHarmonics":
            if n_input_dims != 3:
                raise RuntimeError("loner_amd.tcnn: SphericalHarmonics needs n_input_dims=3")
            self.degree = int(encoding_config.get("degree", 4))
            if not 1 <= self.degree <= 4:
                raise RuntimeError(f"loner_amd.tcnn: SphericalHarmonics degree {self.degree} not supported")
            self._spec = None
            self.n_output_dims = self.degree * self.degree
            self.params = nn.Parameter(torch.zeros(0, dtype=torch.float32, device=device))
        else:
            self._spec = _GridSpec(n_input_dims, encoding_config)
            self.n_output_dims = self._spec.n_output_dims
            # tcnn GridEncoding::initialize_params: U(-1e-4, 1e-4)
            self.params = nn.Parameter(_fill_uniform(self._spec.n_params, seed, -1e-4, 1e-4, device))

    def forward(self, x):
        x = _check_input(x, self.n_input_dims, "loner_amd.tcnn.Encoding")
        if self._spec is None:
            return _SHFn.apply(x, self.degree)
        return _EncodingFn.apply(x, self.params, self._spec)

    def extra_repr(self):
        return f"n_input_dims={self.n_input_dims}, n_output_dims={self.n_output_dims}, config={self.encoding_config}"


# ----------------------------------------------------------------------------- networks
_ACT = {"None": None, "ReLU": torch.relu, "Sigmoid": torch.sigmoid, "Exponential": torch.exp,
        "Softplus": nn.functional.softplus, "Tanh": torch.tanh}


class _MLPSpec:
    """FullyFusedMLP / CutlassMLP config: tcnn pads the input to a multiple of 16 and the output
    to 16; layer l is (out_l, in_l) row-major, flat in layer order; no biases."""

    def __init__(self, n_input_dims, n_output_dims, cfg):
        otype = cfg.get("otype", "FullyFusedMLP")
        if otype not in ("FullyFusedMLP", "CutlassMLP", "MLP"):
            raise RuntimeError(f"loner_amd.tcnn: network otype={otype!r} not supported")
        self.activation = cfg.get("activation", "ReLU")
        self.output_activation = cfg.get("output_activation", "None")
        for a in (self.activation, self.output_activation):
            if a not in _ACT:
                raise RuntimeError(f"loner_amd.tcnn: activation {a!r} not supported")
        self.n_neurons = int(cfg.get("n_neurons", 64))
        self.n_hidden_layers = int(cfg.get("n_hidden_layers", 2))
        if otype == "FullyFusedMLP" and self.n_neurons not in (16, 32, 64, 128):
            raise RuntimeError(f"FullyFusedMLP only supports 16, 32, 64, and 128 neurons, got {self.n_neurons}")
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.in_pad = _next_multiple(n_input_dims, 16)
        self.out_pad = _next_multiple(n_output_dims, 16)
        dims = [self.in_pad] + [self.n_neurons] * self.n_hidden_layers + [self.out_pad]
        self.shapes = [(dims[i + 1], dims[i]) for i in range(len(dims) - 1)]
        self.n_params = sum(o * i for o, i in self.shapes)

    def init_params(self, seed, device):
        """Xavier-uniform per layer over the padded (fan_out, fan_in) shape."""
        chunks = []
        for k, (o, i) in enumerate(self.shapes):
            a = math.sqrt(6.0 / (o + i))
            chunks.append(_fill_uniform(o * i, seed + k, -a, a, device))
        return torch.cat(chunks) if chunks else torch.zeros(0, device=device)

    def is_loner_sigma(self):
        return (self.activation == "ReLU" and self.output_activation == "None" and self.n_neurons == 64
                and self.n_hidden_layers == 1 and self.n_input_dims == 32 and self.n_output_dims == 1)

    def forward_torch(self, x16, params):
        """Generic MLP as fp16 GEMMs (hipBLASLt via torch.matmul, fp32 accumulate)."""
        h = x16
        if self.in_pad != h.shape[1]:
            h = nn.functional.pad(h, (0, self.in_pad - h.shape[1]))
        off = 0
        w16 = params.half()
        for k, (o, i) in enumerate(self.shapes):
            W = w16[off:off + o * i].view(o, i)
            off += o * i
            h = h @ W.t()
            act = _ACT[self.activation if k < len(self.shapes) - 1 else self.output_activation]
            if act is not None:
                h = act(h)
        return h[:, :self.n_output_dims]


class Network(nn.Module):
    """tcnn.Network(n_input_dims, n_output_dims, network_config, seed=1337)."""

    def __init__(self, n_input_dims, n_output_dims, network_config, seed=1337, device=None):
        super().__init__()
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.network_config = dict(network_config)
        self.seed = seed
        self.dtype = torch.half
        self._spec = _MLPSpec(n_input_dims, n_output_dims, network_config)
        self.params = nn.Parameter(self._spec.init_params(seed, device or _default_device()))

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("loner_amd.tcnn.Network: input must be a GPU tensor")
        if x.dim() != 2 or x.shape[1] != self.n_input_dims:
            raise RuntimeError(f"loner_amd.tcnn.Network: expected (B, {self.n_input_dims}), got {tuple(x.shape)}")
        return self._spec.forward_torch(x.half(), self.params)


class _SigmaFieldFn(torch.autograd.Function):
    """HashGrid(F=2) + FullyFusedMLP(32 -> 64 ReLU -> 1): the LONER sigma field, all HIP."""

    @staticmethod
    def forward(ctx, pos01, params, spec):
        n = pos01.shape[0]
        dev = pos01.device
        p16 = params.detach().half().contiguous()
        w16 = p16[:L.SIGMA_MLP_PARAMS]
        table16 = p16[L.SIGMA_MLP_PARAMS:]
        enc = _grid_forward(spec, pos01, table16, n)
        sigma = torch.empty(n, dtype=torch.half, device=dev)
        if n:
            L.call("lnr_sigma_mlp_fwd", w16, enc, n, n, sigma, L.stream(dev))
        ctx.spec = spec
        ctx.save_for_backward(pos01, p16, enc)
        return sigma.view(n, 1)

    @staticmethod
    def backward(ctx, g):
        pos01, p16, enc = ctx.saved_tensors
        spec = ctx.spec
        n = pos01.shape[0]
        dev = pos01.device
        w16, table16 = p16[:L.SIGMA_MLP_PARAMS], p16[L.SIGMA_MLP_PARAMS:]
        d_w = torch.zeros(L.SIGMA_MLP_PARAMS, dtype=torch.float32, device=dev)
        d_enc = torch.empty(spec.n_levels, max(n, 1), 2, dtype=torch.float32, device=dev)
        if n:
            ds = g.reshape(n).float().contiguous()
            ws = torch.empty(int(L.lib().lnr_dw_workspace_words(n)), dtype=torch.float32, device=dev)
            L.call("lnr_sigma_mlp_bwd", w16, enc, n, n, ds, d_enc, d_w, ws, L.stream(dev))
        d_table, d_pos = _grid_backward(spec, pos01, d_enc, n, want_table=ctx.needs_input_grad[1],
                                        table16=table16 if ctx.needs_input_grad[0] else None)
        d_params = torch.cat([d_w, d_table]) if ctx.needs_input_grad[1] else None
        return d_pos, d_params, None


class NetworkWithInputEncoding(nn.Module):
    """tcnn.NetworkWithInputEncoding(n_input_dims, n_output_dims, encoding_config, network_config)."""

    def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=1337, device=None):
        super().__init__()
        device = device or _default_device()
        self.n_input_dims = n_input_dims
        self.n_output_dims = n_output_dims
        self.encoding_config = dict(encoding_config)
        self.network_config = dict(network_config)
        self.seed = seed
        self.dtype = torch.half
        self._grid = _GridSpec(n_input_dims, encoding_config)
        self._mlp = _MLPSpec(self._grid.n_output_dims, n_output_dims, network_config)
        self._fused = self._mlp.is_loner_sigma() and self._grid.n_features == 2
        # tcnn layout: network parameters first, then the encoding's.  Seeds: layer k <- seed + k,
        # table <- seed + n_layers (identical to loner_amd.step.FieldState for the sigma field)
        w = self._mlp.init_params(seed, device)
        t = _fill_uniform(self._grid.n_params, seed + len(self._mlp.shapes), -1e-4, 1e-4, device)
        self.params = nn.Parameter(torch.cat([w, t]))
        self.n_network_params = self._mlp.n_params

    def forward(self, x):
        x = _check_input(x, self.n_input_dims, "loner_amd.tcnn.NetworkWithInputEncoding")
        if self._fused:
            return _SigmaFieldFn.apply(x, self.params, self._grid)
        nw = self.n_network_params
        enc = _EncodingFn.apply(x, self.params[nw:], self._grid)
        return self._mlp.forward_torch(enc, self.params[:nw])
