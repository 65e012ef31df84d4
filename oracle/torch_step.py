"""Pure-PyTorch CPU restatement of one sigma-field optimiser step — TEST INFRASTRUCTURE ONLY.

This is the ``cpu_baseline`` leg of ``bench.py`` ("the build's pure-PyTorch
restatement ... torch.set_num_threads(os.cpu_count()) ... forward + backward + Adam"): the
reference's own torch step with tiny-cuda-nn replaced by torch ops, run on all host threads.
It follows the same code path as oracle/step.py (the parity oracle), in fp32 torch with autograd:
  sampler     OccGridRaySampler.get_samples + OccupancyGridModel.interpolate + sample_pdf
              (src/models/ray_sampling.py:53-92, src/models/model_tcnn.py:126-134,
              src/models/rendering_tcnn.py:19-68) with torch.rand draws
  sigma field tcnn v1.7 HashGrid (oracle/hashgrid.py layout) + 32->64->1 MLP, fp16 weights
              upcast, fp32 math (src/models/nerf_tcnn.py:35-38,59-81)
  compositing raw2outputs (rendering_tcnn.py:219-295), noise ~ N(0, 1)
  loss        Optimizer.compute_loss LiDAR branch (src/mapping/optimizer.py:701-859)
  update      torch autograd backward + torch.optim.Adam (optimizer.py:450,460)
It is a timing baseline, not the parity checker: its draws come from torch's generator, and its
MLP does not round activations to fp16.  Never imported by the product path.
"""
import math

import torch

from . import hashgrid as ohg

_PRIMES = (1, 2654435761, 805459861)


class TorchField:
    def __init__(self, n_levels=16, log2_hashmap_size=18, base_resolution=16, table_init=1e-4, seed=0, occ_res=100):
        g = torch.Generator().manual_seed(seed)
        self.layout = ohg.GridLayout(n_levels, 2, log2_hashmap_size, base_resolution)
        self.table = ((torch.rand(self.layout.n_entries, 2, generator=g) * 2 - 1) * table_init).requires_grad_()
        a0, a1 = math.sqrt(6.0 / 96), math.sqrt(6.0 / 80)
        self.w0 = ((torch.rand(64, 32, generator=g) * 2 - 1) * a0).requires_grad_()
        self.w1 = ((torch.rand(16, 64, generator=g) * 2 - 1) * a1).requires_grad_()
        self.occ = torch.zeros(1, 1, occ_res, occ_res, occ_res)
        self.opt = torch.optim.Adam([self.w0, self.w1, self.table], lr=0.01)
        lay = self.layout
        self.hashed = []
        for l in range(lay.n_levels):
            stride = 1
            for _ in range(3):
                if stride > lay.sizes[l]:
                    break
                stride *= lay.resolutions[l]
            self.hashed.append(stride > lay.sizes[l])

    def encode(self, pos01):
        lay, out = self.layout, []
        for l in range(lay.n_levels):
            p = pos01 * float(lay.scales[l]) + 0.5
            cell = torch.floor(p)
            frac = p - cell
            ci = cell.long()
            res, size, off = lay.resolutions[l], lay.sizes[l], lay.offsets[l]
            acc = 0.0
            for k in range(8):
                b = torch.tensor([(k >> d) & 1 for d in range(3)])
                c = ci + b
                if self.hashed[l]:
                    idx = (c[:, 0] * _PRIMES[0]) ^ ((c[:, 1] * _PRIMES[1]) & 0xFFFFFFFF) ^ ((c[:, 2] * _PRIMES[2]) & 0xFFFFFFFF)
                    idx = (idx & 0xFFFFFFFF) % size
                else:
                    idx = (c[:, 0] + c[:, 1] * res + c[:, 2] * res * res) % size
                w = torch.where(b.bool(), frac, 1 - frac).prod(-1, keepdim=True)
                acc = acc + w * self.table[off + idx]
            out.append(acc)
        return torch.cat(out, -1)

    def sigma(self, pos01):
        h = torch.relu(self.encode(pos01) @ self.w0.t())
        return (h @ self.w1.t())[:, :1]


def sample_ogm(field, rays, S, perturb=1.0):
    """OccGridRaySampler.get_samples (ray_sampling.py:53-92) in torch; perturb 1 = training (jitter)."""
    with torch.no_grad():
        R, H = rays.shape[0], S // 2
        near, far = rays[:, -2:-1], rays[:, -1:]
        t = torch.linspace(0, 1, H)
        z = near * (1 - t) + far * t
        mid = 0.5 * (z[:, 1:] + z[:, :-1])
        upper, lower = torch.cat([mid, z[:, -1:]], -1), torch.cat([z[:, :1], mid], -1)
        z = lower + (upper - lower) * torch.rand(R, H) if perturb else z
        pts = rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]
        logits = torch.nn.functional.grid_sample(field.occ, pts.reshape(1, 1, R, H, 3), align_corners=False)
        p = torch.sigmoid(logits.reshape(R, H))
        p = 2 * (p.clamp(0.5, 1.0) - 0.5)
        bins, w = 0.5 * (z[:, 1:] + z[:, :-1]), p[:, 1:-1] + 1e-5
        pdf = w / w.sum(-1, keepdim=True)
        cdf = torch.cat([torch.zeros(R, 1), torch.cumsum(pdf, -1)], -1)
        u = torch.rand(R, H).contiguous()
        inds = torch.searchsorted(cdf, u, right=True)
        below, above = (inds - 1).clamp(min=0), inds.clamp(max=cdf.shape[-1] - 1)
        c0, c1 = cdf.gather(1, below), cdf.gather(1, above)
        b0, b1 = bins.gather(1, below), bins.gather(1, above)
        den = c1 - c0
        den = torch.where(den < 1e-5, torch.ones_like(den), den)
        zi = b0 + (u - c0) / den * (b1 - b0)
        return torch.sort(torch.cat([z, zi], -1), -1)[0]


def train_step(field, rays, depth_gt, scale, cfg, global_step, S=512):
    """One optimiser step; returns the loss (float)."""
    R = rays.shape[0]
    z = sample_ogm(field, rays, S)
    xyz = rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]
    sig = field.sigma(((xyz + 1) / 2).reshape(-1, 3)).reshape(R, S)
    d = torch.cat([z[:, 1:] - z[:, :-1], torch.full((R, 1), 1e10)], -1) * rays[:, 3:6].norm(dim=-1, keepdim=True)
    alpha = 1 - torch.exp(-d * torch.relu(sig + torch.randn(R, S)))
    T = torch.cumprod(torch.cat([torch.ones(R, 1), 1 - alpha + 1e-10], -1), -1)[:, :-1]
    w = alpha * T
    far = rays[:, -1:]
    depth = (w * z).sum(-1) + (1 - w.sum(-1)) * far[:, 0]
    opacity = w.sum(-1)
    # compute_loss (optimizer.py:718-844), L1_JS / L2_JS
    s, g = z * scale, depth_gt.reshape(-1, 1) * scale
    opaque = (depth_gt > 0) & ~(depth_gt > far[0, 0])
    wsum = w.sum(1, keepdim=True)
    mean = (s * w).sum(1, keepdim=True) / (wsum + 1e-10)
    std = (((s - mean) ** 2 * w).sum(1, keepdim=True) / (wsum + 1e-10) + 1e-10).sqrt()
    with torch.no_grad():
        s1 = torch.full_like(g, cfg["min_depth_eps"] / 3)
        mm, sm = 0.5 * (g + mean), 0.5 * (s1 ** 2 + std ** 2).sqrt()
        kl = lambda m1, a, m2, b: torch.log(b / a) + (a ** 2 + (m1 - m2) ** 2) / (2 * b ** 2) - 0.5  # noqa: E731
        js = 0.5 * kl(g, s1, mm, sm) + 0.5 * kl(mean, std, mm, sm)
        js = torch.where(js < cfg["JS_loss"]["min_js_score"], torch.zeros_like(js), js)
        js = js.clamp(max=cfg["JS_loss"]["max_js_score"])
        eps = cfg["min_depth_eps"] * (1 + cfg["JS_loss"]["alpha"] * js)
        sg = eps / 9
        x = (s - g) / sg
        norm = 0.5 * (torch.erf(eps / sg / math.sqrt(2)) - torch.erf(-eps / sg / math.sqrt(2)))
        wgt = torch.exp(-0.5 * x ** 2) / math.sqrt(2 * math.pi) / sg / norm
        wgt = torch.where(((s - (g - eps)) > 0) & (((g + eps) - s) > 0), wgt, torch.zeros_like(wgt))
        wgt = wgt / (wgt.sum(1, keepdim=True) + 1e-6)
        wgt[~opaque] = 0
    lam = cfg["los_lambda"]
    if cfg.get("decay_los_lambda"):
        lam = max(lam * cfg["los_lambda_decay_rate"] ** ((global_step + 1) / cfg["los_lambda_decay_steps"]),
                  cfg["min_los_lambda"])
    dl = ((depth * scale - g[:, 0])[opaque] ** 2).mean()
    los = (w - wgt).abs().mean() if cfg["loss_selection"] == "L1_JS" else ((w - wgt) ** 2).mean()
    op = (opacity[opaque] - 1).abs().mean()
    loss = cfg["depthloss_lambda"] * dl + lam * los + op
    field.opt.zero_grad(set_to_none=True)
    loss.backward()
    field.opt.step()
    return float(loss.detach())


def render_step(field, rays, S=2048):
    """Model.forward(testing=True) for the sigma head in torch, no autograd (the C3 CPU baseline):
    OGM samples without jitter (random importance draws), the sigma field, peak ("adjusted")
    compositing (rendering_tcnn.py:70-214: depth at the first sample with T <= 0.5).  Returns the depths."""
    with torch.no_grad():
        R = rays.shape[0]
        z = sample_ogm(field, rays, S, perturb=0.0)
        xyz = rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]
        sig = field.sigma(((xyz + 1) / 2).reshape(-1, 3)).reshape(R, S)
        d = torch.cat([z[:, 1:] - z[:, :-1], torch.full((R, 1), 1e10)], -1) * rays[:, 3:6].norm(dim=-1, keepdim=True)
        alpha = 1 - torch.exp(-d * torch.relu(sig))
        T = torch.cumprod(torch.cat([torch.ones(R, 1), 1 - alpha + 1e-10], -1), -1)
        hit = (T[:, 1:] <= 0.5) & (T[:, :-1] > 0.5)
        return torch.where(hit.any(-1), z.gather(1, hit.float().argmax(-1, keepdim=True))[:, 0], torch.zeros(R))


def _sh4_torch(d):
    """tcnn SphericalHarmonics degree 4 of unit directions d (R,3) (oracle/render.py sh4, in torch)."""
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    return torch.stack([torch.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
                        -0.48860251190291987 * x, 1.0925484305920792 * x * y, -1.0925484305920792 * y * z,
                        0.94617469575755997 * z * z - 0.31539156525251999, -1.0925484305920792 * x * z,
                        0.54627421529603959 * (x * x - y * y), 0.59004358992664352 * y * (-3 * x * x + y * y),
                        2.8906114426405538 * x * y * z, 0.45704579946446572 * y * (1 - 5 * z * z),
                        0.3731763325901154 * z * (5 * z * z - 3), 0.45704579946446572 * x * (1 - 5 * z * z),
                        1.4453057213202769 * z * (x * x - y * y), 0.59004358992664352 * x * (-x * x + 3 * y * y)], 1)


class TorchColor:
    """The colour head (nerf_tcnn.py:40-52,80-95): HashGrid L16 T=2^19 + SH4 -> 48->64x4->3 MLP, sigmoid,
    with torch.optim.Adam over its parameters (optimizer.py:541-688)."""

    def __init__(self, n_hidden=4, table_init=1e-4, seed=1):
        g = torch.Generator().manual_seed(seed)
        self.grid = TorchField(log2_hashmap_size=19, table_init=table_init, seed=seed)
        dims = [48] + [64] * n_hidden + [16]
        self.mats = []
        for i in range(len(dims) - 1):
            a = math.sqrt(6.0 / (dims[i] + dims[i + 1]))
            self.mats.append(((torch.rand(dims[i + 1], dims[i], generator=g) * 2 - 1) * a).requires_grad_())
        self.opt = torch.optim.Adam([self.grid.table] + self.mats, lr=0.01)

    def color(self, pos01, dirs):
        h = torch.cat([self.grid.encode(pos01), _sh4_torch(dirs)], -1)
        for m in self.mats[:-1]:
            h = torch.relu(h @ m.t())
        return torch.sigmoid((h @ self.mats[-1].t())[:, :3])


def camera_step(field, color, rays, rgb_gt, S=512):
    """One colour-head iteration (optimizer.py:541-688,861-894) in torch: OGM samples, the frozen sigma
    field's compositing weights (no grad), the colour head on every sample, rgb = sum w c + 1 - sum w,
    L1 loss, autograd backward through the colour MLP and colour grid, Adam.  Returns the loss."""
    R = rays.shape[0]
    with torch.no_grad():
        z = sample_ogm(field, rays, S)
        xyz = rays[:, None, 0:3] + rays[:, None, 3:6] * z[..., None]
        pos = ((xyz + 1) / 2).reshape(-1, 3)
        sig = field.sigma(pos).reshape(R, S)
        d = torch.cat([z[:, 1:] - z[:, :-1], torch.full((R, 1), 1e10)], -1) * rays[:, 3:6].norm(dim=-1, keepdim=True)
        alpha = 1 - torch.exp(-d * torch.relu(sig + torch.randn(R, S)))
        T = torch.cumprod(torch.cat([torch.ones(R, 1), 1 - alpha + 1e-10], -1), -1)[:, :-1]
        w = alpha * T
    dirs = rays[:, 3:6].repeat_interleave(S, 0)
    col = color.color(pos, dirs).reshape(R, S, 3)
    rgb = (w[..., None] * col).sum(1) + (1 - w.sum(1, keepdim=True))
    loss = (rgb - rgb_gt).abs().mean()
    color.opt.zero_grad(set_to_none=True)
    loss.backward()
    color.opt.step()
    return float(loss.detach())
