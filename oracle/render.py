"""Sampling and volume rendering restated in numpy — TEST INFRASTRUCTURE ONLY.

Follows (file:line in /root/reference):
  linspace            torch.linspace as called in ``src/models/ray_sampling.py:26,59``
                      (symmetric formula used by torch's CUDA/CPU scalar kernels)
  uniform_samples     ``UniformRaySampler.get_samples``  ``src/models/ray_sampling.py:22-43``
  ogm_samples         ``OccGridRaySampler.get_samples``  ``src/models/ray_sampling.py:53-92``
  grid_sample_3d      ``OccupancyGridModel.interpolate`` ``src/models/model_tcnn.py:126-134``
                      (torch grid_sample 3-D, trilinear, align_corners=False, zero padding)
  sample_pdf          ``src/models/rendering_tcnn.py:19-68``
  raw2outputs         ``src/models/rendering_tcnn.py:219-295`` (default strategy)
  raw2outputs_adjusted``src/models/rendering_tcnn.py:70-214`` (peak rendering; the
                      prominence overrides write into advanced-index copies at :196-199 and
                      therefore have no effect — restated as the T<=0.5 crossing only)
  composite_backward  analytic gradient of raw2outputs w.r.t. sigma (the reference uses autograd
                      through cumprod, ``rendering_tcnn.py:262-266``)
Arrays are (R, S) fp32 unless noted; all arithmetic is fp32 in the reference's op order, with
reductions accumulated in fp64 and rounded once (torch CPU ``cumsum``/``cumprod`` accumulate in
double).
"""
import numpy as np

F32 = np.float32


def linspace(start, end, steps):
    start, end = F32(start), F32(end)
    step = F32((end - start) / F32(steps - 1))
    i = np.arange(steps)
    half = steps // 2
    lo = (start + step * i.astype(F32)).astype(F32)
    hi = (end - step * (steps - 1 - i).astype(F32)).astype(F32)
    return np.where(i < half, lo, hi).astype(F32)


def stratified(near, far, n, u_jitter=None):
    """near/far (R,1); returns (R,n) z, jittered inside midpoint intervals when u given."""
    t = linspace(0.0, 1.0, n)[None, :]
    z = (near * (F32(1.0) - t) + far * t).astype(F32)
    if u_jitter is not None:
        mid = (F32(0.5) * (z[:, :-1] + z[:, 1:])).astype(F32)
        upper = np.concatenate([mid, z[:, -1:]], -1)
        lower = np.concatenate([z[:, :1], mid], -1)
        z = (lower + (upper - lower) * u_jitter.astype(F32)).astype(F32)
    return z


def uniform_samples(rays, n, u_jitter=None):
    return stratified(rays[:, -2:-1], rays[:, -1:], n, u_jitter)


def grid_sample_3d(grid, pts):
    """grid (D,H,W) fp32, pts (...,3) in [-1,1] with x->W, y->H, z->D.  Returns (...) fp32."""
    D, H, W = grid.shape
    x, y, z = pts[..., 0].astype(F32), pts[..., 1].astype(F32), pts[..., 2].astype(F32)
    ix = (((x + F32(1)) * F32(W) - F32(1)) / F32(2)).astype(F32)
    iy = (((y + F32(1)) * F32(H) - F32(1)) / F32(2)).astype(F32)
    iz = (((z + F32(1)) * F32(D) - F32(1)) / F32(2)).astype(F32)
    out = np.zeros(x.shape, dtype=F32)
    for c, (wts, (cx, cy, cz)) in enumerate(zip(*_trilinear(ix, iy, iz))):
        ok = (cx >= 0) & (cx < W) & (cy >= 0) & (cy < H) & (cz >= 0) & (cz < D)
        v = np.where(ok, grid[np.clip(cz, 0, D - 1), np.clip(cy, 0, H - 1), np.clip(cx, 0, W - 1)], F32(0))
        out = (out + v * wts).astype(F32)
    return out


def _trilinear(ix, iy, iz):
    x0 = np.floor(ix).astype(np.int64)
    y0 = np.floor(iy).astype(np.int64)
    z0 = np.floor(iz).astype(np.int64)
    wx = [(F32(1) * (x0 + 1).astype(F32) - ix).astype(F32), (ix - x0.astype(F32)).astype(F32)]
    wy = [((y0 + 1).astype(F32) - iy).astype(F32), (iy - y0.astype(F32)).astype(F32)]
    wz = [((z0 + 1).astype(F32) - iz).astype(F32), (iz - z0.astype(F32)).astype(F32)]
    ws, cs = [], []
    for c in range(8):
        bx, by, bz = c & 1, (c >> 1) & 1, (c >> 2) & 1
        ws.append((wx[bx] * wy[by] * wz[bz]).astype(F32))
        cs.append((x0 + bx, y0 + by, z0 + bz))
    return ws, cs


def grid_sample_3d_backward(grid_shape, pts, g_out):
    """Scatter-add of trilinear weights * g_out into a (D,H,W) fp64 gradient."""
    D, H, W = grid_shape
    pts = pts.reshape(-1, 3)
    g_out = np.asarray(g_out, dtype=np.float64).reshape(-1)
    x, y, z = pts[:, 0].astype(F32), pts[:, 1].astype(F32), pts[:, 2].astype(F32)
    ix = (((x + F32(1)) * F32(W) - F32(1)) / F32(2)).astype(F32)
    iy = (((y + F32(1)) * F32(H) - F32(1)) / F32(2)).astype(F32)
    iz = (((z + F32(1)) * F32(D) - F32(1)) / F32(2)).astype(F32)
    g = np.zeros((D, H, W), dtype=np.float64)
    for wts, (cx, cy, cz) in zip(*_trilinear(ix, iy, iz)):
        ok = (cx >= 0) & (cx < W) & (cy >= 0) & (cy < H) & (cz >= 0) & (cz < D)
        np.add.at(g, (cz[ok], cy[ok], cx[ok]), wts[ok].astype(np.float64) * g_out[ok])
    return g


def sample_pdf(bins, weights, n_importance, u, eps=1e-5):
    """bins (R, M+1), weights (R, M), u (R, n) -> samples (R, n)."""
    R, M = weights.shape
    w = (weights + F32(eps)).astype(F32)
    pdf = (w / w.astype(np.float64).sum(-1, keepdims=True).astype(F32)).astype(F32)
    cdf = np.cumsum(pdf.astype(np.float64), -1).astype(F32)
    cdf = np.concatenate([np.zeros((R, 1), F32), cdf], -1)
    inds = np.stack([np.searchsorted(cdf[r], u[r], side="right") for r in range(R)])
    below = np.maximum(inds - 1, 0)
    above = np.minimum(inds, M)
    cdf0 = np.take_along_axis(cdf, below, 1)
    cdf1 = np.take_along_axis(cdf, above, 1)
    b0 = np.take_along_axis(bins, below, 1)
    b1 = np.take_along_axis(bins, above, 1)
    denom = (cdf1 - cdf0).astype(F32)
    denom = np.where(denom < F32(eps), F32(1), denom)
    return (b0 + (u - cdf0) / denom * (b1 - b0)).astype(F32)


def ogm_samples(rays, n, occ_grid, u_jitter, u_pdf):
    """OccGridRaySampler: n/2 stratified (jittered) + n/2 importance samples, sorted."""
    o, d = rays[:, 0:3], rays[:, 3:6]
    z = stratified(rays[:, -2:-1], rays[:, -1:], n // 2, u_jitter)
    pts = (o[:, None, :] + d[:, None, :] * z[:, :, None]).astype(F32)
    logits = grid_sample_3d(occ_grid, pts)
    probs = (F32(1) / (F32(1) + np.exp(-logits))).astype(F32)
    probs = (F32(2) * (np.clip(probs, F32(0.5), F32(1.0)) - F32(0.5))).astype(F32)
    mid = (F32(0.5) * (z[:, :-1] + z[:, 1:])).astype(F32)
    zi = sample_pdf(mid, probs[:, 1:-1], n // 2, u_pdf)
    return np.sort(np.concatenate([z, zi], -1), -1).astype(F32)


def _deltas(z, rays_d):
    dl = (z[:, 1:] - z[:, :-1]).astype(F32)
    dl = np.concatenate([dl, np.full((z.shape[0], 1), F32(1e10))], -1)
    nrm = np.sqrt((rays_d.astype(F32) ** 2).sum(-1, dtype=F32)).astype(F32)
    return (dl * nrm[:, None]).astype(F32)


def _transmittance(alphas):
    s = (F32(1) - alphas + F32(1e-10)).astype(F32)
    T = np.cumprod(np.concatenate([np.ones((alphas.shape[0], 1)), s.astype(np.float64)], -1), -1)[:, :-1]
    return T.astype(F32), s


def raw2outputs(sigma, z, rays_d, noise=None, far=None, ret_var=True):
    """Default compositing.  sigma (R,S) (fp16-valued), noise (R,S) N(0,1)*raw_noise_std or None."""
    sig = sigma.astype(F32)
    if noise is not None:
        sig = (sig + noise.astype(F32)).astype(F32)
    dl = _deltas(z, rays_d)
    alphas = (F32(1) - np.exp(-dl * np.maximum(sig, F32(0)))).astype(F32)
    T, _ = _transmittance(alphas)
    w = (alphas * T).astype(F32)
    wsum = w.astype(np.float64).sum(-1).astype(F32)
    opacity = wsum
    if far is not None:
        depth = ((w.astype(np.float64) * z).sum(-1) + (F32(1) - wsum).astype(np.float64) * far.reshape(-1)).astype(F32)
    else:
        depth = (w.astype(np.float64) * z).sum(-1).astype(F32)
    var = None
    if ret_var:
        var = (w.astype(np.float64) * ((depth[:, None] - z).astype(F32) ** 2)).sum(-1).astype(F32)
    return dict(weights=w, depth=depth, opacity=opacity, variance=var, alphas=alphas, T=T)


def raw2outputs_adjusted(sigma, z, rays_d, ret_var=True):
    """Peak rendering: depth = z_k at the first k with T_k <= 0.5 < T_{k-1} (T_{-1}=1), else 0.
    Noise is forced to zero (``rendering_tcnn.py:104``)."""
    sig = sigma.astype(F32)
    dl = _deltas(z, rays_d)
    alphas = (F32(1) - np.exp(-dl * np.maximum(sig, F32(0)))).astype(F32)
    T, _ = _transmittance(alphas)
    w = (alphas * T).astype(F32)
    opacity = w.astype(np.float64).sum(-1).astype(F32)
    Tsh = np.concatenate([np.ones((T.shape[0], 1), F32), T[:, :-1]], -1)
    hit = (~(T > F32(0.5))) & (Tsh > F32(0.5))
    depth = np.where(hit.any(-1), z[np.arange(z.shape[0]), hit.argmax(-1)], F32(0)).astype(F32)
    var = None
    if ret_var:
        var = (w.astype(np.float64) * ((depth[:, None] - z).astype(F32) ** 2)).sum(-1).astype(F32)
    return dict(weights=w, depth=depth, opacity=opacity, variance=var, alphas=alphas, T=T)


def composite_backward(sigma, z, rays_d, noise, far, g_w, g_depth, g_opacity, ray_grads=False):
    """d loss / d sigma (R,S) fp64 for the default strategy, given upstream gradients on the
    weights (R,S), the depth (R,) and the opacity (R,).  Uses the division-free suffix scan
    S_k = sum_{i>k} G_i a_i prod_{k<j<i} s_j,  dL/da_k = T_k (G_k - S_k).
    ``ray_grads``: also the render's gradient w.r.t. the ray, (dL/d|d|, dL/dfar) per ray: the deltas
    are dl * |d| (rendering_tcnn.py:248), so dL/d|d| = sum_k dL/da_k dl_k relu(sigma_k + n_k)
    exp(-delta_k relu(.)); the depth's far term (1 - sum w) far (:274-278) gives dL/dfar =
    g_depth (1 - sum w)."""
    f64 = np.float64
    sig = sigma.astype(f64) + (0.0 if noise is None else noise.astype(f64))
    dl = _deltas(z, rays_d).astype(f64)
    sr = np.maximum(sig, 0.0)
    a = 1.0 - np.exp(-dl * sr)
    s = 1.0 - a + 1e-10
    T = np.cumprod(np.concatenate([np.ones((a.shape[0], 1)), s], -1), -1)[:, :-1]
    G = np.asarray(g_w, f64) + np.asarray(g_depth, f64)[:, None] * (z.astype(f64) - np.asarray(far, f64).reshape(-1, 1)) \
        + np.asarray(g_opacity, f64)[:, None]
    R, S = a.shape
    Ssuf = np.zeros((R, S))
    for k in range(S - 2, -1, -1):
        Ssuf[:, k] = G[:, k + 1] * a[:, k + 1] + s[:, k + 1] * Ssuf[:, k + 1]
    dA = T * (G - Ssuf)
    with np.errstate(over="ignore", invalid="ignore"):
        dadsig = np.where(sig > 0, dl * np.exp(-dl * sr), 0.0)
    if not ray_grads:
        return dA * dadsig
    dlr = (z[:, 1:] - z[:, :-1]).astype(F32).astype(f64)
    dlr = np.concatenate([dlr, np.full((R, 1), 1e10)], -1)
    d_dnorm = (dA * dlr * sr * np.exp(-dl * sr)).sum(-1)
    w = a * T
    d_far = np.asarray(g_depth, f64) * (1.0 - w.sum(-1))
    return dA * dadsig, d_dnorm, d_far


def sh4(dir01):
    """tiny-cuda-nn SphericalHarmonics degree 4 of directions in [0,1]^3 (mapped back with 2x-1),
    fp64 arithmetic -> fp16 (the colour head's direction encoding, nerf_tcnn.py:43,86)."""
    x, y, z = (np.asarray(dir01, np.float32).astype(np.float64) * 2 - 1).T
    o = np.stack([np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
                  -0.48860251190291987 * x, 1.0925484305920792 * x * y, -1.0925484305920792 * y * z,
                  0.94617469575755997 * z * z - 0.31539156525251999, -1.0925484305920792 * x * z,
                  0.54627421529603959 * (x * x - y * y), 0.59004358992664352 * y * (-3 * x * x + y * y),
                  2.8906114426405538 * x * y * z, 0.45704579946446572 * y * (1 - 5 * z * z),
                  0.3731763325901154 * z * (5 * z * z - 3), 0.45704579946446572 * x * (1 - 5 * z * z),
                  1.4453057213202769 * z * (x * x - y * y), 0.59004358992664352 * x * (-x * x + 3 * y * y)], 1)
    return o.astype(np.float16)
