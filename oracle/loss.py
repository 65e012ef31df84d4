"""LiDAR loss restated in numpy — TEST INFRASTRUCTURE ONLY.

Follows (file:line in /root/reference):
  los_lambda        ``src/mapping/optimizer.py:712-716`` (decay on global_step + 1)
  js_divergence     ``Optimizer.calculate_JS_divergence`` / ``calculate_KL_divergence``
                    ``src/mapping/optimizer.py:913-925``
  get_weights_gt    ``src/models/losses.py:29-51`` (truncated Gaussian, H(0)=0, row-normalised)
  lidar_loss        ``Optimizer.compute_loss`` LiDAR branch ``src/mapping/optimizer.py:718-844``
                    (L1_JS / L2_JS / L1_LOS / L2_LOS) with analytic gradients w.r.t. the rendered
                    weights, depth and opacity (eps is detached at ``:765``)
  logits_grad       ``get_logits_grad`` ``src/models/losses.py:54-62`` (OGM update)
"""
import math
import numpy as np

F32 = np.float32


def los_lambda(cfg, global_step):
    if cfg["decay_los_lambda"]:
        return max(cfg["los_lambda"] * (cfg["los_lambda_decay_rate"] ** ((global_step + 1) / cfg["los_lambda_decay_steps"])),
                   cfg["min_los_lambda"])
    return cfg["los_lambda"]


def los_depth_eps(cfg, iteration_idx):
    if cfg["decay_depth_eps"]:
        return max(cfg["depth_eps"] * (cfg["depth_eps_decay_rate"] ** (iteration_idx / cfg["depth_eps_decay_steps"])),
                   cfg["min_depth_eps"])
    return cfg["depth_eps"]


def _kl(m1, s1, m2, s2):
    v1 = (s1 * s1).astype(F32)
    v2 = (s2 * s2).astype(F32)
    a = np.log((s2 / s1).astype(F32)).astype(F32)
    num = (v1 + ((m1 - m2) ** 2).astype(F32)).astype(F32)
    return (a + (num / (F32(2) * v2)).astype(F32) - F32(0.5)).astype(F32)


def js_divergence(m1, s1, m2, s2):
    s1 = np.broadcast_to(np.asarray(s1, F32), np.shape(m1)).astype(F32)
    mm = (F32(0.5) * (m1 + m2)).astype(F32)
    sm = (F32(0.5) * np.sqrt((s1 ** 2 + s2 ** 2).astype(F32))).astype(F32)
    return (F32(0.5) * _kl(m1, s1, mm, sm) + F32(0.5) * _kl(m2, s2, mm, sm)).astype(F32)


def _erf(x):
    return np.vectorize(math.erf, otypes=[np.float64])(x)


def get_weights_gt(s, g, eps, norm=True):
    """s (R,S) metres, g (R,1) metres, eps (R,1) or scalar -> (R,S) fp32."""
    eps = np.broadcast_to(np.asarray(eps, F32), g.shape).astype(F32)
    sig = (eps / F32(9)).astype(F32)
    clip_a = (((g - eps) - g) / sig).astype(F32)
    clip_b = (((g + eps) - g) / sig).astype(F32)
    x = ((s - g) / sig).astype(F32)
    pdf = (F32(1.0 / np.sqrt(2 * np.pi)) * np.exp(F32(-0.5) * x ** 2)).astype(F32)
    cdf_b = (F32(0.5) * (F32(1) + _erf(clip_b / F32(np.sqrt(2))).astype(F32))).astype(F32)
    cdf_a = (F32(0.5) * (F32(1) + _erf(clip_a / F32(np.sqrt(2))).astype(F32))).astype(F32)
    wgt = (pdf / sig / (cdf_b - cdf_a)).astype(F32)
    inside = ((s - (g - eps)) > 0) & (((g + eps) - s) > 0)
    wgt = np.where(inside, wgt, F32(0)).astype(F32)
    if norm:
        wgt = (wgt / (wgt.astype(np.float64).sum(1, keepdims=True).astype(F32) + F32(1e-6))).astype(F32)
    return wgt


def lidar_loss(weights, z, depth, opacity, depth_gt, far, scale, cfg, global_step, iteration_idx=0,
               n_opaque=None, n_total=None, far_ref=None):
    """Returns dict(loss, terms..., g_w (R,S), g_depth (R,), g_opacity (R,), eps (R,), js (R,)).

    weights/z (R,S) fp32 normalised units, depth/opacity (R,), depth_gt/far (R,) normalised.
    cfg: the ``loss`` section of the model config (``cfg/model_config/default_model_config.yaml:40-60``).

    Data-parallel shards pass the GLOBAL normalisers: ``n_opaque`` (opaque rays
    over all shards), ``n_total`` (rays x samples over all shards) and ``far_ref`` (far bound of
    global ray 0, see below); the returned loss and gradients are then this shard's share, and
    summing them over shards gives the single-batch values.
    """
    R, S = weights.shape
    scale = F32(scale)
    w = weights.astype(F32)
    s = (z * scale).astype(F32)
    g = (depth_gt.reshape(-1, 1) * scale).astype(F32)
    # optimizer.py:724: ``(lidar_depths.view(-1,1) > far)[...,0]`` broadcasts (R,1) against (R,) and
    # keeps column 0, i.e. every ray is compared with the far bound of ray 0.  Reproduced as is.
    f0 = far.reshape(-1)[0] if far_ref is None else F32(far_ref)
    transparent = depth_gt.reshape(-1) > f0
    opaque = (depth_gt.reshape(-1) > 0) & ~transparent
    n_op = int(opaque.sum()) if n_opaque is None else int(n_opaque)
    n_rs = R * S if n_total is None else int(n_total)
    wsum = w.astype(np.float64).sum(1, keepdims=True).astype(F32)
    mean = ((s * w).astype(np.float64).sum(1, keepdims=True).astype(F32) / (wsum + F32(1e-10))).astype(F32)
    var = (((s - mean) ** 2 * w).astype(np.float64).sum(1, keepdims=True).astype(F32) / (wsum + F32(1e-10)) + F32(1e-10)).astype(F32)
    std = np.sqrt(var).astype(F32)
    eps_min = F32(cfg["min_depth_eps"])
    js = js_divergence(g, F32(eps_min / F32(3)), mean, std).reshape(-1)
    sel = cfg["loss_selection"]
    if sel in ("L1_JS", "L2_JS"):
        jsc = js.copy()
        jsc = np.where(jsc < F32(cfg["JS_loss"]["min_js_score"]), F32(0), jsc)
        jsc = np.where(jsc > F32(cfg["JS_loss"]["max_js_score"]), F32(cfg["JS_loss"]["max_js_score"]), jsc)
        eps = (eps_min * (F32(1) + F32(cfg["JS_loss"]["alpha"]) * jsc)).astype(F32)
    elif sel in ("L1_LOS", "L2_LOS"):
        eps = np.full(R, F32(los_depth_eps(cfg, iteration_idx)), F32)
    else:
        raise ValueError(f"Can't use unknown Loss {sel}")
    wgt = get_weights_gt(s, g, eps.reshape(-1, 1))
    wgt[~opaque, :] = 0
    dscaled = (depth.reshape(-1) * scale).astype(F32)
    lam = los_lambda(cfg, global_step)
    diff_d = (dscaled - g.reshape(-1)).astype(np.float64)
    depth_loss = float((diff_d[opaque] ** 2).sum() / n_op) if n_op else float("nan")
    dw = (w - wgt).astype(np.float64)
    if sel.startswith("L1"):
        los = float(np.abs(dw).sum() / n_rs)
        g_w = lam * np.sign(dw) / n_rs
    else:
        los = float((dw ** 2).sum() / n_rs)
        g_w = lam * 2.0 * dw / n_rs
    op_err = opacity.reshape(-1).astype(np.float64) - 1.0
    op_loss = float(np.abs(op_err[opaque]).sum() / n_op) if n_op else float("nan")
    dl_lambda = cfg["depthloss_lambda"]
    loss = dl_lambda * depth_loss + lam * los + op_loss
    inv = 1.0 / max(n_op, 1)
    g_depth = np.where(opaque, dl_lambda * 2.0 * diff_d * float(scale) * inv, 0.0)
    g_opacity = np.where(opaque, np.sign(op_err) * inv, 0.0)
    return dict(loss=loss, depth_loss=depth_loss, los_loss=los, opacity_loss=op_loss, los_lambda=lam,
                g_w=g_w, g_depth=g_depth, g_opacity=g_opacity, eps=eps, js=js, weights_gt=wgt,
                opaque=opaque, mean_eps=float(eps.astype(np.float64).mean()))


def logits_grad(z_m, depth_gt_m, eps=2.0, l_free=0.25, l_occ=2.5):
    x = (z_m - depth_gt_m.reshape(-1, 1)).astype(F32)
    free = (-x - F32(eps)) > 0
    occ = ((x + F32(eps)) > 0) & ((F32(eps) - x) > 0)
    return (F32(l_free) * free - F32(l_occ) * occ).astype(F32)
