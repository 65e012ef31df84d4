"""Checkpoints in the reference's format.

The reference saves (src/mapping/mapper.py:161-175, examples/fdt_optimize_implicit_map.py:619-624)

    {'global_step': int,
     'network_state_dict': Model.state_dict(),         # one flat tcnn 'params' per module
     'optimizer_state_dict': torch.optim.Adam.state_dict(),
     'poses': ...,                                       # passed through unchanged
     'occ_model_state_dict': {'occupancy_grid': (1,1,V,V,V)},
     'occ_optimizer_state_dict': torch.optim.SGD.state_dict()}

and restores with Model.load_state_dict / OccupancyGridModel.load_state_dict / the global step
(fdt_optimize_implicit_map.py:161,344-359).  Module paths follow the reference's module tree
(model_tcnn.py:24-56, nerf_tcnn.py:19-52): the sigma field is ``nerf_model._model_sigma.params``,
tcnn's NetworkWithInputEncoding layout (network weights first, then the hash table).  tcnn keeps
fp16 ``params``; this build keeps an fp32 master (the optimiser's), written out as fp16 by default
so a reference-side ``load_state_dict`` sees its own dtype.

The Adam state is torch's own layout (``state[i] = {'step', 'exp_avg', 'exp_avg_sq'}`` plus
``param_groups``), param index 0 = the sigma params (optimizer.py:265).  Loading uses
``torch.load(weights_only=True)`` only.
"""
import torch

SIGMA_KEY = "nerf_model._model_sigma.params"
# the colour branch (nerf_tcnn.py:40-52): colour HashGrid, SH direction encoding (no parameters),
# colour FullyFusedMLP
COLOR_GRID_KEY = "nerf_model._pos_encoding.params"
DIR_ENC_KEY = "nerf_model._dir_encoding.params"
COLOR_MLP_KEY = "nerf_model._model_intensity.params"


def color_params(color_state):
    """{module path: flat params} of a ``loner_amd.camera.ColorState``, for ``other_params``."""
    cs = color_state
    return {COLOR_GRID_KEY: cs.params[cs.n_mlp:cs.n_params], DIR_ENC_KEY: cs.params[:0],
            COLOR_MLP_KEY: cs.params[:cs.n_mlp]}


def load_color(ck, color_state):
    """Restore a ColorState from a checkpoint dict's colour-branch params (sizes must match)."""
    net = ck["network_state_dict"]
    for k in (COLOR_GRID_KEY, COLOR_MLP_KEY):
        if k not in net:
            raise KeyError(f"checkpoint has no {k!r}")
    t, m = net[COLOR_GRID_KEY].reshape(-1), net[COLOR_MLP_KEY].reshape(-1)
    cs = color_state
    if t.numel() != cs.n_params - cs.n_mlp or m.numel() != cs.n_mlp:
        raise RuntimeError(f"colour head size mismatch: table {t.numel()} vs {cs.n_params - cs.n_mlp}, "
                           f"mlp {m.numel()} vs {cs.n_mlp}")
    cs.load(t, m)


def _adam_state_dict(m, v, step, lr):
    state = {}
    if step > 0:
        state[0] = {"step": torch.tensor(float(step)), "exp_avg": m, "exp_avg_sq": v}
    group = {"lr": lr, "betas": (0.9, 0.999), "eps": 1e-08, "weight_decay": 0, "amsgrad": False, "maximize": False,
             "foreach": None, "capturable": False, "differentiable": False, "fused": None, "params": [0]}
    return {"state": state, "param_groups": [group]}


def _sgd_state_dict(lr):
    group = {"lr": lr, "momentum": 0, "dampening": 0, "weight_decay": 0, "nesterov": False, "maximize": False,
             "foreach": None, "differentiable": False, "fused": None, "params": [0]}
    return {"state": {}, "param_groups": [group]}


def build_ckpt(state, global_step, poses=None, other_params=None, params_dtype=torch.float16):
    """The reference's checkpoint dict from a ``loner_amd.step.FieldState``.

    ``other_params``: optional {module path: flat params} of the colour head (e.g. from
    ``loner_amd.model.Model.state_dict()``), written next to the sigma field unchanged in layout."""
    n = state.n_params
    net = {SIGMA_KEY: state.params[:n].detach().to(params_dtype).cpu().clone()}
    for k, v in (other_params or {}).items():
        if k != SIGMA_KEY:
            net[k] = v.detach().to(params_dtype).cpu().clone()
    res = state.cfg.occ_res
    return {
        "global_step": int(global_step),
        "network_state_dict": net,
        "optimizer_state_dict": _adam_state_dict(state.m[:n].detach().cpu().clone(), state.v[:n].detach().cpu().clone(),
                                                 state.adam_step, state.cfg.lr),
        "poses": poses,
        "occ_model_state_dict": {"occupancy_grid": state.occ.detach().reshape(1, 1, res, res, res).cpu().clone()},
        "occ_optimizer_state_dict": _sgd_state_dict(state.cfg.occ_lr),
    }


def save_checkpoint(path, state, global_step, poses=None, other_params=None):
    torch.save(build_ckpt(state, global_step, poses, other_params), path)


def load_checkpoint(src, state, load_optimizer=True):
    """Restore a FieldState from a reference-format checkpoint (a path or an already loaded dict).
    Returns the checkpoint dict (global_step, poses, other modules' params for the caller).

    A reference checkpoint's sigma ``params`` must have this field's size (same n_levels,
    log2_hashmap_size, base_resolution and MLP shape); a mismatch raises like ``load_state_dict``."""
    ck = torch.load(src, map_location="cpu", weights_only=True) if not isinstance(src, dict) else src
    net = ck["network_state_dict"]
    if SIGMA_KEY not in net:
        raise KeyError(f"checkpoint has no {SIGMA_KEY!r} (keys: {sorted(net)[:8]})")
    p = net[SIGMA_KEY].reshape(-1)
    n = state.n_params
    if p.numel() != n:
        raise RuntimeError(f"size mismatch for {SIGMA_KEY}: checkpoint {p.numel()} vs this field {n}")
    with torch.no_grad():
        state.params[:n].copy_(p.to(state.params.device, torch.float32))
        occ = ck.get("occ_model_state_dict", {}).get("occupancy_grid")
        if occ is not None:
            if occ.numel() != state.occ.numel():
                raise RuntimeError(f"size mismatch for occupancy_grid: {tuple(occ.shape)}")
            state.occ.copy_(occ.reshape(-1).to(state.occ.device, torch.float32))
        st0 = ck.get("optimizer_state_dict", {}).get("state", {}).get(0) if load_optimizer else None
        if st0 is not None and st0["exp_avg"].numel() == n:
            state.m[:n].copy_(st0["exp_avg"].reshape(-1).to(state.m.device, torch.float32))
            state.v[:n].copy_(st0["exp_avg_sq"].reshape(-1).to(state.v.device, torch.float32))
            state.adam_step = int(float(st0["step"]))
        else:
            state.reset_optimizer()
    state.refresh_shadow()
    return ck
