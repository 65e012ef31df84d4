#!/usr/bin/env python3
"""Feasibility of a lazy encode: how many samples of a trained C2 batch are PROVABLY dead (relu(sigma + n) = 0)
from the coarse levels alone.  sigma = sum_j W1_j relu(h_j), h_j = sum_i W0_ji e_i; with the levels < k known
and every finer feature bounded by the largest |table value| of its level (M_i), h_j lies in [c_j - B_j, c_j + B_j]
and sigma <= U = sum_{W1_j > 0} W1_j relu(c_j + B_j) + sum_{W1_j < 0} W1_j relu(c_j - B_j).  A sample with U + n < 0
needs none of the levels >= k (its alpha is 0 whatever they hold).  Prints, per k, the share of samples proven
dead against the share actually dead.

    python tools/dead_bound.py [--windows 12] [--rays 256]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=12)
    ap.add_argument("--rays", type=int, default=256)
    args = ap.parse_args()
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    from oracle import rng as orng
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS["C2"]
    state = S_.FieldState(S_.StepConfig(n_samples=S), device=dev)
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, device=dev)
    R = window.n_slots
    eng = S_.StepEngine(state, R, seed=12345)
    eng.live_bwd, eng._live = False, False
    g, _ = bench.pretrain(eng, state, kind, nkf, rpk, spk, strat, dev, R, 1, args.windows, 32)
    gs = g + 5
    eng.step_window(window, global_step=gs, prof={})  # eager: enc, z, d_sigma of this batch
    torch.cuda.synchronize()
    n = args.rays * S
    stride = R // args.rays
    ray_ids = np.arange(0, R, stride)[:args.rays]
    samp = (ray_ids[:, None] * S + np.arange(S)[None, :]).reshape(-1)
    enc = eng.enc.view(torch.float16).view(16, eng.N, 2)[:, torch.from_numpy(samp).to(dev)].float()  # (16, n, 2)
    e = enc.permute(1, 0, 2).reshape(n, 32).cpu().numpy().astype(np.float64)
    p16 = state.shadow[:state.n_mlp].float().cpu().numpy().astype(np.float64)
    w0, w1 = p16[:2048].reshape(64, 32), p16[2048:3072].reshape(16, 64)[0]
    tab = state.shadow[state.n_mlp:state.n_mlp + 2 * state.n_entries].float().view(-1, 2).cpu().numpy()
    off = [int(state.desc.offset[l]) for l in range(17)]
    M = np.zeros(32)
    for l in range(16):
        M[2 * l:2 * l + 2] = np.abs(tab[off[l]:off[l + 1]]).max(0)
    a, b = orng.ray_sample_grid(ray_ids, S)
    noise = orng.normal(L.step_key(12345, gs), orng.STREAM_NOISE, a, b).reshape(-1).astype(np.float64)
    h = e @ w0.T
    sigma = np.maximum(h, 0) @ w1
    dead = sigma + noise <= 0
    ds = eng.d_sigma(R).view(R, S)[torch.from_numpy(ray_ids).to(dev)].reshape(-1).cpu().numpy()
    out = {"dead_true": float(dead.mean()), "dsigma_zero": float((ds == 0).mean()),
           "level_max_abs": [float(max(M[2 * l], M[2 * l + 1])) for l in range(16)], "proven": {}}
    for k in range(4, 16):
        c = e[:, :2 * k] @ w0[:, :2 * k].T
        B = (np.abs(w0[:, 2 * k:]) * M[None, 2 * k:]).sum(1)
        U = np.where(w1 > 0, w1 * np.maximum(c + B, 0), w1 * np.maximum(c - B, 0)).sum(1)
        proven = (U + noise) < -1e-3 * (1 + np.abs(U))  # margin for the fp16 roundings
        assert not (proven & ~dead).any(), "bound violated"
        out["proven"][k] = float(proven.mean())
        print(f"levels < {k:2d} known: proven dead {proven.mean():.3f} of samples (dead {dead.mean():.3f})", flush=True)
    # transmittance: samples behind the first opaque one (T = 0 exactly) have weight 0 and dL/dsigma = 0 too
    from oracle import render as orender
    rn = eng.rays[torch.from_numpy(ray_ids).to(dev)].cpu().numpy()
    zz = eng.z[torch.from_numpy(ray_ids).to(dev)].cpu().numpy()
    r2o = orender.raw2outputs(sigma.reshape(args.rays, S).astype(np.float16).astype(np.float32), zz, rn[:, 3:6],
                              noise.reshape(args.rays, S).astype(np.float32), rn[:, -1:])
    T = r2o["T"]
    tz = T == 0
    first = np.where(tz.any(1), tz.argmax(1), S)
    out["T_zero_frac"] = float(tz.mean())
    out["first_T_zero_p10_p50_p90"] = [float(np.percentile(first, q)) for q in (10, 50, 90)]
    out["dead_or_T_zero"] = float((dead.reshape(args.rays, S) | tz).mean())
    print("T == 0:", out["T_zero_frac"], "first index p10/p50/p90:", out["first_T_zero_p10_p50_p90"],
          "dead or T == 0:", out["dead_or_T_zero"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
