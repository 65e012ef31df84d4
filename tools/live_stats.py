#!/usr/bin/env python3
"""How the live samples (dL/dsigma != 0) of a trained C2 batch are laid out, to choose the backward's skip
granularity: the fraction of live samples, of 64-sample waves holding one, of 16-sample MLP tiles holding one,
and of coherent-level runs holding one.  Pre-trains the field as bench.py --field trained does.

    python tools/live_stats.py [--windows 12] [--iters 32]
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
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    import bench
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[args.config]
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    state = S_.FieldState(cfg, device=dev)
    scans = syn.make_window(kind, nkf, seed=1000)
    window = RayWindow(scans, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"], n_lidar=rpk, n_sky=spk,
                       strategy=strat, device=dev)
    R = window.n_slots
    eng = S_.StepEngine(state, R, seed=12345)
    out = {}

    def stats(tag, g):
        eng.step_window(window, global_step=g, prof={})  # eager (profiled) step: d_sigma stays readable
        torch.cuda.synchronize()
        d = eng.d_sigma(R).view(R, S).cpu().numpy()
        live = d != 0
        w = live.reshape(R, S // 64, 64).any(-1)
        t = live.reshape(R, S // 16, 16).any(-1)
        per_ray = live.sum(1)
        out[tag] = {"live_frac": float(live.mean()), "wave_live_frac": float(w.mean()),
                    "tile16_live_frac": float(t.mean()), "rays_all_dead": float((per_ray == 0).mean()),
                    "live_per_ray_p10_p50_p90": [float(np.percentile(per_ray, q)) for q in (10, 50, 90)],
                    "lane_util_in_live_waves": float(live.sum() / max(w.sum() * 64, 1))}
        print(tag, json.dumps(out[tag]), flush=True)

    stats("init", 0)
    g, pre = bench.pretrain(eng, state, kind, nkf, rpk, spk, strat, dev, R, 1, args.windows, args.iters)
    state.reset_optimizer()
    for i in range(5):
        eng.step_window(window, global_step=g + i, iteration_idx=i)
    stats("trained", g + 5)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
