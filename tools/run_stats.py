"""Runs of consecutive samples in one grid cell, per level (GPU box): the bench's loop (on-device rays,
OGM updates) for STEPS steps, then the last step's rays and samples are copied back and, per level,
the lanes of every 64-sample wave are split into runs of equal cells (consecutive samples of one
ray).  Prints the mean run length and the backward's records per sample for the current record
format (coherent levels: 8 per run; fine levels: 4 per sample) and for an adaptive one (a run of
one sample: 4 pair records; a longer run: 8 corner records at its tail).
    python tools/run_stats.py [C2] [STEPS]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(cfg_name="C2", steps="60"):
    import bench
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[cfg_name]
    dev = torch.device("cuda", 0)
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    st = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(st, window.n_slots, seed=12345)
    for i in range(int(steps)):
        eng.step_window(window, global_step=i)
    torch.cuda.synchronize()
    rays = eng.rays.cpu().numpy()
    z = eng.z.cpu().numpy()
    R = rays.shape[0]
    xyz = rays[:, None, 0:3] + rays[:, None, 3:6] * z[:, :, None]
    pos = ((xyz + np.float32(1)) / np.float32(2)).astype(np.float32).reshape(-1, 3)
    d = st.desc
    tot_cur = tot_ad = 0.0
    for l in range(int(d.n_levels)):
        sc = np.float32(d.scale[l])
        cell = np.floor(pos * sc + np.float32(0.5)).astype(np.int64)
        key = (cell[:, 0] * 1000003 + cell[:, 1]) * 1000033 + cell[:, 2]
        kw = key.reshape(-1, 64)
        head = np.ones_like(kw, dtype=bool)
        head[:, 1:] = kw[:, 1:] != kw[:, :-1]
        runs = head.sum()
        n = kw.size
        # run lengths
        idx = np.flatnonzero(head.reshape(-1))
        lens = np.diff(np.append(idx, n))
        single = (lens == 1).sum()
        multi = (lens > 1).sum()
        coherent = int(d.resolution[l]) <= 512 * S // 512
        cur = (8 * runs if coherent else 4 * n) / n
        ad = (4 * single + 8 * multi) / n
        tot_cur += cur
        tot_ad += ad
        print(f"level {l:2d} res {int(d.resolution[l]):6d}  mean run {n / runs:6.2f}  single {single / runs:5.2f}  "
              f"records/sample: current {cur:5.2f} ({'coherent' if coherent else 'fine'})  adaptive {ad:5.2f}")
    print(f"total records/sample: current {tot_cur:.2f}  adaptive {tot_ad:.2f}  ({R} rays x {S})")


if __name__ == "__main__":
    main(*sys.argv[1:])
