"""Host-side cost of enqueueing one optimiser step (GPU box): is a small config launch-bound?
Runs the bench's step loop for a config and prints, per step, the host time to enqueue (no sync),
the wall time with the queue drained, and the same with the bench's per-stage HIP events.
    python tools/host_overhead.py [C1] [--shard-of N]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C1")
    ap.add_argument("--shard-of", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import bench
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[a.config]
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    R = window.n_slots // a.shard_of
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    st = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(st, R, seed=1)
    for i in range(20):
        eng.step_window(window, global_step=i, n_rays_global=window.n_slots)
    torch.cuda.synchronize()
    for prof in (False, True):
        t0 = time.perf_counter()
        p = {} if prof else None
        for i in range(a.steps):
            eng.step_window(window, global_step=100 + i, n_rays_global=window.n_slots, prof=p)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{a.config} shard 1/{a.shard_of} events={prof}: enqueue {1e6 * (t1 - t0) / a.steps:.1f} us/step, "
              f"wall {1e6 * (t2 - t0) / a.steps:.1f} us/step")


if __name__ == "__main__":
    main()
