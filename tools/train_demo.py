"""End-to-end check that the path learns a map (GPU box): optimise the sigma field on a synthetic
quad window (C2 shape, on-device ray building, OGM updates) and report compute_l1_depth on a
held-out scan before and after, as fdt_optimize_implicit_map.py does after each window.

    python tools/train_demo.py [--steps 600] [--kind quad]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--kind", default="quad")
    ap.add_argument("--window", type=int, default=32, help="optimiser steps per window (fdt driver: 32)")
    args = ap.parse_args()
    import bench
    from loner_amd import evaluate as E
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    kind = args.kind
    dev = torch.device("cuda", 0)
    wc, rr = syn.world_cube(kind), syn.SENSORS[kind]["ray_range"]
    scans = syn.make_window(kind, 16, seed=1000)
    window = RayWindow(scans, wc, rr, n_lidar=512, strategy="RANDOM", device=dev)
    held = syn.make_window(kind, 1, seed=77, start=3)[0]  # a pose between the window's keyframes
    cfg = S_.StepConfig(n_samples=512, loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS["default"]))
    state = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(state, window.n_slots, seed=5)
    rend = E.DepthRenderer(state, n_samples=512, chunk=8192)
    sub = torch.arange(0, held["distances"].shape[0], 7)
    held = dict(directions=held["directions"][:, sub].contiguous(), distances=held["distances"][sub].contiguous(),
                pose=held["pose"])

    def l1():
        return float(E.compute_l1_depth(rend, held, held["pose"], wc, rr, key=1).item())

    rec = {"kind": kind, "steps": args.steps, "l1_before_m": l1(), "loss": []}
    t0 = time.perf_counter()
    for it in range(args.steps):
        if it % args.window == 0:
            state.reset_optimizer()  # a new Adam per window (optimizer.py:255-265)
        out = eng.step_window(window, global_step=it, iteration_idx=it % args.window)
        if it % 50 == 0 or it == args.steps - 1:
            rec["loss"].append([it, float(out[0].item())])
            print(f"step {it}: loss {rec['loss'][-1][1]:.4f}", flush=True)
    torch.cuda.synchronize()
    rec["train_s"] = time.perf_counter() - t0
    rec["l1_after_m"] = l1()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
