#!/usr/bin/env python3
"""What the training encode's record histogram costs: k_hashgrid_fwd on the C2 batch of a (pre-trained) field with
and without the backward workspace (the histogram), HIP events over 20 launches each, interleaved.

    python tools/enc_hist_cost.py [--windows 6]
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
    ap.add_argument("--windows", type=int, default=6)
    args = ap.parse_args()
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS["C2"]
    state = S_.FieldState(S_.StepConfig(n_samples=S), device=dev)
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, device=dev)
    R = window.n_slots
    eng = S_.StepEngine(state, R, seed=12345)
    out = {}
    for phase in ("init", "trained"):
        if phase == "trained":
            bench.pretrain(eng, state, kind, nkf, rpk, spk, strat, dev, R, 1, args.windows, 32)
        eng.step_window(window, global_step=10 ** 6 + 1, prof={})  # rays + z of the bench window, eager
        torch.cuda.synchronize()
        s = L.stream(dev)
        t = {"hist": [], "nohist": []}
        for rep in range(20):
            for k in ("hist", "nohist"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(state.desc), eng.rays, eng.z, R, S, state.table_f16,
                       eng.enc, eng.N, eng.bwd_ws if k == "hist" else None, eng.bwd_ws_bytes if k == "hist" else 0, s)
                e1.record()
                t[k].append((e0, e1))
        torch.cuda.synchronize()
        out[phase] = {k: float(np.median([a.elapsed_time(b) for a, b in v])) for k, v in t.items()}
        print(phase, out[phase], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
