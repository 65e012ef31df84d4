#!/usr/bin/env python3
"""Early ray termination on a trained field: for thresholds of the per-ray transmittance product and phase cuts,
the share of rays still alive after each phase, the encode + field time, and whether the step stays bitwise the
step without termination (params, moments, shadow, occupancy, loss, depth over three steps).  GPU.

    python tools/experiments/r06_ert_tmin.py

(Ran against the first early-ray-termination version, commit 7de94c3: per-ray alive bytes and the LONER_ERT_TMIN
switch, both gone since; the phases now run over lists of the rays still alive)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    import bench
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS["C2"]
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    state = S_.FieldState(cfg, device=dev)
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    R = window.n_slots
    eng = S_.StepEngine(state, R, seed=12345)
    g, _ = bench.pretrain(eng, state, kind, nkf, rpk, spk, strat, dev, R, 1, 12, 32)
    eng.release()
    sd = state.state_dict()
    torch.cuda.synchronize()

    def run(tmin, cuts, ert):
        os.environ["LONER_ERT_TMIN"] = repr(tmin)
        os.environ["LONER_ERT_CUTS"] = cuts
        st = S_.FieldState(cfg, device=dev)
        st.load_state_dict(sd)
        st.reset_optimizer()
        e = S_.StepEngine(st, R, seed=9)
        e.live_bwd, e._live, e.ert = True, True, ert
        e.pipeline, e.use_graph = False, False
        alive = []
        for k in range(3):
            e.step_window(window, global_step=g + 5 + k, iteration_idx=k)
            torch.cuda.synchronize()
            alive.append(float(e.ert_alive.float().mean()))
        e.finish()
        out = {k: getattr(st, k).clone() for k in ("params", "m", "v", "shadow", "occ")}
        out["loss"] = e.loss_out.clone()
        out["depth"] = e.depth[:R].clone()
        # timing: 10 graph-replayed steps after 3 warm
        e.use_graph = True
        for k in range(3):
            e.step_window(window, global_step=g + 20 + k)
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for k in range(10):
            e.step_window(window, global_step=g + 30 + k)
        t1.record()
        torch.cuda.synchronize()
        return out, alive, t0.elapsed_time(t1) / 10

    base, _, tb = run(1e-100, "0.5,0.75", False)
    print(f"no termination: {tb:.4f} ms/step", flush=True)
    sweep = os.environ.get("ERT_SWEEP", "tmin")
    grid = ([(c, t) for c in ("0.5,0.75", "0.375,0.5,0.625,0.75,0.875", "0.25,0.5,0.75")
             for t in (1e-100, 1e-70, 1e-60, 1e-50, 1e-46)] if sweep == "tmin" else
            [(c, 1e-50) for c in ("0.5,0.75", "0.375,0.625", "0.375,0.5,0.75", "0.4375,0.625,0.8125", "0.5,0.625,0.75",
                                  "0.375,0.75", "0.5", "0.625", "0.375,0.5,0.625,0.75", "0.5,0.75")])
    for cuts, tmin in grid:
        if True:
            o, alive, t = run(tmin, cuts, True)
            same = all(torch.equal(base[k], o[k]) for k in base)
            diff = {k: int((base[k] != o[k]).sum()) for k in base if not torch.equal(base[k], o[k])}
            print(f"cuts {cuts:28s} tmin {tmin:8.0e}: alive after the last cut {np.round(alive, 3)}  "
                  f"{t:.4f} ms/step  bitwise {same} {diff}", flush=True)


if __name__ == "__main__":
    main()
