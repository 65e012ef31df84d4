#!/usr/bin/env python3
"""Where rays terminate on a trained field: after the bench's untimed pre-training of a config (bench.pretrain), one
step of the bench window, then the encode + sigma of that step's rays re-run in 64-sample phases
(lnr_hashgrid_fwd_rays_phase + lnr_field_sigma_phase, the early-ray-termination kernels), printing the share of
rays still alive (transmittance product >= 1e-50) after each phase, split into sky and LiDAR rays.  GPU.

    python tools/ert_profile.py C4
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd import _lib as L
    from loner_amd.rays import RayWindow
    import bench
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[name]
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    state = S_.FieldState(cfg, device=dev)
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    R = window.n_slots
    eng = S_.StepEngine(state, R, seed=12345)
    g, _ = bench.pretrain(eng, state, kind, nkf, rpk, spk, strat, dev, R, 1, 12, 32)
    eng.release()
    state.reset_optimizer()
    eng.pipeline, eng.use_graph = False, False
    eng.step_window(window, global_step=g, iteration_idx=0)
    eng.finish()
    torch.cuda.synchronize()
    n = eng._r_last
    rays, z = eng.rays[:n], eng.z
    s = L.stream(dev)
    lp = eng.loss_params(g, 0, window.scale, 0.0, n)
    T, keep = eng.ert_T, eng.ert_keep
    lists, counts = eng.ert_lists, eng.ert_counts
    sky = torch.zeros(n, dtype=torch.bool)
    off, nsel = window.ray_off_host, window.n_sel_host
    for k in range(window.n_kf):
        sky[off[k] + nsel[k]:off[k + 1]] = True
    sky = sky[:n].to(dev)
    print(f"{name}: {n} rays ({int(sky.sum())} sky), {S} samples; cfg.raw_noise_std {cfg.raw_noise_std}")
    key = L.step_key(eng.seed, g)
    for q, lo in enumerate(range(0, S, 64)):
        hi = lo + 64
        lin = None if q == 0 else lists[(q - 1) % 2]
        cin = None if q == 0 else counts[(q - 1) % 2:(q - 1) % 2 + 1]
        L.call("lnr_hashgrid_fwd_rays_phase", L.ctypes.byref(state.desc), rays, z, n, S, state.table_f16, eng.enc,
               eng.N, None, 0, lin, cin, 0, lo, hi, s)
        L.call("lnr_field_sigma_phase", state.mlp_f16, eng.enc, eng.N, rays, z, n, S, lo, hi, cfg.raw_noise_std, None,
               key, eng.ray_offset, L.ctypes.byref(lp), eng.ws, lin, cin, lists[q % 2], counts[q % 2:q % 2 + 1], T,
               keep, s)
        if hi < S:
            torch.cuda.synchronize()
            a = torch.zeros(n, dtype=torch.bool, device=dev)
            a[lists[q % 2][:int(counts[q % 2].item())].long()] = True  # (the rays still alive)
            lt = T[:n][~sky].clamp(min=1e-300).log10()
            print(f"  after sample {hi:4d}: alive {float(a.float().mean()):.3f}  lidar {float(a[~sky].float().mean()):.3f}"
                  f"  sky {float(a[sky].float().mean()) if bool(sky.any()) else float('nan'):.3f}   lidar log10 T"
                  f" median {float(lt.median()):8.1f} p90 {float(lt.quantile(0.9)):8.1f}", flush=True)
    # the rays' geometry: depth over far
    dg = eng.depth_gt[:n] if hasattr(eng, "depth_gt") else None
    if dg is not None:
        far = rays[:, 12]
        q = (dg / far)[~sky]
        print("  lidar depth / far quantiles 10/50/90:", [round(float(v), 3) for v in torch.quantile(q.float(), torch.tensor([0.1, 0.5, 0.9], device=dev))])


if __name__ == "__main__":
    main()
