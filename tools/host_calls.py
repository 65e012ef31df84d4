"""Host cost of one optimiser step, per C-ABI entry point (GPU box): wraps loner_amd._lib.call to time
each call on the host (enqueue only), runs a few steps with the GPU kept idle in between (so no call
blocks on a full queue), and prints the mean host microseconds per call and the step's total host
time against its wall time.
    python tools/host_calls.py C4 --shard-of 8"""
import argparse
import collections
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C4")
    ap.add_argument("--shard-of", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--cprofile", action="store_true")
    a = ap.parse_args()
    import bench
    from loner_amd import _lib as L
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
    zero = (0, a.shard_of) if a.shard_of > 1 else None
    eng = S_.StepEngine(st, R, seed=1, zero=zero)
    for i in range(10):
        eng.step_window(window, global_step=i, n_rays_global=window.n_slots)
    torch.cuda.synchronize()
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    orig = L.call

    def timed(name, *args):
        t0 = time.perf_counter()
        r = orig(name, *args)
        acc[name] += time.perf_counter() - t0
        cnt[name] += 1
        return r

    L.call = timed
    tot_host, tot_wall = 0.0, 0.0
    for i in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step_window(window, global_step=100 + i + (i % 10 == 9), n_rays_global=window.n_slots)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tot_host += t1 - t0
        tot_wall += t2 - t0
    L.call = orig
    print(f"{a.config} shard 1/{a.shard_of}: host enqueue {1e6 * tot_host / a.steps:.1f} us/step, "
          f"idle-start wall {1e6 * tot_wall / a.steps:.1f} us/step")
    in_calls = sum(acc.values())
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:36s} {cnt[k] / a.steps:4.1f}/step  {1e6 * v / cnt[k]:7.1f} us/call")
    print(f"  in C-ABI calls {1e6 * in_calls / a.steps:.1f} us/step; other host work "
          f"{1e6 * (tot_host - in_calls) / a.steps:.1f} us/step")
    if a.cprofile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for i in range(a.steps):
            eng.step_window(window, global_step=200 + i, n_rays_global=window.n_slots)
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
