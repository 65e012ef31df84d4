"""Per-level cost of the hash-grid backward's accumulation (GPU box): the bench's C2 loop (60 steps), then the
backward with LNR_BWD_NO_ACCUM and lnr_hashgrid_bwd_accum one level at a time (then any extra
level ranges "l0-l1" in one launch each), HIP events around each.
Usage: python tools/bwd_levels.py [C2|C4] [0-5 5-16 ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(cfg_name="C2", *extra):
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[cfg_name]
    dev = torch.device("cuda", 0)
    from loner_amd.rays import RayWindow
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    st = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(st, window.n_slots, seed=12345)
    for i in range(60):  # the bench's loop: OGM updates concentrate the samples
        eng.step_window(window, global_step=i)
    torch.cuda.synchronize()
    rays, R = eng.rays, window.n_slots
    s = L.stream(dev)
    N = eng.N
    nl = st.desc.n_levels
    times = {}
    ranges = [(l, l + 1) for l in range(nl)] + [tuple(int(x) for x in r.split("-")) for r in extra]
    for rep in range(5):
        L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rays, eng.z, R, S, st.table_f16, eng.enc, N,
               eng.bwd_ws, eng.bwd_ws_bytes, s)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        eng._grid_bwd(rays, R, S, N, L.BWD_COUNTS_READY | L.BWD_LEVEL_MAX_READY | L.BWD_NO_ACCUM, s)
        e1.record()
        evs = [e1]
        for (l0, l1) in ranges:
            L.call("lnr_hashgrid_bwd_accum", L.ctypes.byref(st.desc), N, eng.bwd_ws, eng.bwd_ws_bytes, l0, l1,
                   st.grad_table, s)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        torch.cuda.synchronize()
        if rep == 0:
            continue
        times.setdefault("scatter", []).append(e0.elapsed_time(e1))
        for k, r in enumerate(ranges):
            times.setdefault(r, []).append(evs[k].elapsed_time(evs[k + 1]))
    d = st.desc
    print(f"{cfg_name}: N={N} scatter+scans {sum(times['scatter']) / len(times['scatter']):.3f} ms")
    tot = 0.0
    for l in range(nl):
        t = sum(times[(l, l + 1)]) / len(times[(l, l + 1)])
        tot += t
        print(f"  level {l:2d} res {d.resolution[l]:7d} size {d.size[l]:7d}: accum {t * 1e3:7.1f} us")
    print(f"  accum total {tot:.3f} ms")
    for r in ranges[nl:]:
        print(f"  levels [{r[0]}, {r[1]}) in one launch: {sum(times[r]) / len(times[r]) * 1e3:7.1f} us")


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["C2"]))
