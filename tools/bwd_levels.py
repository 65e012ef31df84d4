"""Per-level cost of the hash-grid backward's accumulation (GPU box): the bench's C2 loop (60 steps), then the
backward with LNR_BWD_NO_ACCUM and lnr_hashgrid_bwd_accum one level at a time (then any extra
level ranges "l0-l1" in one launch each), HIP events around each.  "s<K>" as an extra argument runs one
rank's share of a K-way ray split (bench.py --shard-of K); "--json" prints one JSON line at the end.
Usage: python tools/bwd_levels.py [C2|C4] [s8] [0-5 5-16 ...] [--json]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(cfg_name="C2", *extra):
    shard = next((int(x[1:]) for x in extra if x.startswith("s") and x[1:].isdigit()), 1)
    as_json = "--json" in extra
    extra = [x for x in extra if "-" in x and not x.startswith("-") and not x.startswith("s")]
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
    R = window.n_slots // shard
    eng = S_.StepEngine(st, R, seed=12345)
    for i in range(60):  # the bench's loop: OGM updates concentrate the samples
        eng.step_window(window, global_step=i, n_slots=R, n_rays_global=window.n_slots)
    torch.cuda.synchronize()
    rays = eng.rays
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
    avg = {k: sum(v) / len(v) for k, v in times.items()}
    print(f"{cfg_name} shard 1/{shard}: N={N} scatter+scans {avg['scatter']:.3f} ms")
    tot = 0.0
    for l in range(nl):
        t = avg[(l, l + 1)]
        tot += t
        print(f"  level {l:2d} res {d.resolution[l]:7d} size {d.size[l]:7d}: accum {t * 1e3:7.1f} us")
    print(f"  accum total {tot:.3f} ms")
    for r in ranges[nl:]:
        print(f"  levels [{r[0]}, {r[1]}) in one launch: {avg[r] * 1e3:7.1f} us")
    if as_json:
        print(json.dumps(dict(config=cfg_name, shard=shard, N=N, scatter_ms=avg["scatter"],
                              level_accum_ms=[avg[(l, l + 1)] for l in range(nl)],
                              ranges_ms={f"{a}-{b}": avg[(a, b)] for a, b in ranges[nl:]})))


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["C2"]))
