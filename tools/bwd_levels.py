"""Per-level cost of the hash-grid backward's accumulation (GPU box): one C2/CAM-shaped step, then the
backward with LNR_BWD_NO_ACCUM and lnr_hashgrid_bwd_accum one level at a time, HIP events around
each.  Usage: python tools/bwd_levels.py [C2|C4]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(cfg_name="C2"):
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[cfg_name]
    dev = torch.device("cuda", 0)
    win = syn.make_window(kind, nkf, seed=0, start=5)
    rays, dgt = syn.build_batch(win, kind, rpk, spk, strat, seed=1)
    rays, dgt = rays.to(dev), dgt.to(dev)
    R = rays.shape[0]
    cfg = S_.StepConfig(n_samples=S, loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    st = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(st, R, seed=1)
    for i in range(3):
        eng.step(rays, dgt, global_step=i + 1, scale=syn.CUBES[kind][0], far_ref=float(rays[0, -1]))
    torch.cuda.synchronize()
    s = L.stream(dev)
    N = eng.N
    nl = st.desc.n_levels
    times = {}
    for rep in range(5):
        L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rays, eng.z, R, S, st.table_f16, eng.enc, N,
               eng.bwd_ws, eng.bwd_ws_bytes, s)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        L.call("lnr_hashgrid_bwd_rays", L.ctypes.byref(st.desc), rays, eng.z, R, S, eng.d_enc, N, st.grad_table,
               eng.bwd_ws, eng.bwd_ws_bytes, L.BWD_COUNTS_READY | L.BWD_NO_ACCUM, s)
        e1.record()
        evs = [e1]
        for l in range(nl):
            L.call("lnr_hashgrid_bwd_accum", L.ctypes.byref(st.desc), N, eng.bwd_ws, eng.bwd_ws_bytes, l, l + 1,
                   st.grad_table, s)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        torch.cuda.synchronize()
        if rep == 0:
            continue
        times.setdefault("scatter", []).append(e0.elapsed_time(e1))
        for l in range(nl):
            times.setdefault(l, []).append(evs[l].elapsed_time(evs[l + 1]))
    d = st.desc
    print(f"{cfg_name}: N={N} scatter+scans {sum(times['scatter']) / len(times['scatter']):.3f} ms")
    tot = 0.0
    for l in range(nl):
        t = sum(times[l]) / len(times[l])
        tot += t
        print(f"  level {l:2d} res {d.resolution[l]:7d} size {d.size[l]:7d}: accum {t * 1e3:7.1f} us")
    print(f"  accum total {tot:.3f} ms")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["C2"]))
