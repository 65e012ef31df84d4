"""Kernel experiment driver (GPU box): C2 optimiser steps plus the stand-alone forward (no
histogram) and count+backward sequence, so rocprofv3 --stats separates every kernel's cost.

    LONER_AMD_LIB=<variant .so> rocprofv3 --kernel-trace --stats ... -- python3 tools/exp_kernels.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def read_phases(L):
    """Per-TU phase cycle sums of a -DLNR_EXP_STAMPS build ({} for a production build)."""
    import ctypes
    out = {}
    for tu in ("hashgrid_bwd", "hashgrid", "field"):
        fn = getattr(L.lib(), f"lnr_debug_phases_{tu}", None)
        if fn is None:
            continue
        buf = (ctypes.c_ulonglong * 32)()
        fn.argtypes = [ctypes.c_void_p]
        if fn(ctypes.cast(buf, ctypes.c_void_p)) == 0:
            out[tu] = list(buf)
    return out


def main():
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    cfg_name = os.environ.get("EXP_CONFIG", "C2")
    steps = int(os.environ.get("EXP_STEPS", "10"))
    kind, nkf, rpk, spk, strat, n_samples, preset = syn.CONFIGS[cfg_name]
    dev = torch.device("cuda", 0)
    win = syn.make_window(kind, nkf, seed=0, start=5)
    rays, dgt = syn.build_batch(win, kind, rpk, spk, strat, seed=1)
    rays, dgt = rays.to(dev), dgt.to(dev)
    R = rays.shape[0]
    cfg = S_.StepConfig(n_samples=n_samples, loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    st = S_.FieldState(cfg, device=dev)
    eng = S_.StepEngine(st, R, seed=1, count_in_forward=os.environ.get("EXP_FWD_COUNT", "1") == "1")
    scale = syn.CUBES[kind][0]
    far = float(rays[0, -1])
    for i in range(3):
        eng.step(rays, dgt, global_step=i + 1, scale=scale, far_ref=far)
    torch.cuda.synchronize()
    phases = read_phases(L)  # clears
    t0 = time.perf_counter()
    for i in range(steps):
        eng.step(rays, dgt, global_step=i + 4, scale=scale, far_ref=far, update_ogm=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    phases = read_phases(L)
    for tu, ph in phases.items():
        print(f"phases {tu}: " + " ".join(f"[{k}]={v}" for k, v in enumerate(ph) if v), flush=True)
    s = L.stream(dev)
    N = eng.N
    for i in range(steps):  # forward without histogram, then count + full backward
        L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), rays, eng.z, R, n_samples, st.table_f16, eng.enc, N,
               None, 0, s)
        eng._grid_bwd(rays, R, n_samples, N, 0, s)
    torch.cuda.synchronize()
    print(f"{cfg_name}: {ms:.3f} ms/step (no OGM), {R * n_samples / ms * 1e3:.3e} ray-samples/s", flush=True)


if __name__ == "__main__":
    main()
