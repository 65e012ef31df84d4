"""Per-workgroup time of the balanced accumulation (GPU box, -DLNR_EXP_WG_TIMES variant library):
the bench's C2 loop (60 steps); prints the workgroup duration spread and the slowest workgroups'
first level.  LONER_AMD_LIB=loner_amd/_lib/variants/wg.so python tools/accum_wg.py [C2]"""
import ctypes
import os
import sys

import numpy as np
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
    fn = L.lib().lnr_debug_accum_wg
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * (512 * 4))()
    assert fn(ctypes.cast(buf, ctypes.c_void_p)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 4).astype(np.int64)
    t0 = a[:, 0].min()
    dur = (a[:, 1] - a[:, 0]) / 100.0  # s_memtime: 100 MHz
    print(f"kernel span {(a[:, 1].max() - t0) / 100.0:.1f} us; wg duration min/med/max "
          f"{dur.min():.1f}/{np.median(dur):.1f}/{dur.max():.1f} us; start spread {(a[:, 0].max() - t0) / 100.0:.1f} us")
    for lvl in np.unique(a[:, 3]):
        m = a[:, 3] == lvl
        print(f"  first level {lvl:2d}: {m.sum():3d} wgs, duration med {np.median(dur[m]):.1f} max {dur[m].max():.1f} us, "
              f"records {a[m, 2].mean():.0f}")
    order = np.argsort(-dur)[:8]
    print("slowest:", [(int(i), round(float(dur[i]), 1), int(a[i, 3])) for i in order])


if __name__ == "__main__":
    main(*sys.argv[1:])
