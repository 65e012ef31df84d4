"""Same-address statistics of the accumulation's LDS atomics (GPU box): the bench's C2 loop
(on-device rays, OGM updates) for STEPS steps, then a few buckets of every level copied back; per
atomic wave-instruction (lane i takes record 2i or 2i + 1 of its wave's 128, without the accumulate's
slot mixing) the number of distinct entries, and the mean run of equal words (equal x-pair or corner)
between adjacent records.
    python tools/rec_conflicts.py [C2] [STEPS]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def a256(b):
    return (b + 255) // 256 * 256


def main(cfg_name="C2", steps="60"):
    import bench
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
    for i in range(int(steps)):
        eng.step_window(window, global_step=i)
    torch.cuda.synchronize()
    d = st.desc
    L = d.n_levels
    chunks = [(int(d.size[l]) + 4095) // 4096 for l in range(L)]
    nbk = sum(chunks)
    n = eng.N
    nsb = (n + 511) // 512
    nch = (nsb + 255) // 256
    off = a256(nbk * nsb * 4) + a256(L * nch * 128 * 4) + a256(16 * 4) + a256(2048 * 4)
    ws = eng.bwd_ws
    seg = ws[off:off + 2049 * 8].view(torch.int64).cpu().numpy()
    off += a256(2049 * 8) + a256(2 * 512 * 2 * 4096 * 8)
    rec = ws[off:].view(torch.int32)
    base = 0
    for l in range(L):
        multi, dist, p0, runs_eq = [], [], 0, []
        for b in range(base, base + chunks[l], max(1, chunks[l] // 4)):
            s0, s1 = int(seg[b]), int(seg[b + 1])
            r = rec[2 * s0:2 * s1].view(-1, 2).cpu().numpy()
            w = r[:, 0].astype(np.uint32)
            e0 = w & 4095
            p = (w >> 12) & 15
            e1 = e0 ^ ((1 << p) - 1)
            p0 += int((p == 0).sum())
            runs_eq.append(np.mean(w[1:] == w[:-1]))
            m = (len(w) // 128) * 128
            for u in range(2):  # the two records of a lane's 16-B load
                ee = e0[u:m:2].reshape(-1, 64)
                srt = np.sort(ee, axis=1)
                newv = np.concatenate([np.ones((srt.shape[0], 1), bool), srt[:, 1:] != srt[:, :-1]], axis=1)
                dist.append(newv.sum(1))
                # run lengths of equal values in the sorted rows -> max multiplicity
                idx = np.flatnonzero(np.concatenate([newv, np.ones((srt.shape[0], 1), bool)], axis=1).reshape(-1))
                runs = np.diff(idx)
                multi.append(runs.max() if len(runs) else 1)
                ee1 = e1[u:m:2].reshape(-1, 64)
                both = np.concatenate([ee, ee1], axis=1)
        dist = np.concatenate(dist)
        print(f"level {l:2d}: {chunks[l]:3d} buckets, records/bucket {np.mean(np.diff(seg[base:base + chunks[l] + 1])):.0f}, "
              f"single {p0}, distinct e0 per 64-lane instruction mean {dist.mean():.1f} p10 {np.percentile(dist, 10):.0f}, "
              f"adjacent equal words {np.mean(runs_eq):.3f}",
              flush=True)
        base += chunks[l]


if __name__ == "__main__":
    main(*sys.argv[1:])
