"""Time lnr_sample_ogm alone (GPU box) on a C2-like (8192 rays x 512), a C3-like (4096 rays x 2048, no
jitter) and a C4-shard-like (1152 rays x 512) batch, with HIP events over repeated launches, and print a
digest of the sorted depths so variants can be checked bit for bit:
    LONER_AMD_LIB=<lib> python tools/sampler_time.py [--reps 50]
"""
import argparse
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from loner_amd import _lib as L
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    res = 100
    # occupancy logits: a few dense blobs in a sparse field (the trained grid's shape, roughly)
    g = np.full((res, res, res), -6.0, np.float32)
    for _ in range(40):
        c = rng.integers(5, res - 5, 3)
        r = rng.integers(2, 6)
        g[c[0] - r:c[0] + r, c[1] - r:c[1] + r, c[2] - r:c[2] + r] = rng.uniform(1, 8)
    occ = torch.from_numpy(g).to(dev)
    for name, R, S, perturb in (("C2-like", 8192, 512, 1.0), ("C3-like", 4096, 2048, 0.0), ("C4s8-like", 1152, 512, 1.0)):
        rays = np.zeros((R, 13), np.float32)
        o = rng.uniform(-0.3, 0.3, (R, 3))
        d = rng.normal(0, 1, (R, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays[:, 0:3], rays[:, 3:6] = o, d
        rays[:, 11], rays[:, 12] = 0.01, 1.2
        rt = torch.from_numpy(rays).to(dev)
        z = torch.empty(R, S, dtype=torch.float32, device=dev)

        def launch():
            L.call("lnr_sample_ogm", rt, R, S, occ, res, perturb, None, None, 12345, 0, z, None, L.stream(dev))

        for _ in range(5):
            launch()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            launch()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) / a.reps * 1e3
        fn = getattr(L.lib(), "lnr_debug_phases_sampler", None)  # (a -DLNR_EXP_STAMPS build: per-phase cycles)
        if fn is not None:
            import ctypes
            buf = (ctypes.c_ulonglong * 32)()
            fn.argtypes = [ctypes.c_void_p]
            fn(ctypes.cast(buf, ctypes.c_void_p))
            ph = list(buf)[:5]
            tot = max(sum(ph), 1)
            print("  phases (draws sort, strata + occupancy, cdf, inverse CDF, merge + store):",
                  " ".join(f"{p / tot:.2f}" for p in ph), flush=True)
        zz = z.cpu().numpy()
        ok = bool(np.all(np.diff(zz, axis=1) >= 0))
        print(f"{name}: {us:.1f} us per launch, sorted={ok}, digest {hashlib.sha1(zz.tobytes()).hexdigest()[:16]}",
              flush=True)


if __name__ == "__main__":
    main()
