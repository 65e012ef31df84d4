"""Per-level cost of the hash-grid encode: the C2-size encode (8192 rays x 512 samples, samples on the rays
as the bench's OGM-trained sampler would put them: sorted, clustered near the ray's surface) timed over
the first k levels for k = 1..16 (a grid descriptor with n_levels = k has the same first k levels), so the
differences are each level's own time.  HIP events, eval launch and training launch (+ record histogram).

    python tools/encode_levels.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loner_amd import _lib as L  # noqa: E402


def main():
    R, S = 8192, 512
    N = R * S
    g = torch.Generator(device="cuda").manual_seed(0)
    rays = torch.zeros(R, 13, device="cuda")
    rays[:, 0:3] = torch.rand(R, 3, device="cuda", generator=g) * 0.4 - 0.2
    d = torch.randn(R, 3, device="cuda", generator=g)
    rays[:, 3:6] = d / d.norm(dim=1, keepdim=True)
    # half the samples stratified over [0, 0.6], half clustered within 0.01 of a surface depth
    zs = torch.rand(R, S // 2, device="cuda", generator=g) * 0.6
    surf = torch.rand(R, 1, device="cuda", generator=g) * 0.5 + 0.05
    zi = surf + (torch.rand(R, S // 2, device="cuda", generator=g) - 0.5) * 0.02
    z = torch.sort(torch.cat([zs, zi], 1), 1)[0].contiguous()
    full = L.grid_desc(16, 2, 18, 16)
    table = (torch.rand(2 * int(full.n_entries), device="cuda", generator=g) * 2 - 1).half()
    enc = torch.empty(16, N, dtype=torch.int32, device="cuda")
    s = L.stream()
    out = {}
    ref = None
    for rl in (0, 3, 6):  # LONER_ENC_RUN_LEVELS: coherent levels gathering once per run of lanes in a cell
        os.environ["LONER_ENC_RUN_LEVELS"] = str(rl)
        out[f"run_levels_{rl}"] = one(rays, z, table, enc, R, S, N, s)
        if ref is None:
            ref = enc.clone()
        out[f"run_levels_{rl}"]["bitwise_equal"] = bool(torch.equal(ref, enc))
    print(json.dumps(out))


def one(rays, z, table, enc, R, S, N, s):
    out = {}
    for train in (False, True):
        per = []
        for k in range(1, 17):
            dk = L.grid_desc(k, 2, 18, 16)
            ws = None
            nb = 0
            if train:
                nb = int(L.lib().lnr_hashgrid_bwd_workspace_bytes(ctypes.byref(dk), N))
                ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
            ts = []
            for it in range(8):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                L.call("lnr_hashgrid_fwd_rays", ctypes.byref(dk), rays, z, R, S, table, enc, N, ws, nb, s)
                b.record()
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(a.elapsed_time(b))
            per.append(float(np.median(ts)))
            del ws
        levels = [per[0]] + [per[k] - per[k - 1] for k in range(1, 16)]
        out["train" if train else "eval"] = dict(total_ms=per[-1], per_level_ms=[round(v, 4) for v in levels])
    return out


if __name__ == "__main__":
    main()
