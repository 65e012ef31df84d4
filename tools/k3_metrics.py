"""K3 (hash-grid input gradient) numbers for DESIGN.md: d_pos against the oracle (rel L2, overall and
the worst level) and the cost of the input-gradient launch at the C2 size (4,194,304 samples from rays),
timed with HIP events on the launch stream.  GPU only; prints one JSON line.

    python tools/k3_metrics.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loner_amd import _lib as L  # noqa: E402
from oracle import hashgrid as ohg  # noqa: E402


def main():
    rng = np.random.default_rng(5)
    lay = ohg.GridLayout(16, 2, 18, 16)
    d = L.grid_desc(16, 2, 18, 16)
    table = rng.uniform(-1, 1, (lay.n_entries, 2)).astype(np.float16)
    t16 = torch.from_numpy(table.view(np.int16)).cuda()
    n = 8192
    pos = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    denc = rng.normal(0, 1, (n, 32)).astype(np.float32)

    def dpos(de):
        lm = torch.from_numpy(np.ascontiguousarray(de.reshape(n, 16, 2).transpose(1, 0, 2))).cuda()
        out = torch.empty(n, 3, device="cuda")
        L.call("lnr_hashgrid_bwd", ctypes.byref(d), torch.from_numpy(pos).cuda(), n, lm, n, None, t16, out, None, 0,
               0, L.stream())
        torch.cuda.synchronize()
        return out.cpu().numpy().astype(np.float64)

    def rel(a, b):
        return float(np.linalg.norm(a - b) / np.linalg.norm(b))

    overall = rel(dpos(denc), ohg.encode_input_grad(pos, table, denc, lay))
    per_level = []
    for lvl in range(16):
        dl = np.zeros_like(denc)
        dl[:, 2 * lvl:2 * lvl + 2] = denc[:, 2 * lvl:2 * lvl + 2]
        per_level.append(rel(dpos(dl), ohg.encode_input_grad(pos, table, dl, lay)))
    # cost at the C2 size: rays of 512 samples, d_enc level-major fp32
    R, S = 8192, 512
    N = R * S
    rays = torch.zeros(R, 13, device="cuda")
    rays[:, 0:3] = torch.rand(R, 3, device="cuda") - 0.5
    dr = torch.randn(R, 3, device="cuda")
    rays[:, 3:6] = dr / dr.norm(dim=1, keepdim=True)
    z = torch.sort(torch.rand(R, S, device="cuda") * 0.45, 1)[0]
    de = torch.randn(16, N, 2, device="cuda")
    out = torch.empty(N, 3, device="cuda")
    s = L.stream()
    per_pass = {}
    ref_out = None
    # levels per launch (LONER_DPOS_LEVELS_PER_PASS, read per call), then the one-launch level-outer
    # kernel at K samples per thread (LONER_DPOS_SPT = K)
    for per in (16, 8, 4, 2, 1, "spt2", "spt4", "spt8"):
        if isinstance(per, int):
            os.environ["LONER_DPOS_SPT"] = "0"
            os.environ["LONER_DPOS_LEVELS_PER_PASS"] = str(per)
        else:
            os.environ["LONER_DPOS_SPT"] = per[3:]
        times = []
        for it in range(13):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.call("lnr_hashgrid_bwd_rays", ctypes.byref(d), rays, z, R, S, de, N, None, t16, out, None, 0, 0, s)
            b.record()
            torch.cuda.synchronize()
            if it >= 3:
                times.append(a.elapsed_time(b))
        per_pass[per] = float(np.median(times))
        if ref_out is None:
            ref_out = out.clone()
        assert torch.equal(out, ref_out), per  # the split does not change a bit
    os.environ.pop("LONER_DPOS_LEVELS_PER_PASS")
    os.environ.pop("LONER_DPOS_SPT")
    ms = min(per_pass.values())
    # bytes per sample: 512 B of fp16 corner gathers (16 levels x 8 corners x 4 B), 128 B of d_enc, 12 B out
    print(json.dumps(dict(dpos_rel_l2=overall, dpos_rel_l2_worst_level=max(per_level),
                          dpos_rel_l2_per_level=[float(f"{v:.3g}") for v in per_level], c2_dpos_ms=ms,
                          c2_dpos_ms_by_levels_per_pass=per_pass,
                          c2_samples=N, gathered_gb_per_s=N * 512 / ms / 1e6)))


if __name__ == "__main__":
    main()
