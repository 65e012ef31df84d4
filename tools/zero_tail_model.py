"""Modelled exposure of the sharded optimiser's tail (StepEngine._step_zero) per level cut, for one rank of an
N-GPU step.  Inputs: the measured accumulate time of each level range at that rank's
batch (tools/bwd_levels.py C4 s8 <ranges> --json, profiles/r05_bwd_levels_C4s8.json), the Adam pass rate
(k_adam streams 32 B per parameter at ~7 TB/s), and a ring bandwidth B and per-collective
latency alpha for RCCL over xGMI (not measurable on this pool's one-GPU boxes: swept).

Timeline after the scatter (t = 0), collectives serialised in enqueue order on the one communicator:
  acc1 [0, A1] -> RS1 (levels [cut, L), fp32) ; acc2 [A1, A1 + A2] -> RS2 (levels [0, cut) + MLP)
  Adam1 after max(acc2, RS1) -> AG1 (fp16 shadow chunk) ; Adam2 after max(Adam1, RS2) -> AG2
  the step ends after Adam2; the next step's encode waits for AG1 and AG2 (its ray build and sampling are
  prefetched on a side stream, so nothing else on the main stream hides the gathers).
Exposed = max(end of Adam2, end of AG2) - (A1 + A2): the time the exchange adds beyond the accumulation.
A ring reduce-scatter / all-gather moves (w - 1) / w of the buffer over each rank's link.

    python tools/zero_tail_model.py profiles/r05_bwd_levels_C4s8.json [--world 8]
"""
import argparse
import json
import math


def level_params():
    """Flat parameter offsets of the sigma grid (16 levels, base 16, scale 2, 2^18 entries, 2 features) + MLP."""
    sizes = []
    for l in range(16):
        res = math.ceil(16 * 2 ** l - 1) + 1
        sizes.append(min((res ** 3 + 7) // 8 * 8, 2 ** 18))
    off = [0]
    for z in sizes:
        off.append(off[-1] + z)
    return off


def model(cut, a1_ms, a2_ms, world, bw_gbs, alpha_us, adam_tbs=7.0, n_mlp=3072):
    off = level_params()
    p1 = 2 * (off[16] - off[cut])
    p2 = n_mlp + 2 * off[cut]
    frac = (world - 1) / world
    rs = lambda p: alpha_us + 4 * p * frac / (bw_gbs * 1e3)       # us (fp32 gradient)
    ag = lambda p: alpha_us + 2 * p * frac / (bw_gbs * 1e3)       # us (fp16 shadow)
    adam = lambda p: 32 * p / world / (adam_tbs * 1e6)            # us
    A1, A2 = 1e3 * a1_ms, 1e3 * a2_ms
    rs1_end = A1 + rs(p1)
    rs2_end = max(rs1_end, A1 + A2) + rs(p2)
    adam1_end = max(A1 + A2, rs1_end) + adam(p1)
    ag1_end = max(rs2_end, adam1_end) + ag(p1)
    adam2_end = max(adam1_end, rs2_end) + adam(p2)
    ag2_end = max(ag1_end, adam2_end) + ag(p2)
    return dict(cut=cut, A1_us=A1, A2_us=A2, rs2_MB=4 * p2 / 1e6, step_end_us=adam2_end, gather_end_us=ag2_end,
                exposed_us=max(adam2_end, ag2_end) - (A1 + A2), accumulate_us=A1 + A2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("levels_json")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--alpha", type=float, default=15.0, help="us per collective")
    a = ap.parse_args()
    d = json.loads(open(a.levels_json).read().strip().splitlines()[-1])
    rng = d["ranges_ms"]
    rows = []
    for cut in (4, 6, 8):
        for bw in (100.0, 200.0, 400.0):
            r = model(cut, rng[f"{cut}-16"], rng[f"0-{cut}"], a.world, bw, a.alpha)
            r["bw_GBs"] = bw
            rows.append(r)
    print(f"{'cut':>3} {'B GB/s':>7} {'acc [cut,16)':>12} {'acc [0,cut)':>11} {'RS2 MB':>7} {'step end':>9} "
          f"{'AG end':>8} {'exposed':>8}  (us, one rank of {a.world}, alpha {a.alpha} us)")
    for r in rows:
        print(f"{r['cut']:>3} {r['bw_GBs']:>7.0f} {r['A1_us']:>12.1f} {r['A2_us']:>11.1f} {r['rs2_MB']:>7.2f} "
              f"{r['step_end_us']:>9.1f} {r['gather_end_us']:>8.1f} {r['exposed_us']:>8.1f}")
    print(json.dumps(dict(world=a.world, alpha_us=a.alpha, rows=rows)))


if __name__ == "__main__":
    main()
