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

Two communicators (round 6, bench.py LONER_EXCHANGE_GROUPS=2): the reduce-scatters on one queue, the all-gathers
on a second, so AG1 can start as soon as Adam1 is done instead of after RS2.  Whether that helps depends on
whether concurrent collectives share the link bandwidth: ``--share`` runs a fluid model (collectives that are in
their transfer phase at the same time split B equally); without it each queue gets B (an upper bound on the gain).

    python tools/zero_tail_model.py profiles/r05_bwd_levels_C4s8.json [--world 8] [--queues 2] [--share]
"""
import argparse
import collections
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


def simulate(jobs, bw_gbs, alpha_us, share):
    """Fluid timeline of collectives.  jobs: name -> (ready_us, queue, bytes over the link, deps); a job starts
    when ready, its queue is free and its deps are done, spends alpha_us in latency, then transfers its bytes at
    bw / (number of jobs transferring) if share else at bw.  Returns name -> end time (us)."""
    B = bw_gbs * 1e3  # bytes per us
    end, start, rem = {}, {}, {}
    q_free = collections.defaultdict(float)
    t = 0.0
    pending = dict(jobs)
    active = {}  # name -> transfer-phase start
    while pending or active:
        # start every job that can start now (its queue idle, ready, deps done)
        changed = True
        while changed:
            changed = False
            for nm, (ready, q, nbytes, deps) in sorted(pending.items(), key=lambda kv: kv[1][0]):
                if any(d not in end for d in deps):
                    continue
                st = max(ready, q_free[q], max([end[d] for d in deps], default=0.0))
                busy_q = any(jobs[a][1] == q for a in active) or any(jobs[a][1] == q and a not in end for a in start)
                if st <= t + 1e-9 and not busy_q:
                    start[nm] = t
                    rem[nm] = nbytes
                    active[nm] = t + alpha_us  # transfers after the latency
                    del pending[nm]
                    changed = True
                    break
        # next event: a pending job becoming startable, a latency ending, or a transfer finishing
        cands = []
        for nm, (ready, q, nbytes, deps) in pending.items():
            if all(d in end for d in deps):
                cands.append(max(ready, q_free[q], max([end[d] for d in deps], default=0.0)))
        moving = [a for a, t0 in active.items() if t0 <= t + 1e-9]
        rate = (B / len(moving) if share else B) if moving else 0.0
        for a in moving:
            cands.append(t + rem[a] / rate)
        for a, t0 in active.items():
            if t0 > t + 1e-9:
                cands.append(t0)
        cands = [c for c in cands if c > t + 1e-9]
        if not cands:
            break
        t1 = min(cands)
        for a in moving:
            rem[a] -= rate * (t1 - t)
        t = t1
        for a in list(active):
            if active[a] <= t + 1e-9 and rem[a] <= 1e-6:
                end[a] = t
                q_free[jobs[a][1]] = t
                del active[a]
    return end


def model2(cut, a1_ms, a2_ms, world, bw_gbs, alpha_us, queues, share, adam_tbs=7.0, n_mlp=3072):
    """The same tail as ``model`` with the collectives on ``queues`` communicators (RS on queue 0, AG on queue
    queues - 1) through the fluid simulation."""
    off = level_params()
    p1 = 2 * (off[16] - off[cut])
    p2 = n_mlp + 2 * off[cut]
    frac = (world - 1) / world
    adam = lambda p: 32 * p / world / (adam_tbs * 1e6)
    A1, A2 = 1e3 * a1_ms, 1e3 * a2_ms
    qa = queues - 1
    # Adam1 runs after RS1 and the second accumulate (stream order), Adam2 after Adam1 and RS2: modelled as
    # pseudo-jobs on a compute queue with zero link bytes and their duration as latency
    jobs = {"RS1": (A1, "A", 4 * p1 * frac, []), "RS2": (A1 + A2, "A", 4 * p2 * frac, ["RS1"])}
    e = simulate(jobs, bw_gbs, alpha_us, share)
    adam1_end = max(A1 + A2, e["RS1"]) + adam(p1)
    adam2_end = max(adam1_end, e["RS2"]) + adam(p2)
    jobs.update({"AG1": (adam1_end, "A" if qa == 0 else "B", 2 * p1 * frac, ["RS2"] if qa == 0 else []),
                 "AG2": (adam2_end, "A" if qa == 0 else "B", 2 * p2 * frac, ["AG1"])})
    e = simulate(jobs, bw_gbs, alpha_us, share)
    return dict(cut=cut, queues=queues, share=share, step_end_us=adam2_end, gather_end_us=e["AG2"],
                exposed_us=max(adam2_end, e["AG2"]) - (A1 + A2), accumulate_us=A1 + A2)


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
    rows2 = []
    print(f"\n{'cut':>3} {'B GB/s':>7} {'1 queue':>8} {'2 queues, shared B':>19} {'2 queues, B each':>17}   exposed us "
          f"(fluid model; the 1-queue column reproduces the table above)")
    cuts = sorted(int(k.split('-')[0]) for k in rng if k.endswith('-16'))
    for cut in cuts:
        for bw in (100.0, 200.0, 400.0):
            r1 = model2(cut, rng[f"{cut}-16"], rng[f"0-{cut}"], a.world, bw, a.alpha, 1, True)
            r2s = model2(cut, rng[f"{cut}-16"], rng[f"0-{cut}"], a.world, bw, a.alpha, 2, True)
            r2 = model2(cut, rng[f"{cut}-16"], rng[f"0-{cut}"], a.world, bw, a.alpha, 2, False)
            rows2 += [dict(r1, bw_GBs=bw), dict(r2s, bw_GBs=bw), dict(r2, bw_GBs=bw)]
            print(f"{cut:>3} {bw:>7.0f} {r1['exposed_us']:>8.1f} {r2s['exposed_us']:>19.1f} {r2['exposed_us']:>17.1f}")
    print(json.dumps(dict(world=a.world, alpha_us=a.alpha, rows=rows, two_queue_rows=rows2)))


if __name__ == "__main__":
    main()
