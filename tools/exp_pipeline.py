"""Would a row-pipelined step pay?  (GPU box.)  The step's batch split into K chunks (K independent engines,
each 1/K of the config's keyframes, own parameters and buffers): every chunk runs encode -> field ->
scatter (the backward up to its records).  Timed two ways, per step of all K chunks:
  sequential: E0 F0 S0 E1 F1 S1 ... on one stream (what a chunked step costs with no overlap)
  pipelined:  the encodes on stream 1 (E0 E1 ...), each chunk's field + scatter on stream 2 after its encode,
              so chunk c's field and scatter co-run with chunk c+1's encode.
Against the whole batch in one engine: E F S.  The accumulate is the same in every form and left out.
    python tools/exp_pipeline.py [C2] [--chunks 2 4] [--reps 20]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C2")
    ap.add_argument("--chunks", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[a.config]
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))

    def engines(k):
        out = []
        for c in range(k):
            w = RayWindow(syn.make_window(kind, nkf // k, seed=1000 + c), syn.world_cube(kind),
                          syn.SENSORS[kind]["ray_range"], n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
            st = S_.FieldState(cfg, device=dev, seed=7 + c)
            e = S_.StepEngine(st, w.n_slots, seed=1 + c)
            e.pipeline = False
            e.use_graph = False
            for i in range(12):
                e.step_window(w, global_step=i + 1, n_rays_global=w.n_slots)
            out.append(stages(e))
        torch.cuda.synchronize()
        return out

    def stages(e):
        st, N, R = e.state, e.N, e.n_rays

        def enc():
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), e.rays, e.z, R, S, st.table_f16, e.enc, N,
                   e.bwd_ws, e.bwd_ws_bytes, L.stream(dev))

        lp = e.loss_params(5, 0, 1.0, None, R, e.far_ref)

        def field():
            L.call("lnr_field_train", st.mlp_f16, e.enc, N, e.rays, e.z, e.depth_gt, R, S, cfg.raw_noise_std, None,
                   L.step_key(e.seed, 5), e.ray_offset, L.ctypes.byref(lp), e.d_enc, st.grad_mlp, e.ws, e.stats,
                   e.depth, e.opacity, None, e.level_max_ptr, e.d_jac, L.stream(dev))

        def scatter():
            e._grid_bwd(e.rays, R, S, N, L.BWD_COUNTS_READY | L.BWD_LEVEL_MAX_READY | L.BWD_NO_ACCUM, L.stream(dev))

        # the scan turns the encode's histogram into offsets in place: a scatter timed on its own (no encode before
        # it) first restores the encode's counts (a ~10 us copy, in the alone times only)
        nb = sum((int(st.desc.size[l]) + 4095) // 4096 for l in range(cfg.n_levels))
        hist = e.bwd_ws[256:256 + 4 * nb * ((N + 511) // 512)]
        enc()
        snap = hist.clone()

        def scatter_alone():
            hist.copy_(snap)
            scatter()

        return dict(enc=enc, field=field, scatter=scatter, scatter_alone=scatter_alone)

    def run(seq_fns, reps):
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            seq_fns()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / reps * 1e3

    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def pipelined(ch):
        main = torch.cuda.current_stream(dev)
        f = torch.cuda.Event()
        f.record(main)
        evs = [torch.cuda.Event() for _ in ch]
        with torch.cuda.stream(s1):
            s1.wait_event(f)
            for c, ev in zip(ch, evs):
                c["enc"]()
                ev.record(s1)
        with torch.cuda.stream(s2):
            s2.wait_event(f)
            for c, ev in zip(ch, evs):
                s2.wait_event(ev)
                c["field"]()
                c["scatter"]()
            d2 = torch.cuda.Event()
            d2.record(s2)
        d1 = torch.cuda.Event()
        d1.record(s1)
        main.wait_event(d1)
        main.wait_event(d2)

    one = engines(1)[0]
    base = {k: run(one[k if k != "scatter" else "scatter_alone"], a.reps) for k in ("enc", "field", "scatter")}
    whole = run(lambda: (one["enc"](), one["field"](), one["scatter"]()), a.reps)
    print(f"{a.config} whole batch: enc {base['enc']:.1f} field {base['field']:.1f} scatter {base['scatter']:.1f} us;"
          f" E F S in sequence {whole:.1f} us", flush=True)
    del one
    torch.cuda.empty_cache()
    for k in a.chunks:
        ch = engines(k)
        for _ in range(2):  # warm both forms
            run(lambda: [f() for c in ch for f in (c["enc"], c["field"], c["scatter"])], 3)
            run(lambda: pipelined(ch), 3)
        alone = {s: sum(run(c[s if s != "scatter" else "scatter_alone"], a.reps) for c in ch)
                 for s in ("enc", "field", "scatter")}
        seq = run(lambda: [f() for c in ch for f in (c["enc"], c["field"], c["scatter"])], a.reps)
        pip = run(lambda: pipelined(ch), a.reps)
        print(f"  K={k}: chunks' stages summed: enc {alone['enc']:.1f} field {alone['field']:.1f} scatter "
              f"{alone['scatter']:.1f} us; sequential {seq:.1f} us; pipelined {pip:.1f} us "
              f"(saved {seq - pip:.1f} vs sequential, {whole - pip:.1f} vs the whole batch)", flush=True)
        del ch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
