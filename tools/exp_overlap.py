"""Do the step's stages co-run on the chip? (GPU box.)  Two independent engines at one config (own
parameters and buffers, so no data is shared); each stage is timed alone and then launched
concurrently with another engine's stage on a second stream.  A pair whose concurrent time is well
below the sum of the alone times can be overlapped inside the step by splitting the batch.
    python tools/exp_overlap.py [C2] [--reps 20]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C2")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from loner_amd import _lib as L
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[a.config]
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, n_sky=spk, strategy=strat, device=dev)
    R = window.n_slots
    cfg = S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(bench.LOSS_PRESETS[preset]))
    engs = []
    for k in range(2):
        st = S_.FieldState(cfg, device=dev, seed=7 + k)
        e = S_.StepEngine(st, R, seed=1 + k)
        e.pipeline = False
        for i in range(12):
            e.step_window(window, global_step=i + 1, n_rays_global=R)
        engs.append(e)
    torch.cuda.synchronize()

    def stages(e):
        st, N = e.state, e.N

        def enc():
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), e.rays, e.z, R, S, st.table_f16, e.enc, N,
                   e.bwd_ws, e.bwd_ws_bytes, L.stream(dev))

        def enc0():  # no record histogram (the eval encode)
            L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(st.desc), e.rays, e.z, R, S, st.table_f16, e.enc, N,
                   None, 0, L.stream(dev))

        lp = e.loss_params(5, 0, window.scale, None, R, e.far_ref)

        def field():
            L.call("lnr_field_train", st.mlp_f16, e.enc, N, e.rays, e.z, e.depth_gt, R, S, cfg.raw_noise_std, None,
                   L.step_key(e.seed, 5), e.ray_offset, L.ctypes.byref(lp), e.d_enc, st.grad_mlp, e.ws, e.stats,
                   e.depth, e.opacity, None, e.level_max_ptr, e.d_jac, L.stream(dev))

        # the scan turns the histogram into offsets in place: each scatter restores the forward's counts
        nb = sum((int(st.desc.size[l]) + 4095) // 4096 for l in range(cfg.n_levels))
        nsb = (N + 511) // 512
        hist = e.bwd_ws[256:256 + 4 * nb * nsb]
        enc()
        snap = hist.clone()

        def scatter():
            hist.copy_(snap)
            e._grid_bwd(e.rays, R, S, N, L.BWD_COUNTS_READY | L.BWD_LEVEL_MAX_READY | L.BWD_NO_ACCUM, L.stream(dev))

        def accum():
            L.call("lnr_hashgrid_bwd_accum", L.ctypes.byref(st.desc), R * S, e.bwd_ws, e.bwd_ws_bytes, 0,
                   cfg.n_levels, st.grad_table, L.stream(dev))

        def sample():
            L.call("lnr_sample_ogm", e.rays, R, S, st.occ, cfg.occ_res, cfg.perturb, None, None, L.step_key(e.seed, 5),
                   e.ray_offset, e.z, None, L.stream(dev))

        def restore():
            hist.copy_(snap)

        return dict(sample=sample, enc=enc, enc0=enc0, field=field, scatter=scatter, accum=accum, restore=restore)

    A, B = stages(engs[0]), stages(engs[1])
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def timed(fn_pairs):
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        main = torch.cuda.current_stream(dev)
        t0.record(main)
        f = torch.cuda.Event()
        f.record(main)
        ends = []
        for s, fns in zip((s1, s2), fn_pairs):
            with torch.cuda.stream(s):
                s.wait_event(f)
                for _ in range(a.reps):
                    for fn in fns:
                        fn()
                ev = torch.cuda.Event()
                ev.record(s)
                ends.append(ev)
        for ev in ends:
            main.wait_event(ev)
        t1.record(main)
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / a.reps * 1e3

    # warm
    for k in A:
        timed(([A[k]], []))
    alone = {k: timed(([A[k]], [])) for k in A}
    print(f"{a.config} alone (us): " + ", ".join(f"{k} {v:.1f}" for k, v in alone.items()), flush=True)
    if os.environ.get("ALONE_ONLY"):
        return
    pairs = [("enc", "field"), ("enc", "scatter"), ("enc", "accum"), ("scatter", "field"), ("scatter", "accum"),
             ("accum", "field"), ("enc", "sample"), ("scatter", "sample")]
    for x, y in pairs:
        both = timed(([A[x]], [B[y]]))
        print(f"  {x:8s} || {y:8s}: {both:7.1f} us  (sum {alone[x] + alone[y]:7.1f}, max {max(alone[x], alone[y]):7.1f},"
              f" saved {alone[x] + alone[y] - both:6.1f})", flush=True)
    # half-batch chain: what a two-chunk split of the step would see (enc A -> field A || enc B)
    seq = timed(([A["enc"], A["field"]], []))
    print(f"  enc+field sequential: {seq:.1f} us", flush=True)


if __name__ == "__main__":
    main()
