#!/usr/bin/env python3
"""Benchmark: ray-samples/s per optimiser step of the LONER sigma-field path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu-baseline]

A "step" is one full optimiser step of the reference's step loop (src/mapping/optimizer.py:354-475)
on one ray batch: OGM sampling -> hash-grid encode -> sigma MLP -> compositing -> LiDAR loss ->
backward -> [all-reduce] -> Adam (+ the OGM update every N_iters_acc=10 global steps, which falls
inside the timed region as in the reference).  Default workload: BASELINE.json configs[1],
Newer College quad-easy: 16 keyframes x 512 rays = 8192 rays x 512 samples, L=16 hash grid +
64-wide MLP, synthetic analytic scene (no datasets reachable).  By default every step also selects
and builds its rays on the device from the keyframe window's scans, which are resident in HBM
before timing (optimizer.py:363-424; ``--rays resident`` instead cycles prebuilt ray batches).

Multi-GPU (torchrun): one process per GPU, each rank optimises its own 8192-ray shard of a global
batch of 8192*N rays (weak scaling) and the sigma gradients (7.4 M params, 29.7 MB fp32) plus the
loss normaliser are all-reduced over RCCL once per step.

Rank 0 prints one JSON line (contract in the task statement), including
  roofline      hash-grid backward stage (the dominant stage) against HBM peak, algorithmic bytes
                1024 B/sample, duration from HIP events on the launch stream
  mfma          the sigma MLP (12,672 FLOP/sample) over the field stage against the dense fp16 MFMA
                peak, plus the PMC MFMA-busy fraction of its kernels from profiles/*_mfma_<cfg>.json
  cpu_baseline  the pure-PyTorch CPU restatement (oracle/torch_step.py) on a bounded sample, host threads
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 TB/s measured copy)
MFMA_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA (MI355X_MICROARCH.md; sparsity figures excluded)
MLP_FLOP_PER_SAMPLE = 12672  # sigma MLP 32->64->1(16): fwd 2*(32*64 + 64*1) = 4224, bwd 2x
PROF_STEPS = 20  # untimed steps with per-stage HIP events, after the timed region (two OGM updates)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1).  Without a launcher "
                         "(WORLD_SIZE unset) and N > 1, bench.py starts the N rank processes itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C2", choices=["C1", "C2", "C3", "C4", "C5", "CAM"],
                    help="C1/C2/C4: optimiser step; C5: C4-shaped independent submap jobs, one per GPU "
                         "(replicas, no collectives); C3: inference render (peak depth, N_samples_test=2048); "
                         "CAM: colour-head training iteration (camera phase)")
    ap.add_argument("--rays", default="device", choices=["device", "resident"],
                    help="device: select + build each step's rays on the GPU from the resident window; "
                         "resident: cycle prebuilt ray batches")
    ap.add_argument("--batches", type=int, default=4, help="--rays resident: distinct batches cycled per rank")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="weak: each rank optimises the config's full batch (global batch grows with N); "
                         "strong: the config's batch is split over the N ranks (SURVEY.md §8(e)).  Default: "
                         "strong for C4 at N > 1 (the headline C4 curve at R = 9216), weak otherwise")
    ap.add_argument("--shard-of", type=int, default=None, metavar="N",
                    help="one GPU runs rank 0's shard of the config's batch split N ways (the per-rank step of an "
                         "N-GPU strong-scaling run, without the collective): the shard floor (C4, N in 2/4/8)")
    ap.add_argument("--field", default=None, choices=["init", "trained"],
                    help="init: time steps from the tcnn-like random init; trained (default with --rays device, "
                         "not C5): first time the from-init steps (kept under 'from_init'), then pre-train the field "
                         "untimed along the synthetic trajectory as the north-star driver does (shuffled windows of "
                         "the config's keyframe count, a new Adam per window, --pretrain-iters steps each, OGM on), "
                         "then time --steps on the bench window: the regime the driver spends its steps in")
    ap.add_argument("--pretrain-windows", type=int, default=12)
    ap.add_argument("--pretrain-iters", type=int, default=32,
                    help="steps per pre-training window (examples/fdt_optimize_implicit_map.py:76 NUM_ITERATIONS)")
    ap.add_argument("--field-cache", default=None, metavar="PATH",
                    help="--field trained: save the pre-trained field here, or load it if PATH exists and skip the "
                         "from-init steps and the pre-training (profiling runs: kernel statistics of the trained "
                         "window only)")
    ap.add_argument("--joint-poses", action="store_true",
                    help="the timed window optimises the keyframe poses with the map (the joint config of the "
                         "reference's default mapper schedule, cfg/defaults.yaml:93-97; keyframe 0 anchored)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=512, help="rays per reduced-config CPU-baseline step (x512 samples)")
    ap.add_argument("--cpu-steps", type=int, default=24)
    return ap.parse_args()


LOSS_PRESETS = {
    # cfg/model_config/default_model_config.yaml:40-60
    "default": dict(loss_selection="L1_JS", JS_loss=dict(min_js_score=1.0, max_js_score=10.0, alpha=1.0),
                    decay_los_lambda=False, los_lambda=1000.0, min_los_lambda=10.0, los_lambda_decay_rate=0.001,
                    los_lambda_decay_steps=15000, decay_depth_eps=True, depth_eps=3.0, min_depth_eps=0.5,
                    depth_eps_decay_rate=0.95, depth_eps_decay_steps=1, depthloss_lambda=0.005),
    # cfg/haveri_hpk/02_02_04.yaml:92-107
    "haveri": dict(loss_selection="L1_JS", JS_loss=dict(min_js_score=0.1, max_js_score=10.0, alpha=1.0),
                   decay_los_lambda=True, los_lambda=1000.0, min_los_lambda=10.0, los_lambda_decay_rate=0.0001,
                   los_lambda_decay_steps=15000, decay_depth_eps=True, depth_eps=3.0, min_depth_eps=0.5,
                   depth_eps_decay_rate=0.95, depth_eps_decay_steps=100, depthloss_lambda=0.005),
}


def pmc_traffic(cfg_name):
    """HBM bytes per launch of the hash-grid backward stage, from the newest committed PMC pass of
    this bench command (profiles/<round>_traffic_<cfg>.json, written by tools/refresh_profiles.py
    from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs); None if there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{cfg_name}.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    return rec["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def pmc_step_traffic(cfg_name):
    """HBM bytes per whole optimiser step (every kernel of the step; OGM kernels at their 1-in-10
    cadence), from profiles/<round>_traffic_<cfg>_step.json (tools/refresh_profiles.py, rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes over this bench command); None if there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{cfg_name}_step.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    return rec["hbm_bytes_per_step"], os.path.relpath(files[-1], ROOT)


def pmc_mfma(cfg_name):
    """Per sigma-MLP kernel MFMA busy fractions from the newest committed PMC pass of this bench
    command (profiles/<round>_mfma_<cfg>.json, tools/refresh_profiles.py); None if there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_mfma_{cfg_name}.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    return {k: v["mfma_busy_frac"] for k, v in rec["kernels"].items()}, os.path.relpath(files[-1], ROOT)


def pmc_kernel_traffic(cfg_name, kernel):
    """HBM bytes per optimiser step of one kernel (every launch of it in the step: early ray termination's encode
    phases together), from the newest committed per-step PMC pass (profiles/<round>_traffic_<cfg>_step.json);
    (None, None) if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_traffic_{cfg_name}_step.json")))
    if not files:
        return None, None
    rec = json.load(open(files[-1]))
    hits = [v for k, v in rec["kernels"].items() if kernel in k]
    if not hits:
        return None, None
    return sum(v["bytes_per_step"] for v in hits), os.path.relpath(files[-1], ROOT)


def pmc_ta_busy(cfg_name):
    """The encode's texture-addresser busy fraction (TA_BUSY_avr / GRBM_GUI_ACTIVE of k_hashgrid_fwd) from the
    newest committed profiles/<round>_ta_<cfg>.json (tools/pmc_l2req.sh + tools/refresh_profiles.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_ta_{cfg_name}.json")))
    if not files:
        return None, None
    return json.load(open(files[-1])).get("ta_busy_frac"), os.path.relpath(files[-1], ROOT)


def host_cpu_share():
    """(threads, why): the host threads this job may use.  The GPU pool sets OMP_NUM_THREADS to the job's
    CPU share (16 per GPU) while os.cpu_count() reports every core of the shared host, so the share
    caps the count; without it, the affinity mask."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        n = min(omp, n_aff)
        return n, (f"the job's CPU share: OMP_NUM_THREADS={omp} (os.cpu_count()={os.cpu_count()} counts the whole "
                   f"shared host, affinity {n_aff})")
    return n_aff, f"the affinity mask ({n_aff} of os.cpu_count()={os.cpu_count()})"


def _cpu_model():
    try:
        return next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        return "host CPU"


def _time_torch_steps(kind, strat, preset, n_rays, S, n_steps):
    """ray-samples/s and seconds of n_steps pure-PyTorch CPU steps (oracle/torch_step.py) of n_rays x S."""
    from oracle import torch_step as ts
    from loner_amd import synthetic as syn
    nkf = 1 if n_rays <= 512 else 2
    win = syn.make_window(kind, nkf, seed=99)
    rays, dgt = syn.build_batch(win, kind, n_rays // nkf, 0, strat, seed=7)
    field = ts.TorchField()
    scale = syn.CUBES[kind][0]
    ts.train_step(field, rays, dgt, scale, LOSS_PRESETS[preset], 1, S=S)  # warm-up (discarded)
    t0 = time.perf_counter()
    for it in range(n_steps):
        ts.train_step(field, rays, dgt, scale, LOSS_PRESETS[preset], 2 + it, S=S)
    dt = time.perf_counter() - t0
    return rays.shape[0] * S * n_steps / dt, dt, rays.shape[0]


def cpu_baseline(cfg_name, n_rays, n_steps):
    """The pure-PyTorch CPU restatement of the step (oracle/torch_step.py: forward + autograd backward +
    Adam) on BASELINE.md's two CPU shapes, on the host threads this job may use (rank 0, N=1 only;
    SURVEY.md §8(d)): C1 (1 keyframe x 512 rays x 64 samples) and a reduced C2 (512 rays x 512 samples)
    of this config's scene.  ``value`` is the reduced-C2 rate (the C1 rate on the C1 line)."""
    from loner_amd import synthetic as syn
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS[cfg_name]
    threads, why = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    c1_rate, c1_dt, _ = _time_torch_steps("quad", "RANDOM", "default", 512, 64, 20)
    rate, dt, r = _time_torch_steps(kind, strat, preset, n_rays, 512, n_steps)
    torch.set_num_threads(prev)
    cpu = _cpu_model()
    c1 = {"value": c1_rate, "unit": "ray-samples/s", "cores": threads,
          "sample": f"C1: 20 steps of 1 keyframe x 512 rays x 64 samples (quad), {c1_dt:.1f} s"}
    main = {"value": rate, "unit": "ray-samples/s", "cores": threads, "kind": "port", "cores_why": why,
            "cpu_model": cpu,
            "sample": f"reduced {cfg_name}: {n_steps} optimiser steps of {r} rays x 512 samples ({cfg_name} scene), "
                      f"pure-PyTorch CPU restatement (oracle/torch_step.py: forward + autograd backward + Adam), "
                      f"{threads} threads on {cpu}, {dt:.1f} s", "c1": c1}
    if cfg_name == "C1":
        main.update(value=c1_rate, sample=c1["sample"] + f", {threads} threads on {cpu}")
    return main


def rendered_depth_vs_oracle(state, window, n_rays, S, key_seed=21):
    """BASELINE.json's second metric, "rendered-depth L1 vs reference" (SURVEY.md §8(d)): the benched field,
    as trained by the timed steps, renders a strided n_rays subset of the bench batch through
    loner_amd.evaluate.DepthRenderer (HIP), and the CPU oracle (oracle/: the reference's sampler,
    compositing and tcnn-v1.7 restatement) renders the same rays on the GPU's samples.  Checker leg only
    (rank 0, N=1, after timing), as tests/test_gpu_depth_parity.py does.  Depths in metres.
      default   mean / max |depth - oracle| and the fraction of rays within 1 cm (bar: mean <= 1e-3 m,
                >= 99.9 % within 1 cm)
      adjusted  the fraction of rays whose peak depth differs, and the largest difference in sample
                positions (bar: <= 0.1 % of rays, by at most one sample spacing)"""
    from loner_amd import _lib as L
    from loner_amd import evaluate as E
    from oracle import hashgrid as ohg
    from oracle import mlp as omlp
    from oracle import render as orender
    from oracle import rng as orng
    t0 = time.perf_counter()
    R = window.n_slots
    rays = torch.empty(R, 13, dtype=torch.float32, device=state.device)
    dgt = torch.empty(R, dtype=torch.float32, device=state.device)
    key = L.step_key(key_seed, 0)
    window.build(key, 0, R, rays, dgt)
    stride = max(1, R // n_rays)
    rays = rays[::stride][:n_rays].contiguous()
    n = rays.shape[0]
    p16 = state.params[:state.n_params].cpu().numpy().astype(np.float16)
    nm = state.n_mlp
    w0, w1, table = p16[:2048].reshape(64, 32), p16[2048:nm].reshape(16, 64), p16[nm:].reshape(-1, 2)
    rn = rays.cpu().numpy()
    scale = float(window.scale)
    out = {"rays": n, "samples_per_ray": S, "subset": f"every {stride}th ray of the bench batch (step key {key_seed})"}
    for strategy in ("default", "adjusted"):
        rend = E.DepthRenderer(state, n_samples=S, chunk=n)
        depth, _, _ = rend.render(rays, key, strategy)
        d = depth.cpu().numpy()
        z = rend.z[:n].cpu().numpy()
        xyz = (rn[:, None, 0:3] + rn[:, None, 3:6] * z[:, :, None]).astype(np.float32)
        pos = ((xyz + np.float32(1)) / np.float32(2)).astype(np.float32).reshape(-1, 3)
        out16, _ = omlp.forward(ohg.encode(pos, table, ohg.GridLayout(16, 2, 18, 16)), [w0, w1])
        sig = out16[:, 0].astype(np.float32).reshape(n, S)
        if strategy == "adjusted":
            ref = orender.raw2outputs_adjusted(sig, z, rn[:, 3:6])["depth"]
            diff = np.flatnonzero(d != ref)
            steps = [abs(int(np.argmax(z[r] == d[r])) - int(np.argmax(z[r] == ref[r]))) for r in diff]
            out["adjusted"] = {"frac_rays_differ": float(len(diff) / n), "max_sample_steps": max(steps, default=0)}
        else:
            a, b = orng.ray_sample_grid(np.arange(n), S)
            ref = orender.raw2outputs(sig, z, rn[:, 3:6], orng.normal(key, orng.STREAM_NOISE, a, b), rn[:, -1:])["depth"]
            err = np.abs(d - ref).astype(np.float64) * scale
            out["depth_l1_vs_oracle_m"] = float(err.mean())
            out["default"] = {"mean_m": float(err.mean()), "max_m": float(err.max()),
                              "frac_within_1cm": float((err <= 1e-2).mean())}
    out["seconds"] = time.perf_counter() - t0
    return out


def cpu_baseline_render(kind, n_rays, S):
    """The same pure-PyTorch restatement's forward render (oracle/torch_step.render_step: OGM sampler,
    sigma field, peak compositing) on a bounded sample of the C3 workload, same threads as above."""
    from oracle import torch_step as ts
    from loner_amd import synthetic as syn
    threads, why = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    win = syn.make_window(kind, 1, seed=99)
    rays, _ = syn.build_batch(win, kind, n_rays, 0, "RANDOM", seed=7)
    field = ts.TorchField()
    ts.render_step(field, rays[:8], S)  # warm-up (discarded)
    t0 = time.perf_counter()
    ts.render_step(field, rays, S)
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    cpu = _cpu_model()
    return {"value": n_rays * S / dt, "unit": "ray-samples/s", "cores": threads, "kind": "port", "cores_why": why,
            "cpu_model": cpu,
            "sample": f"one render of {n_rays} rays x {S} samples (C3 scene), sigma head + peak depth, pure-PyTorch "
                      f"CPU restatement (oracle/torch_step.render_step), {threads} threads on {cpu}, {dt:.1f} s"}


def bench_render(args):
    """C3 (BASELINE.json configs[2]): inference rendering, Model.forward(testing=True) shape -- 4096 rays
    (one chunk, analysis/fdt_analysis_render_trajectory.py:40) x 2048 samples, peak ('adjusted')
    depth and the colour map (sigma head + colour head: SH4 + 2^19 HashGrid + 48->64x4->3 MLP).
    Roofline: the sigma-grid encode (the dominant kernel), 512 B/sample of gathers.  The colour grid is
    encoded only for samples of non-zero weight (lnr_hashgrid_fwd_rays_live: exact, since rgb adds
    w * colour)."""
    from loner_amd import evaluate as E
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd import _lib as L
    from loner_amd.rays import RayWindow
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    kind, nkf, rpk, spk, strat, S, preset = syn.CONFIGS["C3"]
    window = RayWindow(syn.make_window(kind, nkf, seed=1000), syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                       n_lidar=rpk, strategy=strat, device=dev)
    R = window.n_slots
    state = S_.FieldState(S_.StepConfig(n_samples=S), device=dev)
    color = E.ColorHead.init(4, device=dev)  # nerf_config intensity_network: 4 hidden layers of 64
    rend = E.DepthRenderer(state, n_samples=S, chunk=R, color=color)
    rgb = torch.empty(R, 3, dtype=torch.float32, device=dev)
    rays = torch.empty(R, 13, dtype=torch.float32, device=dev)
    dgt = torch.empty(R, dtype=torch.float32, device=dev)
    outs = [torch.empty(R, dtype=torch.float32, device=dev) for _ in range(3)]
    st = L.stream(dev)
    ev = {}

    def mark(k):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.setdefault(k, []).append(e)

    def run(i, prof):
        key = L.step_key(7, i)
        window.build(key, 0, R, rays, dgt)
        if prof:
            mark("sample")
        L.call("lnr_sample_ogm", rays, R, S, state.occ, 100, 0.0, None, None, key, 0, rend.z, None, st)
        if prof:
            mark("sample")
            mark("encode")
        L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(state.desc), rays, rend.z, R, S, state.table_f16, rend.enc,
               R * S, None, 0, st)
        if prof:
            mark("encode")
            mark("render")
        L.call("lnr_field_render", state.mlp_f16, rend.enc, R * S, rays, rend.z, R, S, 1, 1.0, None, key, 0, outs[0],
               outs[1], outs[2], rend.weights, st)
        if prof:
            mark("render")
            mark("encode_rgb")
        L.call("lnr_hashgrid_fwd_rays_live", L.ctypes.byref(color.desc), rays, rend.z, R, S, color.table,
               rend.weights, rend.enc_rgb, R * S, st)
        if prof:
            mark("encode_rgb")
            mark("rgb")
        L.call("lnr_rgb_render", color.mlp, 4, rend.enc_rgb, R * S, rays, rend.weights, R, S, rgb, st)
        if prof:
            mark("rgb")

    for i in range(args.warmup):
        run(i, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(args.warmup + i, False)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for i in range(PROF_STEPS):  # per-stage events, untimed
        run(args.warmup + args.steps + i, True)
    torch.cuda.synchronize()
    stage_ms = {k: float(np.mean([v[j].elapsed_time(v[j + 1]) for j in range(0, len(v), 2)])) for k, v in ev.items()}
    N = R * S
    # dominant kernel: the sigma-grid encode, 512 B/sample of gathers (the colour-grid encode skips
    # the samples of weight exactly 0, so its algorithmic bytes depend on the scene; not used here)
    enc_ms = stage_ms["encode"]
    achieved = 512.0 * N / (enc_ms * 1e-3) / 1e9
    line = {"metric": "ray-samples/sec per render (inference)", "value": N * args.steps / elapsed,
            "unit": "ray-samples/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp16 params/activations, fp32 compositing",
            "data": f"synthetic {kind} LiDAR scene, rays built on the GPU per render; random-init sigma field",
            "config": {"workload": f"C3: {R} rays x {S} samples, peak rendering, sigma head (L=16 T=2^18 + 64-wide "
                                   f"MLP) + colour head (SH4 + L=16 T=2^19 + 48->64x4->3 MLP)",
                       "rays": R, "samples_per_ray": S, "parallelism": "single"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "sigma hash-grid forward (k_hashgrid_fwd), 512 B/sample of gathers",
                         "algorithmic_bytes_per_launch": 512 * N, "ms_per_launch": enc_ms},
            "stage_ms": stage_ms}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_render(kind, 4096, S)
        line["cpu_baseline"]["rendered_depth_vs_oracle"] = rendered_depth_vs_oracle(state, window, 256, S)
    print(json.dumps(line), flush=True)


def cpu_baseline_camera(n_rays, S, steps):
    """The pure-PyTorch CPU restatement of one colour-head iteration (oracle/torch_step.camera_step: OGM
    sampler, frozen sigma field's weights, colour hash grid T=2^19 + SH4 + 48->64x4->3 MLP, L1 colour loss,
    autograd backward, Adam), as the C2/C3 baselines restate theirs, on a bounded sample (same host threads)."""
    from oracle import torch_step as ts
    from loner_amd import synthetic as syn
    threads, why = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    win = syn.make_window("forest", 1, seed=99)
    rays, _ = syn.build_batch(win, "forest", n_rays, 0, "RANDOM", seed=7)
    gt = torch.rand(rays.shape[0], 3, generator=torch.Generator().manual_seed(0))
    field, color = ts.TorchField(), ts.TorchColor()
    ts.camera_step(field, color, rays[:8], gt[:8], S)  # warm-up (discarded)
    t0 = time.perf_counter()
    for _ in range(steps):
        ts.camera_step(field, color, rays, gt, S)
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    cpu = _cpu_model()
    return {"value": rays.shape[0] * S * steps / dt, "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "cores_why": why, "cpu_model": cpu,
            "sample": f"{steps} colour-head iterations of {rays.shape[0]} rays x {S} samples, pure-PyTorch CPU "
                      f"restatement with both hash grids (oracle/torch_step.camera_step), {threads} threads on {cpu}, "
                      f"{dt:.1f} s"}


def bench_camera(args):
    """Camera phase (examples/fdt_optimize_implicit_map.py:826-873, optimizer.py:541-688): one colour
    head iteration on a MAX_WINDOW_LENGTH_CAMERA = 6 keyframe window x num_samples.lidar = 512 rays
    (the steady-state iterations; the first has 511) x N_samples_train = 512, 1280x720 images
    (640x360 x IMAGE_UPSAMPLING 2) resident in HBM.  Per iteration: camera rays on the GPU, OGM
    sampler, sigma encode + compositing weights (frozen, detached), colour encode, lnr_rgb_train,
    colour hash-grid backward, Adam over the colour parameters."""
    from loner_amd import camera as C
    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    from loner_amd import _lib as L
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n_kf, per_kf, S, W, H = 6, 512, 512, 1280, 720
    kind = "forest"
    K = np.array([[640.0, 0, (W - 1) / 2], [0, 640.0, (H - 1) / 2], [0, 0, 1]])
    dirs = C.pinhole_directions(W, H, K)
    lidar_to_cam = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], dtype=np.float64)  # camera z = lidar x
    poses, imgs = [], []
    yy, xx = np.mgrid[0:H, 0:W]
    for k, P in enumerate(syn.keyframe_poses(kind, n_kf, np.random.default_rng(0))):
        Pc = np.array(P, dtype=np.float64)
        Pc[:3, :3] = Pc[:3, :3] @ lidar_to_cam
        poses.append(Pc[:3])
        imgs.append(np.stack([0.5 + 0.4 * np.sin(xx / 37.0 + k), 0.5 + 0.4 * np.cos(yy / 23.0),
                              0.3 + 0.2 * np.sin((xx + yy) / 50.0)], -1).reshape(-1, 3).astype(np.float32))
    fr = C.CameraFrames(dirs, W, H, imgs, poses, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"],
                        n_rays_per_kf=per_kf, seed=0, device=dev)
    # the sigma field (frozen during the camera phase) in the LiDAR phase's configuration of this scene (C4's)
    _, nkf4, rpk4, spk4, strat4, S4, preset4 = syn.CONFIGS["C4"]
    state = S_.FieldState(S_.StepConfig(n_samples=S, occ_lr=1e-3 if preset4 == "haveri" else 1e-4,
                                        loss=S_.LossConfig.from_dict(LOSS_PRESETS[preset4])), device=dev)
    color = C.ColorState(4, device=dev)
    R = n_kf * per_kf
    eng = C.CameraStepEngine(state, color, n_rays=R, n_samples=S, seed=0)
    rays = torch.empty(R, 13, dtype=torch.float32, device=dev)
    inten = torch.empty(R, 3, dtype=torch.float32, device=dev)
    ev = {}

    def mark(k):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.setdefault(k, []).append(e)

    def run(i, prof):
        it = 1 + i % (fr.n_iter - 1)  # steady-state iterations: 512 rays per keyframe
        if prof:
            mark("iteration")
        n = fr.build(it, rays, inten)
        eng.step(rays[:n], inten[:n])
        if prof:
            mark("iteration")
        return n

    def measure():
        for i in range(args.warmup):
            run(i, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_tot = 0
        for i in range(args.steps):
            n_tot += run(args.warmup + i, False)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        for i in range(PROF_STEPS):  # whole-iteration events, untimed
            run(args.warmup + args.steps + i, True)
        # one extra profiled iteration split by stage (events between the engine's launches)
        stage = _camera_stages(eng, fr, rays, inten, L)
        live = float((eng.weights[:R * S] != 0).float().mean())
        return elapsed, n_tot, stage, live

    field = args.field or "trained"
    from_init, pre = None, None
    if field == "trained":
        # the driver's camera phase runs on a sigma field its LiDAR phase has trained: most samples have weight 0
        # there (free space, and everything behind the surface), which the colour kernels skip (zero-weight tiles,
        # the live colour encode).  Timed first from init, then after the LiDAR phase's windows (bench.pretrain over
        # the scene's trajectory, C4's shape), with a fresh colour head for the timed iterations.
        elapsed, n_tot, stage_i, live_i = measure()
        from_init = {"ms_per_step": elapsed / args.steps * 1e3, "value": n_tot * S / elapsed, "stage_ms": stage_i,
                     "live_sample_frac": live_i}
        R4 = nkf4 * (rpk4 + spk4)
        leng = S_.StepEngine(state, R4, seed=12345)
        t_pre = time.perf_counter()
        _, pre = pretrain(leng, state, kind, nkf4, rpk4, spk4, strat4, dev, R4, 1, args.pretrain_windows,
                          args.pretrain_iters)
        pre["seconds"] = time.perf_counter() - t_pre
        leng.release()
        del leng
        color = C.ColorState(4, device=dev)  # a fresh colour head (and its engine) for the timed iterations
        eng = C.CameraStepEngine(state, color, n_rays=R, n_samples=S, seed=0)
        torch.cuda.synchronize()
    elapsed, n_tot, stage_ms, live_frac = measure()
    N = n_tot * S
    bwd_ms = stage_ms["rgb_train"]
    flop = 2 * 3 * (64 * 48 + 3 * 64 * 64 + 16 * 64) * R * S  # forward (x2: recomputed) + backward GEMMs
    achieved = flop / (bwd_ms * 1e-3) / 1e12
    line = {"metric": "ray-samples/sec per colour-head iteration", "value": N / elapsed, "unit": "ray-samples/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp16 params/activations, fp32 accumulate+optimizer",
            "data": "synthetic 1280x720 images resident in HBM, camera rays built on the GPU each iteration; "
                    + ("sigma field (frozen) pre-trained untimed by the LiDAR phase's windows (config.field_state)"
                       if field == "trained" else "random-init sigma field (frozen)") + ", random-init colour head",
            "config": {"workload": f"CAM: {n_kf} KF x {per_kf} camera rays x {S} samples, colour head SH4 + L=16 "
                                   f"T=2^19 + 48->64x4->3 MLP, L1 loss, Adam",
                       "rays": R, "samples_per_ray": S, "parallelism": "single",
                       "field_state": ("trained: the sigma field after %d untimed LiDAR steps (config.pretrain)"
                                       % pre["steps"] if field == "trained" else "from init"),
                       **({"pretrain": pre} if pre is not None else {})},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / MFMA_PEAK_TFLOPS, "traffic": None,
                         "kernel": "lnr_rgb_train (colour forward x2 + L1 + MLP backward, MFMA fp16)",
                         "algorithmic_flop_per_launch": flop, "ms_per_launch": bwd_ms},
            "stage_ms": stage_ms,
            # the share of ray-samples with a non-zero compositing weight (the colour kernels' live samples)
            "live_sample_frac": live_frac,
            **({"from_init": from_init} if from_init is not None else {})}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_camera(96, S, 4)
    print(json.dumps(line), flush=True)


def _camera_stages(eng, fr, rays, inten, L):
    """Per-stage HIP-event times of one camera iteration (same launches as CameraStepEngine.step)."""
    fs, cs = eng.field, eng.color
    s = L.stream(fs.device)
    ev = []

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append((name, e))

    R, S, N = eng.R, eng.S, eng.N
    key = L.step_key(0, 12345)
    mark("rays")
    fr.build(1, rays, inten)
    mark("sample")
    L.call("lnr_sample_ogm", rays, R, S, fs.occ, fs.cfg.occ_res, 1.0, None, None, key, 0, eng.z, None, s)
    mark("encode")
    L.call("lnr_hashgrid_fwd_rays", L.ctypes.byref(fs.desc), rays, eng.z, R, S, fs.table_f16, eng.enc, N, None, 0, s)
    mark("weights")
    L.call("lnr_field_render", fs.mlp_f16, eng.enc, N, rays, eng.z, R, S, 0, 1.0, None, key, 0, eng.depth,
           eng.opacity, None, eng.weights, s)
    mark("encode_rgb")
    eng.colour_encode(rays, R, S, s)
    mark("rgb_train")
    L.call("lnr_rgb_train", cs.mlp_f16, cs.n_hidden_layers, eng.enc_rgb, N, rays, eng.weights, inten, R, S,
           1.0 / (3.0 * R), eng.rgb, eng.loss, eng.d_enc, cs.grad_mlp, eng.ws, eng.ws_bytes, eng.level_max_ptr, s)
    mark("grid_bwd")
    eng.colour_grid_backward(rays, R, S, s)
    mark("adam")
    L.call("lnr_adam_step", cs.params, cs.shadow, cs.grad, cs.m, cs.v, cs.n_padded, 1, 0.0, 0.9, 0.999, 1e-8, None, s)
    mark("end")
    torch.cuda.synchronize()
    return {ev[i][0]: float(ev[i][1].elapsed_time(ev[i + 1][1])) for i in range(len(ev) - 1)}


def pretrain(eng, state, kind, n_kf, rpk, spk, strat, dev, r_glob, g_start, n_windows, iters, pool_size=48):
    """Untimed pre-training of the benched field in the north-star driver's regime
    (examples/fdt_optimize_implicit_map.py:576-616): the trajectory's keyframes are shuffled once per
    repetition and cut into windows of ``n_kf`` (MAX_WINDOW_LENGTH_LIDAR = 16 at C2); each window is a new
    Adam (optimizer.py:255-265) run for ``iters`` (NUM_ITERATIONS = 32) steps through the same engine, rays
    selected and built on the GPU, the OGM updated every N_iters_acc global steps.  The keyframe pool is
    ``pool_size`` poses of the config's synthetic trajectory (the quad loop's 48 poses include every pose
    of the bench window).  Returns (the next global step, a description for the bench line)."""
    from loner_amd import synthetic as syn
    from loner_amd.rays import RayWindow
    pool = syn.make_window(kind, pool_size, seed=2000)
    rng = np.random.default_rng(5)
    order, g = [], g_start
    for _ in range(n_windows):
        while len(order) < n_kf:
            order += list(rng.permutation(pool_size))
        idx, order = order[:n_kf], order[n_kf:]
        win = RayWindow([pool[i] for i in idx], syn.world_cube(kind), syn.SENSORS[kind]["ray_range"], n_lidar=rpk,
                        n_sky=spk, strategy=strat, device=dev)
        state.reset_optimizer()
        for it in range(iters):
            eng.step_window(win, global_step=g, iteration_idx=it, n_rays_global=r_glob)
            g += 1
        eng.release()
        del win
    torch.cuda.synchronize()
    return g, {"windows": n_windows, "iterations_per_window": iters, "steps": n_windows * iters,
               "keyframes_per_window": n_kf, "pool": f"{pool_size} poses of the synthetic {kind} trajectory, shuffled "
                                                    "per repetition (the driver's SCHUFFLE)",
               "adam": "new per window", "ogm": "updated every N_iters_acc = 10 global steps",
               "global_step_after": g}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """``--gpus N`` without a launcher: start N rank processes of this same command (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT set as torch.distributed.run sets them), one per GPU,
    and wait.  This process never touches the GPU (it only counts devices, which does not initialise
    HIP).  Any rank failing ends the others and the exit status is that rank's; rank 0 prints the line."""
    import signal
    import subprocess
    backend = os.environ.get("LONER_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if backend == "nccl" and n_dev < n:
        raise SystemExit(f"bench.py --gpus {n}: only {n_dev} GPU(s) visible (one rank per GPU over RCCL; "
                         f"LONER_DIST_BACKEND=gloo shares GPUs between ranks)")
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:  # a failed rank would leave the others blocked in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    if rc:
        print(f"bench.py: a rank exited with status {rc}", file=sys.stderr)
    sys.exit(rc)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        return spawn_ranks(args.gpus)
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.config in ("C3", "CAM"):
        if world > 1:
            raise SystemExit(f"bench.py --config {args.config} is a single-GPU bench (no sharded path)")
        return bench_render(args) if args.config == "C3" else bench_camera(args)
    if args.scaling is None:
        args.scaling = "strong" if args.config == "C4" and world > 1 else "weak"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LONER_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin); the driver's N-GPU runs use RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("LONER_DIST_BACKEND", "nccl")
    gpu = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu)

    from loner_amd import step as S_
    from loner_amd import synthetic as syn
    kind, nkf, rpk, spk, strat, n_samples, preset = syn.CONFIGS[args.config]
    scale = syn.CUBES[kind][0]
    replicas = args.config == "C5"  # independent jobs: own window per rank, no data-path collective

    # ---- workload
    submap = None
    if args.rays == "device" and replicas:
        # rank r optimises submap r (mod the part count) of the segmented trajectory, in its own cube
        from loner_amd.rays import RayWindow
        scans, cube, submap = syn.submap_window(rank, nkf, seed=1000 + rank)
        window = RayWindow(scans, cube, syn.SENSORS[kind]["ray_range"], n_lidar=rpk, n_sky=spk, strategy=strat,
                           device=dev)
        win_kf = len(scans)
        del scans
        if not window.all_valid:
            raise RuntimeError("bench window must give a fixed batch")
        R = window.n_slots
    elif args.rays == "device" and args.shard_of:
        # rank 0's slice of the config's batch split --shard-of ways: the strong-scaling per-rank step
        from loner_amd.rays import RayWindow
        if world != 1:
            raise SystemExit("--shard-of runs one rank's shard on one GPU (world size 1)")
        scans = syn.make_window(kind, nkf, seed=1000)
        window = RayWindow(scans, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"], n_lidar=rpk, n_sky=spk,
                           strategy=strat, device=dev)
        win_kf = len(scans)
        del scans
        if not window.all_valid or window.n_slots % args.shard_of:
            raise RuntimeError("bench window must give a fixed, evenly sharded batch")
        R = window.n_slots // args.shard_of
    elif args.rays == "device":
        # one global keyframe window (nkf keyframes per rank), resident on every rank; rank r builds
        # the slots of its own nkf keyframes each step (a contiguous R/g slice)
        from loner_amd.rays import RayWindow
        scans = syn.make_window(kind, nkf if args.scaling == "strong" else nkf * world, seed=1000)
        window = RayWindow(scans, syn.world_cube(kind), syn.SENSORS[kind]["ray_range"], n_lidar=rpk, n_sky=spk,
                           strategy=strat, device=dev)
        win_kf = len(scans)
        del scans
        if not window.all_valid or window.n_slots % world:
            raise RuntimeError("bench window must give a fixed, evenly sharded batch")
        R = window.n_slots // world
    else:
        if args.scaling == "strong":
            raise SystemExit("--scaling strong needs --rays device")
        batches = []
        for b in range(args.batches):
            win = syn.make_window(kind, nkf, seed=1000 * rank + b, start=17 * b + 5 * rank)
            rays, dgt = syn.build_batch(win, kind, rpk, spk, strat, seed=31 * b + rank)
            batches.append((rays.to(dev), dgt.to(dev)))
        R = batches[0][0].shape[0]
        assert all(b[0].shape[0] == R for b in batches)
        far_ref = [float(b[0][0, -1]) for b in batches]

    cfg = S_.StepConfig(n_samples=n_samples, occ_lr=1e-3 if preset == "haveri" else 1e-4,
                        loss=S_.LossConfig.from_dict(LOSS_PRESETS[preset]))
    state = S_.FieldState(cfg, device=dev)
    allreduce = None
    zero, hooks = None, {}
    # the sharded optimiser (ZeRO-1: reduce-scatter, Adam on 1/N of the parameters, all-gather of the fp16
    # shadow) for the data-parallel step; LONER_ZERO=0 keeps the all-reduce + replicated Adam
    use_zero = os.environ.get("LONER_ZERO", "1") != "0"
    if dist is not None and not replicas:
        def allreduce(t, async_op=False):
            return dist.all_reduce(t, async_op=async_op)
        if use_zero and world in (2, 4, 8):
            zero = (rank, world)
            # LONER_EXCHANGE_GROUPS=2 (default): the shadow all-gathers on a process group of their own, i.e. a
            # second communicator, so range r's gather runs beside range r + 1's reduce-scatter instead of after it
            # in one communicator's queue (tools/zero_tail_model.py); 1: one group
            ag_group = dist.new_group(list(range(world))) if os.environ.get("LONER_EXCHANGE_GROUPS", "2") == "2" else None
            hooks = dict(reduce_scatter=lambda o, i, async_op=False: dist.reduce_scatter_tensor(o, i, async_op=async_op),
                         all_gather=lambda o, i, async_op=False: dist.all_gather_into_tensor(o, i, group=ag_group,
                                                                                            async_op=async_op),
                         two_groups=ag_group is not None)
    elif args.shard_of and use_zero:
        zero = (0, args.shard_of)  # one rank's share of the sharded Adam, no exchange (world size 1)
    eng = S_.StepEngine(state, R, seed=12345 + (rank if replicas else 0), allreduce=allreduce,
                        ray_offset=0 if replicas else rank * R, zero=zero,
                        ar_cut=S_.AR_CUT_TWO_GROUPS if hooks.get("two_groups") else None,
                        **{k: v for k, v in hooks.items() if k != "two_groups"})
    r_glob = R if replicas else R * world
    if args.shard_of:
        r_glob = R * args.shard_of

    if args.field is None:
        args.field = "trained" if args.rays == "device" and not replicas else "init"
    if args.field == "trained" and (args.rays != "device" or replicas):
        raise SystemExit("--field trained needs --rays device and a sharded/single config (not C5)")

    def run(i, prof=None, g0=0):
        # g0: the global step the timed window starts at; the iteration index within the window drives the
        # depth-eps decay as in the driver's windows (optimizer.py:781-785)
        if args.rays == "device":
            return eng.step_window(window, global_step=g0 + i, iteration_idx=i if g0 else 0, n_rays_global=r_glob,
                                   prof=prof)
        rays, dgt = batches[i % len(batches)]
        return eng.step(rays, dgt, global_step=i, scale=scale, far_ref=far_ref[i % len(batches)],
                        n_rays_global=r_glob, prof=prof)

    def measure(g0=0):
        """W untimed warm-up steps, then K timed steps (barrier + synchronize on both sides, the max over ranks),
        then PROF_STEPS untimed steps with per-stage HIP events; returns (seconds, loss, stage ms, the fraction
        of ray-samples whose dL/dsigma is exactly 0 in the profiled steps)."""
        for i in range(args.warmup):
            run(i, g0=g0)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.warmup, args.warmup + args.steps):
            out = run(i, g0=g0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if dist is not None:
            dist.barrier()
        elapsed = t1 - t0
        if dist is not None:
            e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        loss = out.cpu().numpy()
        # per-stage HIP events in a separate pass after the timed region (recording them costs host time:
        # 47 us per step at C1, where the host issues the step faster than the GPU runs it only without them)
        prof = {}
        zeros = torch.zeros(2, dtype=torch.float64, device=dev)
        nw = R * n_samples // 64
        th0 = eng.term_hist.clone() if eng.term_hist is not None else None
        for i in range(args.warmup + args.steps, args.warmup + args.steps + PROF_STEPS):
            run(i, prof, g0=g0)
            ds = eng.d_sigma(R)  # (after the step's events: outside every stage)
            zeros[0] += (ds == 0).sum()
            zeros[1] += (ds[:64 * nw].view(nw, 64) != 0).any(1).logical_not().sum()  # dead 64-sample waves
        torch.cuda.synchronize()
        stage = {k: float(np.mean([v[j].elapsed_time(v[j + 1]) for j in range(0, len(v), 2)])) for k, v in prof.items()}
        ert = {"phases": eng.ert_bounds(), "mode": eng.ert}
        if ert["phases"] is not None and "sigma_phase" in stage:
            # early ray termination: the encode stage holds the phases' encode and sigma launches; the sigma ones
            # are timed on their own (one pair per phase), the rest is the encode kernels'
            stage["sigma_phases"] = stage.pop("sigma_phase") * (len(ert["phases"]) - 1)
        if th0 is not None:
            d = (eng.term_hist.long().sum(0) - th0.long().sum(0)).cpu().numpy()
            alive = S_.ert_alive(d, n_samples)
            ert["alive_after"] = {int(64 * k): round(float(alive[k]), 4) for k in range(1, n_samples // 64)}
            b = ert["phases"] or [0, n_samples]
            # the share of ray-samples the encode gathered (the rays still alive at each phase's start)
            ert["encoded_frac"] = float(sum(alive[lo // 64] * (hi - lo) for lo, hi in zip(b[:-1], b[1:])) / n_samples)
        z = zeros.cpu().numpy()
        return elapsed, loss, stage, (float(z[0]) / (PROF_STEPS * R * n_samples), float(z[1]) / (PROF_STEPS * max(nw, 1)),
                                      ert)

    poses_desc = "fixed (ground-truth poses, use_gt_poses: the north-star driver)"

    def arm_poses(n_iter):
        """--joint-poses: the keyframes' pose tensors (keyframe 0 anchored) in an Adam at lrate_pose 1e-3."""
        nonlocal poses_desc
        if not args.joint_poses:
            return
        from loner_amd.pose import PoseWindow
        pw = PoseWindow(window, [k > 0 for k in range(window.n_kf)], 1e-3, allreduce=allreduce, n_iter=n_iter)
        eng.set_poses(pw)
        poses_desc = (f"joint pose + map: {window.n_kf - 1} keyframe poses in an Adam at 1e-3 beside the map "
                      f"(keyframe 0 anchored; optimizer.py:258-262)"
                      + ("" if pw.stay_valid else ", rays filtered every step (window near the cube's faces)"))

    cache = args.field_cache if args.field == "trained" else None
    from_init = None
    if args.field != "trained":
        arm_poses(args.warmup + args.steps + PROF_STEPS)
    if cache and os.path.exists(cache):
        # a profiling run: the pre-trained field of an earlier run (no from-init steps, no pre-training here, so
        # the kernel statistics hold the trained window's steps only)
        ck = torch.load(cache, map_location=dev, weights_only=True)
        state.params.copy_(ck["params"])
        state.occ.copy_(ck["occ"])
        state.refresh_shadow()
        g0, pre = int(ck["g0"]), dict(json.loads(ck["pre"]), loaded_from=cache)
    else:
        elapsed, loss, stage_ms, zero_frac = measure()
    if args.field == "trained":
        if not (cache and os.path.exists(cache)):
            from_init = {"ms_per_step": elapsed / args.steps * 1e3,
                         "value": world * R * n_samples * args.steps / elapsed,
                         "loss": float(loss[0]), "dsigma_zero_frac": zero_frac[0], "dead_wave_frac": zero_frac[1],
                         "ert": zero_frac[2],
                         "backward": "live" if eng._live else "full", "stage_ms": stage_ms}
            t_pre = time.perf_counter()
            g0, pre = pretrain(eng, state, kind, win_kf, rpk, spk, strat, dev, r_glob,
                               args.warmup + args.steps + PROF_STEPS, args.pretrain_windows, args.pretrain_iters)
            pre["seconds"] = time.perf_counter() - t_pre
            if cache and rank == 0:
                torch.save({"params": state.params.cpu(), "occ": state.occ.cpu(), "g0": g0, "pre": json.dumps(pre)},
                           cache)
        state.reset_optimizer()  # the timed window: a new Adam (optimizer.py:255-265)
        arm_poses(args.warmup + args.steps + PROF_STEPS)
        elapsed, loss, stage_ms, zero_frac = measure(g0)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    N = R * n_samples
    ms = elapsed / args.steps * 1e3
    value = world * N * args.steps / elapsed
    bwd_ms = stage_ms["grid_bwd"]
    # one GPU: the table's Adam runs inside the backward's accumulation (lnr_hashgrid_bwd_rays_jac_adam),
    # so the stage's algorithmic bytes add Adam's 32 B per table parameter
    fused_adam = eng.fuses_adam(N)
    # algorithmic work counts the samples that have it: every sample is encoded and goes through the MLP forward
    # (its sigma decides whether it is dead), but a sample with dL/dsigma = 0 has no scatter-adds and no MLP
    # backward to do (its contributions are exactly 0; the reference's tcnn path does them all the same)
    zero_frac, dead_wave_frac, ert = zero_frac
    n_live = N * (1.0 - zero_frac)
    bwd_bytes = 1024.0 * n_live + (32.0 * 2 * state.n_entries if fused_adam else 0.0)
    achieved = bwd_bytes / (bwd_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.config)
    traffic_step, traffic_step_src = pmc_step_traffic(args.config)
    enc_traffic, enc_traffic_src = pmc_kernel_traffic(args.config, "k_hashgrid_fwd")
    # the whole step against the HBM bound: 512 B per ray-sample of gathers, 1024 B per live
    # ray-sample of scatter-adds, 32 B per parameter (Adam), 52 B per ray
    n_enc = N * ert.get("encoded_frac", 1.0) if ert["phases"] is not None else N
    step_bytes = 512.0 * n_enc + 1024.0 * n_live + 32.0 * state.n_params + 52.0 * R
    busy, busy_src = pmc_mfma(args.config)
    # (with early ray termination the forward runs in the sigma phases, over the encoded samples)
    mlp_flop = 4224.0 * n_enc + 8448.0 * n_live
    mlp_ms = stage_ms["field"] + stage_ms.get("sigma_phases", 0.0)
    mlp_tflops = mlp_flop / (mlp_ms * 1e-3) / 1e12
    # the encode launches' time: with early ray termination the stage also holds the sigma phases (timed apart);
    # the algorithmic gathers are those of the samples encoded (512 B each), as the backward counts live samples
    enc_ms = stage_ms["encode"] - stage_ms.get("sigma_phases", 0.0)
    enc_achieved = 512.0 * n_enc / (enc_ms * 1e-3) / 1e9
    ta, ta_src = pmc_ta_busy(args.config)
    line = {
        # BASELINE.json metric: the rate here, the rendered-depth L1 in cpu_baseline.rendered_depth_vs_oracle
        "metric": "ray-samples/sec per optimizer step; rendered-depth L1 vs reference",
        "value": value,
        "unit": "ray-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong" if args.scaling == "strong" and not replicas else "weak",
        "vs_baseline": None,
        "dtype": "fp16 params/activations, fp32 accumulate+optimizer",
        "data": f"synthetic {kind} LiDAR scene (analytic ray-cast), "
                + ("keyframe scans resident in HBM, rays selected + built on the GPU every step"
                   if args.rays == "device" else "prebuilt rays resident in HBM")
                + ("; sigma field pre-trained untimed along the synthetic trajectory (config.field_state)"
                   if args.field == "trained" else "; random-init sigma field"),
        "config": {"workload": f"{args.config}: {nkf} KF x ({rpk} + {spk} sky) rays x {n_samples} samples "
                               + ("in total, split over the GPUs, " if args.scaling == "strong" else "per GPU, ")
                               + f"L=16 T=2^18 hash grid + 64-wide sigma MLP, {preset} loss (L1_JS)",
                   "rays_per_gpu": R, "samples_per_ray": n_samples, "global_rays": R * world,
                   "parallelism": (f"replicas{world}" if replicas else f"dp{world}") if world > 1 else
                   (f"shard 0 of {args.shard_of} (one rank's strong-scaling step: its rays, its 1/{args.shard_of} "
                    f"of the sharded Adam; no collective)" if args.shard_of else "single"),
                   "optimizer": ("sharded (ZeRO-1)" + (", all-gathers on a second communicator" if world > 1 and
                                 os.environ.get("LONER_EXCHANGE_GROUPS", "2") == "2" else "")
                                 if zero is not None else "replicated"),
                   "launch": ("HIP graph replay (one graph per window and OGM-or-not step)"
                              if eng.use_graph and args.rays == "device" and eng.allreduce is None else
                              "eager, next step's ray build + sampling prefetched on a side stream"),
                   "field_state": ("trained: the steps below follow %d untimed pre-training steps (config.pretrain)"
                                   % pre["steps"] if args.field == "trained" else
                                   "from init: tcnn-like U(+-1e-4) table, Xavier MLP, steps %d-%d after it"
                                   % (args.warmup, args.warmup + args.steps - 1)),
                   "poses": poses_desc,
                   **({"pretrain": pre} if args.field == "trained" else {}),
                   **({"submap_rank0": submap} if submap is not None else {})},
        # the dominant kernel, the training encode (k_hashgrid_fwd: 8 gathers per sample and level, 512 B per
        # ray-sample algorithmic; the longest kernel of the step from init and trained), against HBM peak; what
        # bounds it is the texture addresser, not bytes ("What bounds the forward encode")
        "roofline": {"bound": "hbm", "achieved": enc_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": enc_achieved / HBM_PEAK_GBS, "traffic": enc_traffic, "traffic_source": enc_traffic_src,
                     "kernel": "k_hashgrid_fwd (training encode: every launch of the step, i.e. early ray termination's "
                               "phases, + the full backward's record histogram when that backward runs)",
                     "algorithmic_bytes_per_launch": 512 * n_enc, "ms_per_launch": enc_ms,
                     "encoded_samples_per_launch": n_enc,
                     "limiter": "texture addresser: TA busy %s of the launch (%s)" % (
                         "n/a" if ta is None else "%.2f" % ta, ta_src or "no committed PMC pass"),
                     "step_algorithmic_bytes": step_bytes,
                     "step_frac": step_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic_step": traffic_step, "traffic_step_source": traffic_step_src},
        # the hash-grid backward stage (the scatter-adds: 1024 B per live ray-sample)
        "backward_stage": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                           "kernel": "hash-grid backward stage (" + (
                               "live: k_bwd_col_totals, k_bwd_count_live, " if eng._live else "") +
                               "k_bwd_chunk_sums, k_bwd_scan_*, k_bwd_scatter_rows, " + (
                               "k_bwd_accum_buckets)" if N <= (1 << 17) else
                               "k_bwd_accum_units: whole buckets and pieces of the large ones)" if N <= (1 << 21) else
                               "k_bwd_accum: record-balanced, k_bwd_finalize)") + (
                               "; the table's Adam fused into the accumulation" if fused_adam else ""),
                           "backward": "live (records for samples with dL/dsigma != 0 only)" if eng._live else "full",
                           "algorithmic_bytes_per_launch": bwd_bytes, "live_samples_per_launch": n_live,
                           "ms_per_launch": bwd_ms},
        # the sigma MLP (fwd 4224 + bwd 8448 FLOP/sample) over the field stage
        # (k_sigma_fwd_tiles + k_composite_wave + k_mlp_bwd_tiles), against the dense fp16 MFMA peak
        "mfma": {"achieved": mlp_tflops, "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": mlp_tflops / MFMA_PEAK_TFLOPS,
                 "flop_per_sample": MLP_FLOP_PER_SAMPLE, "flop_per_launch": mlp_flop,
                 "flop_note": "forward 4224 per encoded ray-sample, backward 8448 per live ray-sample",
                 "ms_per_launch": mlp_ms,
                 "busy": busy, "busy_source": busy_src},
        "stage_ms": stage_ms,
        "loss": float(loss[0]),
        # the fraction of ray-samples whose dL/dsigma is exactly 0 (alpha = 1 - exp(-delta relu(sigma + n)) with
        # sigma + n <= 0, rendering_tcnn.py:252,260) over the profiled steps: they contribute exactly nothing
        "dsigma_zero_frac": zero_frac,
        # the fraction of 64-sample waves without a live sample: the live backward's work skips by wave, and it
        # runs (LONER_LIVE_BWD=auto) while this share exceeds StepEngine.live_on (backward_stage.backward)
        "dead_wave_frac": dead_wave_frac,
        # early ray termination over the profiled steps: the phases in use (None: off), the share of rays still alive
        # after each 64-sample boundary (the compositing's termination counts), the share of ray-samples encoded
        "ert": ert,
        # the same bench on the from-init field, timed first in this run (--field trained only)
        **({"from_init": from_init} if from_init is not None else {}),
        # the process group as torch.distributed reports it (None: a single process, no group)
        "dist": ({"backend": dist.get_backend(), "ranks": dist.get_world_size()} if dist is not None else None),
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_rays, args.cpu_steps)
        if args.rays == "device":
            line["cpu_baseline"]["rendered_depth_vs_oracle"] = rendered_depth_vs_oracle(state, window, 512, n_samples)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
